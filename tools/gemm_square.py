"""Large plain bf16 GEMMs on the 256x256 phased kernel vs hipBLASLt (torch.matmul), uniform
random [-1, 1) operands (the guide's reference condition for the 256^2 template)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    from fastspeech2 import ops, _native
    _native.load()
    shapes = ((8192, 8192, 8192), (4096, 4096, 4096), (31264, 1536, 3456), (31264, 3456, 1536))
    only = os.environ.get("GS_ONLY")   # comma-separated shape indices
    if only:
        shapes = [shapes[int(i)] for i in only.split(",")]
    for M, N, K in shapes:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        u1 = t(lambda: ops.gemm(M, N, K, A, K, W, K, C, N, dt=1))
        u2 = t(lambda: torch.matmul(A, W.t()))
        print(f"{M}x{N}x{K}: ours {u1:8.1f} us {fl / u1 / 1e6:7.1f} TF/s | hipBLASLt {u2:8.1f} us "
              f"{fl / u2 / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
