"""The FFN conv2 data-gradient shape (M x 1536 = M x 384 . 384 x 1536, bf16 out, ReLU gate from
the forward's Hc) and its conv2-forward mirror (M x 384 = M x 1536 . 1536 x 384) at the decoder
(M = 31264) and encoder (M = 6400) sizes, plain and with the gate; with the experiments library
the FS2_GEMM_NO_PK / FS2_PK_FLAGS switches pick the kernel / timing-only variants.  us per call."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FS2_HIP_LIB", os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd",
                                                  "fastspeech2", "libfs2_hip_exp.so"))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402
from fastspeech2 import ops  # noqa: E402


def timeit(fn, n=20):
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
    bf = torch.bfloat16
    torch.manual_seed(0)
    D, F = 384, 1536
    for M in (31264, 6400):
        dY = torch.randn(M, D, device="cuda").to(bf)
        W = (torch.randn(D, F, device="cuda") * 0.05).to(bf)     # [K=D][N=F] -> K-major B: [F][D]
        Wt = W.t().contiguous()
        Hc = torch.relu(torch.randn(M, F, device="cuda")).to(bf)
        out = torch.empty(M, F, device="cuda", dtype=bf)
        fl = 2.0 * M * D * F
        us = timeit(lambda: ops.gemm(M, F, D, dY, D, Wt, D, out, F, dt=1))
        print(f"M={M} dgrad-shape plain   {us:8.1f} us {fl / us / 1e6:8.1f} TF/s", flush=True)
        us = timeit(lambda: ops.gemm(M, F, D, dY, D, Wt, D, out, F, dt=1, gate=Hc, ldg=F))
        print(f"M={M} dgrad-shape gate    {us:8.1f} us {fl / us / 1e6:8.1f} TF/s", flush=True)
        W2 = (torch.randn(D, F, device="cuda") * 0.05).to(bf)    # conv2 fwd: [N=D][K=F]
        Y = torch.empty(M, D, device="cuda", dtype=bf)
        bias = torch.randn(D, device="cuda")
        us = timeit(lambda: ops.gemm(M, D, F, Hc, F, W2, F, Y, D, dt=1, bias=bias))
        print(f"M={M} conv2-fwd bias      {us:8.1f} us {fl / us / 1e6:8.1f} TF/s", flush=True)
        X = torch.randn(M, D, device="cuda").to(bf)
        Wo = (torch.randn(D, D, device="cuda") * 0.05).to(bf)
        us = timeit(lambda: ops.gemm(M, D, D, X, D, Wo, D, Y, D, dt=1, bias=bias))
        print(f"M={M} out_proj bias       {us:8.1f} us {2.0 * M * D * D / us / 1e6:8.1f} TF/s", flush=True)
        Wq = (torch.randn(3 * D, D, device="cuda") * 0.05).to(bf)
        Q = torch.empty(M, 3 * D, device="cuda", dtype=bf)
        bq = torch.randn(3 * D, device="cuda")
        us = timeit(lambda: ops.gemm(M, 3 * D, D, X, D, Wq, D, Q, 3 * D, dt=1, bias=bq))
        print(f"M={M} in_proj bias        {us:8.1f} us {6.0 * M * D * D / us / 1e6:8.1f} TF/s", flush=True)
        Wqt = Wq.t().contiguous()                                # [N=D][K=3D]
        us = timeit(lambda: ops.gemm(M, D, 3 * D, Q, 3 * D, Wqt, 3 * D, Y, D, dt=1))
        print(f"M={M} in_proj dgrad plain {us:8.1f} us {6.0 * M * D * D / us / 1e6:8.1f} TF/s", flush=True)
        us = timeit(lambda: ops.gemm(M, D, 3 * D, Q, 3 * D, Wqt, 3 * D, Y, D, dt=1, residual=X, ldr=D))
        print(f"M={M} in_proj dgrad resid {us:8.1f} us {6.0 * M * D * D / us / 1e6:8.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
