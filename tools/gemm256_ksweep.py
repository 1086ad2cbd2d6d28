"""Main-loop rate vs fixed cost of the 256x256 kernel at the decoder FFN conv1 output shape
(M = 31264, N = 1536, plain K-major operands, persistent short-K kernel disabled): t = a + b*K."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
os.environ["FS2_GEMM_NO_PK"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from fastspeech2 import ops, _native
    _native.load()
    for M, N in ((31264, 1536), (4096, 4096)):
        res = []
        for K in (512, 1024, 2048, 3456, 6912):
            A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            W = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            fn = lambda: ops.gemm(M, N, K, A, K, W, K, C, N, dt=1)
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                fn()
            b.record()
            torch.cuda.synchronize()
            res.append((K, a.elapsed_time(b) / 10 * 1e3))
        ks, us = np.array([r[0] for r in res], float), np.array([r[1] for r in res])
        bb, aa = np.polyfit(ks, us, 1)
        print(f"M{M} N{N}: " + " ".join(f"K{k}:{u:.1f}us({2 * M * N * k / u / 1e6:.0f})" for k, u in res)
              + f" | fit fixed {aa:.1f} us, loop {2 * M * N / bb / 1e6:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
