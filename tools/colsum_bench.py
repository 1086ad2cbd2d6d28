"""fs2_colsum (bias gradients) standalone at the step's shapes, bf16: us per call (colsum
kernel + reduce_parts) and GB/s of the matrix read.  FS2_COLSUM_SLAB=0 on the experiments
library: the sub-row kernel for every width."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import ops, _native
    _native.load()
    for M, N in ((31264, 1152), (31264, 384), (31264, 1536), (6400, 1152), (6400, 384), (31264, 80)):
        X = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        out = torch.zeros(N, device="cuda")
        ws = torch.empty(int(ops.colsum_ws(M, N)), device="cuda")
        fn = lambda: ops.colsum(X, N, M, N, out, dt=1, ws=ws, accumulate=1)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            fn()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 20 * 1e3
        print(f"M={M} N={N} colsum {us:7.1f} us  {M * N * 2 / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
