"""hipBLASLt kernel choice (torch.matmul, bf16) on the FFT-block GEMM shapes: run under
rocprofv3 --kernel-trace --stats to read the macro-tile / stream-K fields of the kernel names."""
import torch

bf = torch.bfloat16
D, F = 384, 1536
for M in (6400, 31264):
    X = torch.randn(M, D, device="cuda").to(bf)
    Hc = torch.randn(M, F, device="cuda").to(bf)
    Xc = torch.randn(M, 9 * D, device="cuda").to(bf)
    W3 = torch.randn(3 * D, D, device="cuda").to(bf)
    Wf = torch.randn(F, D, device="cuda").to(bf)
    Wc = torch.randn(F, 9 * D, device="cuda").to(bf)
    for name, fn in (("in_proj", lambda: X @ W3.t()), ("conv2_dgrad", lambda: X @ Wf.t()),
                     ("conv2_fwd", lambda: Hc @ Wf), ("conv1_fwd", lambda: Xc @ Wc.t())):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            fn()
        b.record()
        torch.cuda.synchronize()
        print(M, name, round(a.elapsed_time(b) / 20 * 1e3, 1), "us", flush=True)
