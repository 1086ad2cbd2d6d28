"""4-wave GEMM diagnostics: relative error per shape (plain, no epilogue) against torch, and
where the error sits (rows / columns / K).  Usage: python tools/w4_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402
from fastspeech2 import ops  # noqa: E402


def run(M, N, K, c32=0, kwin=None):
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    if kwin is not None:      # only K columns kwin[0] .. kwin[1] nonzero
        A[:, :kwin[0]] = 0
        A[:, kwin[1]:] = 0
    W = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    C = torch.zeros(M, N, device="cuda", dtype=torch.float32 if c32 else torch.bfloat16)
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, c_fp32=c32)
    torch.cuda.synchronize()
    err = (C.float() - ref).abs()
    bad = err > 0.05 * ref.abs().max()
    rel = (err.norm() / ref.norm()).item()
    msg = f"{M}x{N}x{K} c32={c32} kwin={kwin}: rel {rel:.2e}"
    if bad.any():
        r = bad.any(1).nonzero().flatten()
        c = bad.any(0).nonzero().flatten()
        msg += f"  bad rows {r.numel()} [{r.min().item()}..{r.max().item()}] (mod 256: {sorted(set((r % 256).tolist()))[:12]})"
        msg += f"  bad cols {c.numel()} [{c.min().item()}..{c.max().item()}] (mod 192: {sorted(set((c % 192).tolist()))[:12]})"
    print(msg, flush=True)


for shp in [(2100, 520, 256), (2048, 576, 1024), (31264, 1536, 3456), (2048, 384, 256),
            (4096, 1536, 256)]:
    run(*shp)
run(2100, 520, 256, 1)
