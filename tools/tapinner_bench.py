"""Decoder FFN conv1 data gradient over the padded dY image (M = 31520 padded rows, N = 384,
K = 9 x 1536): natural K order vs the tap-inner order (fs2_gemm_desc.a_kw), standalone.
Usage: python tools/tapinner_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402
from fastspeech2 import ops  # noqa: E402


def t(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


B, T, O, C, KW = 32, 977, 1536, 384, 9
P = (KW - 1) // 2
Mp = B * (T + 2 * P)
img = (torch.randn(Mp + 2 * P, O, device="cuda") * 0.5).to(torch.bfloat16)
Wm = torch.randn(O, KW, C, device="cuda") * 0.05
ldf = ops.round_up(KW * C, 8)
Wf = torch.empty(O, ldf, device="cuda", dtype=torch.bfloat16)
Wr = torch.empty(C, KW * O, device="cuda", dtype=torch.bfloat16)
Wt = torch.empty(C, KW * O, device="cuda", dtype=torch.bfloat16)
ops.weight_prep(Wm, O, C, KW, Wf, ldf, Wr, KW * O, dt=1, w_okc=3)
ops.weight_prep(Wm, O, C, KW, Wf, ldf, Wt, KW * O, dt=1, w_okc=7)
X = torch.empty(Mp, C, device="cuda")
nat = t(lambda: ops.gemm(Mp, C, KW * O, img, O, Wr, KW * O, X, C, dt=1, c_fp32=1))
ti = t(lambda: ops.gemm(Mp, C, KW * O, img, O, Wt, KW * O, X, C, dt=1, c_fp32=1, a_kw=KW))
fl = 2.0 * Mp * C * KW * O
print(f"natural {nat:.1f} us ({fl / nat / 1e6:.0f} TF/s)   tap-inner {ti:.1f} us ({fl / ti / 1e6:.0f} TF/s)")
