"""Short-K GEMM shapes of the encoder / predictors / mel linear (M = 6400 or the decoder's
31264 x 80) on the persistent short-K kernel's tile configurations: run once per FS2_PK_CFG
(44 / 24 / 22, or unset = the dispatcher's choice) with the experiments library; prints us per
call, TF/s and the relative error against an fp32 reference on the same bf16 values."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FS2_HIP_LIB", os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd",
                                                  "fastspeech2", "libfs2_hip_exp.so"))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402
from fastspeech2 import ops  # noqa: E402


def timeit(fn, n=30):
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


SHAPES = [  # name, M, N, K, epilogue
    ("enc out_proj fwd", 6400, 384, 384, "bias"),
    ("enc in_proj fwd", 6400, 1152, 384, "bias"),
    ("enc conv2 fwd", 6400, 384, 1536, "bias"),
    ("enc in_proj dgrad", 6400, 384, 1152, "residual"),
    ("enc out_proj dgrad", 6400, 384, 384, None),
    ("enc conv2 dgrad", 6400, 1536, 384, "gate"),
    ("concat_proj fwd", 6400, 384, 776, "rowscale"),
    ("concat_proj dgrad", 6400, 768, 384, None),
    ("mel linear fwd", 31264, 80, 384, "bias"),
    ("mel linear dgrad", 31264, 384, 80, None),
]


def main():
    bf = torch.bfloat16
    cfg = os.environ.get("FS2_PK_CFG", "auto")
    for name, M, N, K, epi in SHAPES:
        torch.manual_seed(M + N + K)
        A = torch.randn(M, K, device="cuda").to(bf)
        W = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        C = torch.empty(M, N, device="cuda", dtype=bf)
        ref = A.float() @ W.float().t()
        kw = {}
        if epi == "bias":
            b = torch.randn(N, device="cuda")
            kw = dict(bias=b)
            ref = ref + b
        elif epi == "residual":
            R = torch.randn(M, N, device="cuda").to(bf)
            kw = dict(residual=R, ldr=N)
            ref = ref + R.float()
        elif epi == "gate":
            G = torch.randn(M, N, device="cuda").to(bf)
            kw = dict(gate=G, ldg=N)
            ref = torch.where(G.float() > 0, ref, 0.0)
        elif epi == "rowscale":
            rs = (torch.rand(M, device="cuda") > 0.2).float()
            kw = dict(row_scale=rs)
            ref = ref * rs[:, None]
        us = timeit(lambda: ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, **kw))
        err = ((C.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"cfg={cfg:4s} {name:20s} M={M:6d} N={N:5d} K={K:5d} {us:8.1f} us "
              f"{2.0 * M * N * K / us / 1e6:7.1f} TF/s  rel {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
