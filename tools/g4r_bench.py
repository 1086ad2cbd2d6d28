"""gemm256r_kernel (full-row LDS regions) vs gemm256_kernel (K-half regions): run once with
FS2_G4R=1 and once with FS2_G4R=0 (experiments library); prints time per shape and saves the
outputs to /tmp/g4r_<flag>.pt so the two runs can be compared bit for bit (same K order)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
os.environ.setdefault("FS2_HIP_LIB", os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd",
                                                  "fastspeech2", "libfs2_hip_exp.so"))
import torch  # noqa: E402


def timed(fn, n=20):
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
    from fastspeech2 import ops
    flag = os.environ.get("FS2_G4R", "1")
    torch.manual_seed(0)
    bf = torch.bfloat16
    outs = {}
    cases = [("dec conv1 fwd (reflect k9)", 32, 977, 384, 1536, 9, 1),
             ("postnet conv fwd (reflect k5)", 32, 977, 512, 512, 5, 1),
             ("enc conv1 fwd (reflect k9, T200)", 32, 200, 384, 1536, 9, 1),
             ("plain 31264x1536x3456", 32, 977, 3456, 1536, 1, 0),
             ("plain 8192^3", 8, 1024, 8192, 8192, 1, 0),
             ("plain 4096^3", 4, 1024, 4096, 4096, 1, 0)]
    only = os.environ.get("G4R_ONLY")
    for name, B, T, C, O, KW, conv in cases:
        if only and only not in name:
            continue
        M, K = B * T, KW * C
        data = os.environ.get("G4R_DATA", "rand")
        if data == "zero":
            X = torch.zeros(M, C, device="cuda", dtype=bf)
            W = torch.zeros(O, K, device="cuda", dtype=bf)
        elif data == "act":   # LayerNorm-output-like activations, init-scale weights
            X = torch.randn(M, C, device="cuda").to(bf)
            W = (torch.randn(O, K, device="cuda") * (1.0 / K) ** 0.5).to(bf)
        else:
            X = (torch.rand(M, C, device="cuda") * 2 - 1).to(bf)
            W = (torch.rand(O, K, device="cuda") * 2 - 1).to(bf) * 0.05
        bias = torch.randn(O, device="cuda")
        Y = torch.empty(M, O, device="cuda", dtype=bf)
        kw = dict(conv=(1, T, KW, C)) if conv else {}
        fn = lambda: ops.gemm(M, O, K, X, C, W, K, Y, O, dt=1, bias=bias, relu=1, **kw)
        t = timed(fn)
        outs[name] = Y.cpu()
        print(f"G4R={flag} data={data} flags={os.environ.get('FS2_G4_FLAGS', '0')} {name:32s} {t:8.1f} us  {2.0 * M * O * K / t / 1e6:6.0f} TF/s", flush=True)
    # FFN conv1 data gradient over the zero-padded dY image: A rows overlap (lda = F < K = 9F),
    # N = 384, fp32 output (the 256x192 instance)
    name = "dgrad 31680x384x13824 overlap"
    if not only or only in name:
        Mp, F, C, KW = 32 * 990, 1536, 384, 9
        img = (torch.rand(Mp + 16, F, device="cuda") * 2 - 1).to(bf)
        Wb = ((torch.rand(C, KW * F, device="cuda") * 2 - 1) * 0.05).to(bf)
        Y = torch.empty(Mp, C, device="cuda")
        fn = lambda: ops.gemm(Mp, C, KW * F, img, F, Wb, KW * F, Y, C, dt=1, c_fp32=1)
        t = timed(fn)
        outs[name] = Y.cpu()
        print(f"G4R={flag} {name:32s} {t:8.1f} us  "
              f"{2.0 * Mp * C * KW * F / t / 1e6:6.0f} TF/s", flush=True)
    if not only:
        torch.save(outs, f"/tmp/g4r_{flag}.pt")


if __name__ == "__main__":
    main()
