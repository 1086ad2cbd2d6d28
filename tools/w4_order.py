"""The decoder / encoder FFN conv1 forward exactly as the engine issues it (tap-inner K order
over the reflect-padded image, a_kw = 9, pad rows dropped by c_row), timed per launch; run
under FS2_W4_FLAGS=0 / 8 (experiments library: 8 = column-tile-major block order)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
os.environ.setdefault("FS2_HIP_LIB", os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd",
                                                  "fastspeech2", "libfs2_hip_exp.so"))
import torch  # noqa: E402


def timed(fn, n=30):
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
    torch.manual_seed(0)
    C, O, KW = 384, 1536, 9
    P = (KW - 1) // 2
    res = {}
    for name, B, T in (("dec", 32, 977), ("enc", 32, 200)):
        Mp = B * (T + 2 * P)
        img = (torch.rand(Mp + 64, C, device="cuda") * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand(O, KW * C, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.randn(O, device="cuda")
        Y = torch.empty(B * T, O, device="cuda", dtype=torch.bfloat16)
        fn = lambda: ops.gemm(Mp, O, KW * C, img, C, W, KW * C, Y, O, dt=1, c_row=(T, -2 * P),
                              a_kw=KW, bias=bias, relu=1)
        t = timed(fn)
        fn()
        torch.cuda.synchronize()
        res[name] = Y.float().sum().item()
        print(f"flags={os.environ.get('FS2_W4_FLAGS', '0')} {name} conv1 fwd {t:7.1f} us "
              f"{2.0 * B * T * O * KW * C / t / 1e6:6.0f} TF/s  checksum {res[name]:.6e}", flush=True)


if __name__ == "__main__":
    main()
