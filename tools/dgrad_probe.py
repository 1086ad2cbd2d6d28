"""Conv data gradient (decoder FFN conv1, k = 9): the shift-conv GEMM (conv_mode 4, per-K-tile
tap offsets and row bounds) vs a plain K-major GEMM whose A rows overlap (lda = O < K) over a
zero-padded token-major dY image -- the form the data gradient takes with the taps of the
weight image reversed.  Timing only (the plain call's tap order is not the conv's)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def case(name, B, T, O, C, KW):
    from fastspeech2 import ops
    from fastspeech2.engine import dgrad_split
    P = (KW - 1) // 2
    M = B * T
    Mp = B * (T + 2 * P)
    K = KW * O
    bf = torch.bfloat16
    dY = (torch.randn(M, O, device="cuda") * 0.5).to(bf)
    Wb = (torch.randn(C, K, device="cuda") * 0.05).to(bf)
    split = dgrad_split(Mp, C, K, 1)
    Xpad = torch.empty(split, Mp, C, dtype=torch.float32, device="cuda")
    fl = 2.0 * Mp * C * K
    img = torch.zeros(Mp + 2 * P + 8, O, device="cuda", dtype=bf)

    def a():
        ops.gemm(Mp, C, K, dY, O, Wb, K, Xpad, C, dt=1, conv=(4, T, KW, O), c_fp32=1,
                 split_k=split, split_stride=Mp * C if split > 1 else 0)
    ta = timed(a)

    def b():
        ops.gemm(Mp, C, K, img, O, Wb, K, Xpad, C, dt=1, c_fp32=1, split_k=split,
                 split_stride=Mp * C if split > 1 else 0)
    tb = timed(b)
    print(f"{name}: split {split}  conv_mode 4 {ta:7.1f} us ({fl / ta / 1e6:5.0f} TF/s)   "
          f"plain overlapping rows {tb:7.1f} us ({fl / tb / 1e6:5.0f} TF/s)", flush=True)


def main():
    from fastspeech2 import _native
    _native.load()
    case("decoder conv1 dgrad", 32, 977, 1536, 384, 9)
    case("encoder conv1 dgrad", 32, 200, 1536, 384, 9)
    case("postnet mid dgrad  ", 32, 977, 512, 512, 5)


if __name__ == "__main__":
    main()
