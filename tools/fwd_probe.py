"""Conv forward (FFN conv1, k = 9): the reflect implicit conv (conv_mode 1) vs a plain K-major
GEMM with overlapping A rows (lda = C < K) over a reflect-padded token-major X image, i.e. the
padded-domain form of the forward (2P garbage rows per utterance).  Timing only."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402
from dgrad_probe import timed  # noqa: E402


def case(name, B, T, C, O, KW):
    from fastspeech2 import ops
    P = (KW - 1) // 2
    M, Mp, K = B * T, B * (T + 2 * P), KW * C
    bf = torch.bfloat16
    X = (torch.randn(M, C, device="cuda") * 0.5).to(bf)
    Wf = (torch.randn(O, K, device="cuda") * 0.05).to(bf)
    bias = torch.randn(O, device="cuda")
    Y = torch.empty(Mp, O, device="cuda", dtype=bf)
    img = torch.zeros(Mp + 2 * P + 8, C, device="cuda", dtype=bf)
    fl = 2.0 * M * O * K
    ta = timed(lambda: ops.gemm(M, O, K, X, C, Wf, K, Y, O, dt=1, conv=(1, T, KW, C), bias=bias,
                                relu=1))
    tb = timed(lambda: ops.gemm(Mp, O, K, img, C, Wf, K, Y, O, dt=1, bias=bias, relu=1))
    print(f"{name}: conv_mode 1 {ta:7.1f} us ({fl / ta / 1e6:5.0f} TF/s)   plain padded "
          f"{tb:7.1f} us ({fl / tb / 1e6:5.0f} TF/s of useful FLOPs)", flush=True)


def main():
    from fastspeech2 import _native
    _native.load()
    case("decoder conv1 fwd", 32, 977, 384, 1536, 9)
    case("encoder conv1 fwd", 32, 200, 384, 1536, 9)
    case("postnet mid fwd  ", 32, 977, 512, 512, 5)


if __name__ == "__main__":
    main()
