"""fs2_loss_fwd_bwd (MSE x 5 + SSIM, forward and gradients) at the bench shape: B=32, T_mel=977
(lengths 489..977), T_phon=200, 80 mels, bf16 predictions.  Prints us per call; run under
rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import _native
    from fastspeech2.loss import fused_loss
    _native.load()
    B, Tm, Tp, NM = 32, 977, 200, 80
    g = torch.Generator().manual_seed(3)
    mel_len = torch.tensor(sorted([Tm] + torch.randint(Tm // 2, Tm + 1, (B - 1,), generator=g).tolist(),
                                  reverse=True))
    phon_len = torch.full((B,), Tp)
    d = torch.ones(B, Tp, dtype=torch.int64)
    bf = torch.bfloat16
    dev = "cuda"
    tgt = torch.randn(B, Tm, NM, device=dev) * 2 - 4
    mel = (torch.randn(B, Tm, NM, device=dev) * 2 - 4).to(bf)
    post = (mel.float() + 0.1 * torch.randn(B, Tm, NM, device=dev)).to(bf)
    ld, pp, pe = (torch.randn(B, Tp, device=dev).to(bf) for _ in range(3))
    ap, ae = torch.randn(B, Tp, device=dev), torch.randn(B, Tp, device=dev)
    args = (mel, post, ld, pp, pe, tgt, d.to(dev), ap, ae, mel_len.to(dev), phon_len.to(dev),
            (1.0,) * 6)
    for _ in range(3):
        fused_loss(*args)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fused_loss(*args)
    b.record()
    torch.cuda.synchronize()
    print(f"fs2_loss_fwd_bwd B={B} Tm={Tm}: {a.elapsed_time(b) / 20 * 1e3:.1f} us per call "
          f"(includes fused_loss's host-side tensor setup)", flush=True)


if __name__ == "__main__":
    main()
