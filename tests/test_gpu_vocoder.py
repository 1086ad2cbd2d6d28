"""GPU: HiFi-GAN generator forward through libfs2_hip.so against the CPU
restatement oracle/vocoder_oracle.py -- "parity unpinned": speechbrain and its hub weights are
absent, so the oracle restates SB 1.0.x HifiganGenerator / ResBlock1.
Weights are re-drawn with fan-in scaling so the signal survives the four stages.
Tolerances: fp32 max|a-b| / max|b| <= 1e-3; bf16 <= 5e-2."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


def _gen(dt, seed=0):
    from fastspeech2.vocoder import HifiganGenerator
    torch.manual_seed(seed)
    g = HifiganGenerator(act_dtype=dt)
    with torch.no_grad():
        for name, p in g.named_parameters():
            if name.endswith("weight_v"):
                fan = p[0].numel() if "ups" not in name else 2 * p.shape[0]
                p.normal_(0.0, 1.0 / math.sqrt(fan))
                gname = name[:-1] + "g"
                dict(g.named_parameters())[gname].copy_(
                    p.flatten(1).norm(dim=1).reshape(-1, *([1] * (p.dim() - 1))) * 1.2)
            elif name.endswith("bias"):
                p.normal_(0.0, 0.1)
    return g


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-3), (torch.bfloat16, 5e-2)])
def test_vocoder_matches_restatement(cuda, dt, tol):
    from oracle.vocoder_oracle import generator_forward
    g = _gen(dt)
    params = {k: v.detach().clone() for k, v in g.state_dict().items()}
    g = g.to(cuda)
    mel = (torch.randn(2, 80, 23, generator=torch.Generator().manual_seed(1)) * 2 - 4)
    wav = g.decode_batch(mel.to(cuda))
    ref = generator_forward(params, mel)
    assert wav.shape == ref.shape == (2, 1, 256 * (23 + 10))
    assert ref.abs().max() > 1e-2          # the signal survives the four stages
    assert rel(wav, ref) <= tol
