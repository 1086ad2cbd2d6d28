"""GPU: HiFi-GAN generator forward through libfs2_hip.so against the CPU
restatement oracle/vocoder_oracle.py -- "parity unpinned": speechbrain and its hub weights are
absent, so the oracle restates SB 1.0.x HifiganGenerator / ResBlock1.
Weights are re-drawn with fan-in scaling so the signal survives the four stages.
Tolerances: fp32 max|a-b| / max|b| <= 1e-3; bf16 <= 5e-2.

``test_config5_vocoder_256_sentences`` runs BASELINE config 5's vocoder leg at its workload:
the 256-sentence intensity sweep's mels (fastspeech2/inference.py:82-83) decoded as ONE padded
batch, checked by properties over the whole batch and against the restatement on 8 sentences
at their full length."""
import math

import numpy as np

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


def _sweep_mels(cfg_all, n=256, seed=8):
    """the 256-sentence sweep of test_gpu_inference.py (4 speakers x 5 emotions x 3 levels,
    20-70 phonemes, predicted durations) through a 2 + 2-layer FS2 in fp32"""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.inference import get_intensity_rep, synthesize
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
    torch.manual_seed(seed)
    m = FastSpeech2(**kw, n_speakers=4).cuda().eval()
    with torch.no_grad():
        m.durPred.linear.w.weight.mul_(0.05)
        m.durPred.linear.w.bias.fill_(1.8)     # ~5 frames per phoneme from random weights
    g = torch.Generator().manual_seed(5)
    bank = np.random.default_rng(2).standard_normal((4, 5, 3, 5)).astype(np.float32)
    phs, spk, inten = [], [], []
    for i in range(n):
        L = int(torch.randint(20, 71, (1,), generator=g))
        phs.append(torch.randint(1, 95, (L,), generator=g))
        s, e, lv = i % 4, (i // 4) % 5, (i // 20) % 3
        spk.append(s)
        inten.append(get_intensity_rep(s, e, lv, L, bank)[0])
    return synthesize(m, phs, spk, inten)


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-3), (torch.bfloat16, 5e-2)])
def test_config5_vocoder_256_sentences(cuda, cfg_all, dt, tol, parity_log):
    """BASELINE config 5 (256 sentences, mel-gen + HiFi-GAN) at its workload: the sweep's mels
    decoded as one (256, 80, T_max) batch, as the reference's decode_batch(model(...)[0]
    .permute(0, 2, 1)) (inference.py:82-83).  Held: the shape 256 x hop (T_max + 10); every
    sample finite and inside tanh's range; the batched rows equal single-sentence calls on the
    same padded rows (utterances are independent in the generator: its convs pad per
    utterance); and on 8 sentences decoded at their own full length, the restatement
    (fp32 1e-3, bf16 5e-2 relative, as the small-shape test)."""
    from fastspeech2.inference import vocode
    from oracle.vocoder_oracle import generator_forward
    mels, lens = _sweep_mels(cfg_all)
    assert len(mels) == 256 and min(lens) > 0
    g = _gen(dt)
    params = {k: v.detach().clone() for k, v in g.state_dict().items()}
    g = g.to(cuda)
    wav, nsamp = vocode(g, mels)
    torch.cuda.synchronize()
    Tmax = max(lens)
    assert wav.shape == (256, 1, 256 * (Tmax + 10))
    assert nsamp == [256 * L for L in lens]
    assert bool(torch.isfinite(wav).all())
    assert float(wav.abs().max()) <= 1.0
    assert float(wav.abs().max()) > 1e-2          # the signal survives the four stages
    pick = [0, 1, 37, 101, 128, 200, 254, 255]
    # batched rows == single-sentence calls on the same padded input rows
    batch_in = torch.zeros(len(pick), 80, Tmax, device=cuda)
    for r, i in enumerate(pick):
        batch_in[r, :, :lens[i]] = mels[i].float().t()
    same = [rel(g.decode_batch(batch_in[r:r + 1])[0], wav[i]) for r, i in enumerate(pick)]
    # the two calls may take different GEMM kernels (tile counts follow the batch size): equal
    # to fp32 rounding, and for bf16 to its one-ulp flips carried through 40 layers
    assert max(same) <= (1e-5 if dt == torch.float32 else 2e-2), same
    # 8 sentences at their own full length against the restatement (CPU, fp32)
    errs = []
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    for i in pick:
        mel_i = mels[i].float().t()[None]                    # (1, 80, T_i)
        got = g.decode_batch(mel_i.to(cuda))
        ref = generator_forward(params, mel_i.cpu())
        assert got.shape == ref.shape == (1, 1, 256 * (lens[i] + 10))
        errs.append(rel(got, ref))
    parity_log[f"config5_vocoder_256_{str(dt).split('.')[-1]}"] = {
        "batched_vs_single_rel_max": max(same), "restatement_rel_max": max(errs),
        "sentences": 256, "samples": int(wav.numel()), "frames": int(sum(lens))}
    assert max(errs) <= tol, errs
