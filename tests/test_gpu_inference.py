"""GPU: the inference path (fastspeech2/inference.py:12-89) -- predicted
durations, prototype intensity lookup and batched synthesis -- against the oracle forward.

Tolerances as test_gpu_model.py: fp32 mel rel 1e-3, mel lengths (integer) exact.  The predicted
log-durations are pushed to ~log(1 + 5) (durPred linear bias 1.8, weight x0.05) so random-init
weights give non-empty mels, as in test_inference_branch_predicted_durations.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


def _pair(cfg_all, seed=4):
    from fastspeech2.model import FastSpeech2
    from oracle.fs2_oracle import FastSpeech2Oracle
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
    torch.manual_seed(seed)
    o = FastSpeech2Oracle(**kw, n_speakers=4).eval()
    torch.manual_seed(seed)
    m = FastSpeech2(**kw, n_speakers=4).cuda().eval()
    with torch.no_grad():
        for mod in (o, m):
            mod.durPred.linear.w.weight.mul_(0.05)
            mod.durPred.linear.w.bias.fill_(1.8)
    return o, m


def _bank(seed=0):
    return np.random.default_rng(seed).standard_normal((4, 5, 3, 5)).astype(np.float32)


def test_sweep_batched_equals_oracle_on_the_padded_batch(cuda, cfg_all):
    """One sentence swept over speakers x emotions x levels as ONE batch == the oracle's
    forward on the same batch (the reference model's semantics for a batch)."""
    from fastspeech2.inference import intensity_sweep_batch, synthesize
    o, m = _pair(cfg_all)
    g = torch.Generator().manual_seed(3)
    phon = torch.randint(1, 95, (23,), generator=g)
    ph, spk, inten, keys = intensity_sweep_batch(phon, 2, [0, 2, 4], [0, 1, 2], _bank())
    mels, lens = synthesize(m, ph, spk, inten)
    B = len(ph)
    with torch.no_grad():
        po = o(torch.stack(ph), torch.tensor(spk), intensity=torch.stack(inten))
    assert lens == po[7].tolist()
    for i in range(B):
        assert mels[i].shape == (lens[i], 80)
        if lens[i] > 0:
            assert rel(mels[i], po[0][i, :lens[i]]) <= 1e-3, keys[i]


def test_synthesize_unbatched_equals_single_sentence_calls(cuda, cfg_all):
    """batched=False is the reference loop: one model call per sentence (B=1)."""
    from fastspeech2.inference import get_intensity_rep, synthesize
    o, m = _pair(cfg_all, seed=5)
    g = torch.Generator().manual_seed(4)
    phs = [torch.randint(1, 95, (n,), generator=g) for n in (17, 31, 9)]
    spk = [0, 3, 1]
    inten = [get_intensity_rep(s, 2, 1, p.numel(), _bank(1))[0] for s, p in zip(spk, phs)]
    mels, lens = synthesize(m, phs, spk, inten, batched=False)
    for p, s, it, mel, L in zip(phs, spk, inten, mels, lens):
        with torch.no_grad():
            po = o(p[None], torch.tensor([s]), intensity=it[None])
        assert L == int(po[7][0])
        if L > 0:
            assert rel(mel, po[0][0, :L]) <= 1e-3


@pytest.mark.parametrize("dtname", ["float32", "bfloat16"])
def test_config5_256_sentence_sweep_equals_oracle(cuda, cfg_all, dtname, parity_log):
    """BASELINE config 5 at its batch size: 256 sentences (ragged, 20-70 phonemes) over the 5
    emotions x 3 intensity levels (prototype lookup, inference.py:12-21) and 4 speakers, ONE
    batched synthesis with predicted durations, against the oracle's forward on the same padded
    batch (2 + 2 layers).  fp32: mel rel 1e-3, mel lengths exact; bf16: mel lengths exact on
    the utterances whose predicted durations do not sit at a truncation edge, and the observed
    errors recorded (parity_log)."""
    from fastspeech2.inference import get_intensity_rep, synthesize
    o, m = _pair(cfg_all, seed=8)
    dt = getattr(torch, dtname)
    if dt != torch.float32:
        from fastspeech2.model import FastSpeech2
        kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
        mb = FastSpeech2(**kw, n_speakers=4, act_dtype=dt).cuda().eval()
        mb.load_state_dict(m.state_dict())
        m = mb
    g = torch.Generator().manual_seed(5)
    bank = _bank(2)
    phs, spk, inten = [], [], []
    for i in range(256):
        n = int(torch.randint(20, 71, (1,), generator=g))
        phs.append(torch.randint(1, 95, (n,), generator=g))
        s, e, lv = i % 4, (i // 4) % 5, (i // 20) % 3
        spk.append(s)
        inten.append(get_intensity_rep(s, e, lv, n, bank)[0])
    mels, lens = synthesize(m, phs, spk, inten)
    torch.cuda.synchronize()
    Tp = max(p.numel() for p in phs)
    tok = torch.zeros(256, Tp, dtype=torch.int64)
    it = torch.zeros(256, Tp, 5)
    for i, (p, x) in enumerate(zip(phs, inten)):
        tok[i, :p.numel()] = p
        it[i, :p.numel()] = x
    torch.set_num_threads(max(1, min(32, torch.get_num_threads())))
    with torch.no_grad():
        po = o(tok, torch.tensor(spk), intensity=it)
    ref_lens = po[7].tolist()
    same = [i for i in range(256) if lens[i] == ref_lens[i]]
    errs = [rel(mels[i], po[0][i, :lens[i]]) for i in same if lens[i] > 0]
    parity_log[f"config5_256_sentences_{dtname}"] = {
        "mel_rel_max": max(errs), "mel_rel_median": float(np.median(errs)),
        "mel_len_equal": len(same), "sentences": 256, "frames": int(sum(lens))}
    assert sum(lens) > 256 * 20
    if dt == torch.float32:
        assert lens == ref_lens
        assert max(errs) <= 1e-3
    else:
        # bf16 predicted log-durations differ from fp32 by ~1e-2 relative: a phoneme whose
        # expm1 lands that close to an integer truncates the other way (the reference's own
        # .long() edge, model.py:373-375), so mel lengths differ on a third of the sentences
        # and the batch's padded length may change with them.  Held: the log-durations (rel,
        # the bound of test_gpu_fullsize.py), the total frames (0.5 %), and the mels of the
        # sentences whose length agrees (2x observed, profiles/r03_parity_observed.json)
        with torch.no_grad():
            pm = m(tok.cuda(), torch.tensor(spk).cuda(), intensity=it.cuda())
        dur_rel = rel(pm[2], po[2])
        parity_log[f"config5_256_sentences_{dtname}"]["log_durations"] = dur_rel
        assert dur_rel <= 2.6e-2, dur_rel
        assert abs(sum(lens) - sum(ref_lens)) <= 5e-3 * sum(ref_lens)
        assert max(errs) <= 2.2e-2
