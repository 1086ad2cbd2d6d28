"""Seeded synthetic batches shaped like EmoV-DB collates.

Reproduces the layout of ``TextMelCollateWithAlignment`` (fastspeech2/dataset.py:62-133):
utterances sorted by phoneme length (descending), tokens / durations zero-padded to the
longest utterance, mel (B, T_mel_max, 80), pitch / energy (B, T_mel_max) zero-padded, and
durations summing exactly to each mel length (MFA alignments).  ``intensity`` is the
(B, T_phon, 5) phoneme-level emotion-intensity input (train.py:16-51), zero in padding.

Draws: tokens ~ U{1..n_char-1} (0 = pad), T_phon ~ U{tp_min..tp_max}, durations ~ U{1..9}
rescaled so that sum <= t_mel_cap, mel ~ N(-4, 2) clipped to [-11.5, 2.5] (log-mel range),
pitch / energy ~ N(0, 1) with 15 % unvoiced (exact zero) pitch frames, speakers ~ U{0..n_spk-1},
intensity ~ N(0, 1) (zeros if ``emotion=False``), emotion ids ~ U{0..4} (``single_speaker``: every
speaker id 0, BASELINE config 2's 'bea', other draws unchanged); ``rank_x`` is the collate's
(B, n_mels + 2, T_mel) extractor input built from mel / pitch / energy.
"""

import torch


def _durations(g, tp, cap):
    d = torch.randint(1, 10, (tp,), generator=g)
    s = int(d.sum())
    if s > cap:
        d = torch.clamp((d.float() * cap / s).floor().long(), min=1)
        while int(d.sum()) > cap:
            d[int(torch.argmax(d))] -= 1
    return d


def make_batch(B=32, tp_min=100, tp_max=200, t_mel_cap=1000, n_mels=80, n_char=95, n_spk=4,
               seed=0, emotion=True, max_shape=False, device="cpu", fixed_tp=None,
               single_speaker=False):
    g = torch.Generator().manual_seed(seed)
    if max_shape:
        tps = [tp_max] * B
    elif fixed_tp is not None:
        tps = [fixed_tp] * B
    else:
        tps = torch.randint(tp_min, tp_max + 1, (B,), generator=g).tolist()
    tps = sorted(tps, reverse=True)                       # collate sorts descending
    Tp = tps[0]
    durs = []
    for tp in tps:
        if max_shape:
            durs.append(torch.full((tp,), max(1, t_mel_cap // tp), dtype=torch.long))
        else:
            durs.append(_durations(g, tp, t_mel_cap))
    mel_lens = [int(d.sum()) for d in durs]
    Tm = max(mel_lens)
    phoneme = torch.zeros(B, Tp, dtype=torch.long)
    duration = torch.zeros(B, Tp, dtype=torch.long)
    intensity = torch.zeros(B, Tp, 5)
    mel = torch.zeros(B, Tm, n_mels)
    pitch = torch.zeros(B, Tm)
    energy = torch.zeros(B, Tm)
    for b, (tp, d, L) in enumerate(zip(tps, durs, mel_lens)):
        phoneme[b, :tp] = torch.randint(1, n_char, (tp,), generator=g)
        duration[b, :tp] = d
        if emotion:
            intensity[b, :tp] = torch.randn(tp, 5, generator=g)
        mel[b, :L] = (torch.randn(L, n_mels, generator=g) * 2.0 - 4.0).clamp(-11.5, 2.5)
        p = torch.randn(L, generator=g)
        p[torch.rand(L, generator=g) < 0.15] = 0.0
        pitch[b, :L] = p
        energy[b, :L] = torch.randn(L, generator=g)
    speakers = torch.randint(0, n_spk, (B,), generator=g)
    emotions = torch.randint(0, 5, (B,), generator=g)     # drawn last: earlier fields unchanged
    if single_speaker:           # BASELINE config 2: EmoV-DB speaker 'bea' (id 0) only
        speakers = torch.zeros_like(speakers)
    # rank_X as the collate builds it: cat(mel^T, pitch, energy) -> (B, n_mels + 2, T_mel)
    # (dataset.py:94,116-117), the frozen IntensityExtractor's input (train.py:27)
    rank_x = torch.cat([mel.transpose(1, 2), pitch[:, None], energy[:, None]], dim=1)
    batch = dict(phoneme=phoneme, speakers=speakers, phon_len=torch.tensor(tps, dtype=torch.long),
                 mel=mel, pitch=pitch, energy=energy, duration=duration,
                 mel_len=torch.tensor(mel_lens, dtype=torch.long), intensity=intensity,
                 rank_x=rank_x, emotions=emotions)
    return {k: v.to(device) for k, v in batch.items()}


def as_tuple(batch):
    """The reference train loop's 8 leading collate fields (train.py:62-65) + intensity."""
    return ((batch["phoneme"], batch["speakers"], batch["phon_len"], batch["mel"], batch["pitch"],
             batch["energy"], batch["duration"], batch["mel_len"]), batch["intensity"])


def as_collate(batch):
    """The reference collate's full 12-tuple (dataset.py:120-133; labels / wavs are None)."""
    return (batch["phoneme"], batch["speakers"], batch["phon_len"], batch["mel"], batch["pitch"],
            batch["energy"], batch["duration"], batch["mel_len"], None, None, batch["rank_x"],
            batch["emotions"])


def valid_frames(batch):
    return int(batch["mel_len"].sum())
