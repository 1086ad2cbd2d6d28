"""Inference path (BASELINE config 5): emotion-intensity sweeps through the
MI355X FastSpeech2 forward with predicted durations.

Reference: emo_rank_tts/fastspeech2/inference.py
* ``get_intensity_rep`` -- :12-21 (prototype lookup in the rank model's ``intensity.npy`` bank of
  shape (n_speakers, n_emotions, bucket_size, n_emotions), rank_model/inference.py:93-118);
* ``load_model``        -- :24-28;
* the sweep loop        -- :55-89: for every (speaker, emotion, level) one ``model(phon_ids,
  spkr_ids, intensity=...)`` call (durations predicted: ``clamp(expm1(log_d), 0)`` then
  truncation, model.py:372-375,408) and the vocoder.

Differences, each deliberate:
* the reference's ``emotion == 'neutral'`` branch (:13-14) compares the STRING 'neutral' with the
  integer ``emo_id`` its caller passes (:34, :76), so it never fires and every emotion, neutral
  included, reads ``intensity_bank[spk][emo][lv]``.  ``get_intensity_rep`` does the same for
  every integer id.  Only when it is given the string 'neutral' (the dead branch) does it return
  zeros, of width n_emotions: the reference's (1, T_phon, 256) there would be rejected by the
  concat projection (model.py:201: 2*D + 5 inputs);
* ``synthesize`` runs many sentences as ONE padded batch on the GPU.  Its outputs equal the
  model's forward on that padded batch (what the reference's model computes for a batch, e.g.
  valid_one_epoch), not B=1 calls: padded rows are live inside the FFT blocks
  and the attention masks tile across the batch (App. B-1), so a sentence's mel can depend on
  the batch it shares.  ``synthesize(..., batched=False)`` runs one sentence per call, which is
  the reference loop exactly;
* ``synthesize`` returns mel spectrograms; ``vocode`` then decodes them the way the reference
  does (inference.py:82-83: ``model(...)[0].permute(0, 2, 1)`` -> ``vocoder.decode_batch``) with
  the HIP HiFi-GAN generator of ``fastspeech2.vocoder`` (architecture only: the
  speechbrain hub weights are not available offline).
"""

import numpy as np
import torch

from .model import FastSpeech2


def get_intensity_rep(speaker, emotion, intensity_lv, T_phon, intensity_bank, n_emotions=5):
    """Per-phoneme intensity input (1, T_phon, n_emotions) for one (speaker, emotion, level)
    (fastspeech2/inference.py:12-21 as called at :76, i.e. with an integer emotion id).
    ``intensity_bank`` is the (n_spk, n_emo, bucket, n_emo) prototype array (or a path to the
    .npy, loaded without pickle).  ``emotion == 'neutral'`` (a string, the reference's
    unreachable branch) gives zeros."""
    if isinstance(emotion, str) and emotion == "neutral":
        return torch.zeros(1, T_phon, n_emotions, dtype=torch.float32)
    if isinstance(intensity_bank, str):
        intensity_bank = np.load(intensity_bank, allow_pickle=False)
    proto = torch.from_numpy(np.asarray(intensity_bank[speaker][emotion][intensity_lv],
                                        dtype=np.float32))
    return proto.reshape(1, 1, -1).expand(1, T_phon, -1)


def load_model(fastspeech2_pth_path, model_config, speaker_list, device, act_dtype=torch.float32):
    """fastspeech2/inference.py:24-28 (weights-only checkpoint load)."""
    model = FastSpeech2(**model_config, n_speakers=len(speaker_list), act_dtype=act_dtype)
    model.load_state_dict(torch.load(fastspeech2_pth_path, map_location="cpu", weights_only=True))
    return model.to(device).eval()


@torch.no_grad()
def synthesize(model, phonemes, speakers, intensities, pace=1.0, batched=True):
    """Mel spectrograms for a list of sentences.

    phonemes: list of 1-D int64 token tensors; speakers: list / tensor of speaker ids;
    intensities: list of (T_i, n_emotions) tensors (or (1, T_i, n_emotions)).  Returns a list
    of (T_mel_i, n_mels) mel tensors -- ``model(...)[0]`` as the reference's inference.py:82
    uses, i.e. ``mel_post``, the mel-linear output BEFORE the PostNet residual
    (model.py:430,433) -- trimmed to the predicted mel length, and the list of mel lengths."""
    dev = next(model.parameters()).device
    if not batched:
        mels, lens = [], []
        for p, s, it in zip(phonemes, speakers, intensities):
            m, l = synthesize(model, [p], [s], [it], pace=pace, batched=True)
            mels += m
            lens += l
        return mels, lens
    B = len(phonemes)
    Tp = max(int(p.numel()) for p in phonemes)
    n_emo = intensities[0].shape[-1]
    tok = torch.zeros(B, Tp, dtype=torch.int64)
    inten = torch.zeros(B, Tp, n_emo, dtype=torch.float32)
    for i, (p, it) in enumerate(zip(phonemes, intensities)):
        L = int(p.numel())
        tok[i, :L] = p.reshape(-1).long()
        inten[i, :L] = it.reshape(-1, n_emo)[:L].float()
    spk = torch.as_tensor(speakers, dtype=torch.int64).reshape(B)
    out = model(tok.to(dev), spk.to(dev), intensity=inten.to(dev), pace=pace)
    mel, mel_lens = out[0], out[7]
    lens = [int(x) for x in mel_lens.tolist()]
    return [mel[i, :lens[i]] for i in range(B)], lens


def intensity_sweep_batch(phoneme, n_speakers, emotions, levels, intensity_bank, n_emotions=5):
    """The reference sweep's inputs (inference.py:55-89) for one sentence as batch lists:
    every (speaker, emotion, level) combination, in the reference's loop order."""
    T = int(phoneme.numel())
    ph, spk, inten, keys = [], [], [], []
    for s in range(n_speakers):
        for e in emotions:
            for lv in levels:
                ph.append(phoneme)
                spk.append(s)
                inten.append(get_intensity_rep(s, e, lv, T, intensity_bank, n_emotions)[0])
                keys.append((s, e, lv))
    return ph, spk, inten, keys


@torch.no_grad()
def vocode(vocoder, mels, n_mels=80):
    """Waveforms for ``synthesize``'s mels: the list is zero-padded to its longest mel into ONE
    (B, n_mels, T_max) batch -- the padded ``model(...)[0].permute(0, 2, 1)`` the reference
    hands to ``vocoder.decode_batch`` (inference.py:82-83) -- and decoded by ``vocoder`` (a
    ``fastspeech2.vocoder.HifiganGenerator``).  Returns (wav (B, 1, hop * (T_max + 10)),
    per-sentence valid sample counts hop * T_i)."""
    dev = next(vocoder.parameters()).device
    B = len(mels)
    T = max(1, max(int(m.shape[0]) for m in mels))
    batch = torch.zeros(B, n_mels, T, dtype=torch.float32, device=dev)
    for i, m in enumerate(mels):
        if m.shape[0]:
            batch[i, :, :m.shape[0]] = m.to(device=dev, dtype=torch.float32).t()
    wav = vocoder.decode_batch(batch)
    hop = wav.shape[-1] // (T + 2 * vocoder.hp["inference_padding"])
    return wav, [hop * int(m.shape[0]) for m in mels]
