"""CPU oracle for the batch collate.  TEST INFRASTRUCTURE ONLY: used by tests/
as the checker, never by the product package.

Restates TextMelCollateWithAlignment (/root/reference/emo_rank_tts/fastspeech2/dataset.py:62-133)
in numpy: order = torch.sort(phoneme lengths, descending) (:64-66, the same call, so ties
resolve identically); zero-padded phoneme / duration (:72-80), mel (:88-89,106 then the
permute at :119), pitch / energy (:90-93,107-108), rank_X = cat(mel, pitch, energy) (:94-95,
116-117), output lengths = mel frames (:109), speakers / emotions / labels / wavs in sorted order.
Pinned by tests/golden/collate_ref.npz (the reference class run on seeded items,
make_golden_collate.py) in tests/test_oracle.py.
"""
import numpy as np
import torch


def collate_np(batch):
    lens, order = torch.sort(torch.LongTensor([len(x["phoneme"]) for x in batch]), dim=0,
                             descending=True)
    order = order.tolist()
    B, Tp = len(batch), int(lens[0])
    n_mels = batch[0]["mel"].shape[0]
    Tm = max(int(x["mel"].shape[1]) for x in batch)
    ph = np.zeros((B, Tp), np.int64)
    du = np.zeros((B, Tp), np.int64)
    mel = np.zeros((B, n_mels, Tm), np.float32)
    pitch = np.zeros((B, Tm), np.float32)
    energy = np.zeros((B, Tm), np.float32)
    rank = np.zeros((B, n_mels + 2, Tm), np.float32)
    out_len = np.zeros(B, np.int64)
    for i, u in enumerate(order):
        it = batch[u]
        p = np.asarray(it["phoneme"])
        ph[i, :len(p)] = p
        d = np.asarray(it["duration"])
        du[i, :len(d)] = d
        m = np.asarray(it["mel"], np.float32)
        T = m.shape[1]
        mel[i, :, :T] = m
        pitch[i, :len(it["pitch"])] = np.asarray(it["pitch"])
        energy[i, :len(it["energy"])] = np.asarray(it["energy"])
        out_len[i] = T
        rank[i, :, :T] = np.concatenate([m, np.asarray(it["pitch"])[None],
                                         np.asarray(it["energy"])[None]], 0)
    return {"phoneme": ph, "speakers": np.array([int(batch[u]["speaker"]) for u in order]),
            "input_lengths": lens.numpy(), "mel": mel.transpose(0, 2, 1), "pitch": pitch,
            "energy": energy, "duration": du, "output_lengths": out_len,
            "labels": [batch[u]["text"] for u in order],
            "wavs": [batch[u]["audio_path"] for u in order], "rank_X": rank,
            "emotions": np.array([int(batch[u]["emotion"]) for u in order])}


def items_from_golden(z):
    """The golden fixture's input items as the dataset's item dicts."""
    out = []
    for i in range(int(z["n_items"])):
        it = {k: torch.from_numpy(z[f"in{i}_{k}"]) for k in
              ("mel", "pitch", "energy", "duration", "phoneme", "speaker", "emotion")}
        it["text"] = str(z[f"in{i}_text"])
        it["audio_path"] = str(z[f"in{i}_audio_path"])
        out.append(it)
    return out
