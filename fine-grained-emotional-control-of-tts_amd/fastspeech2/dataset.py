"""Input format and batch collate: the reference's FastSpeech2Dataset item layout
and TextMelCollateWithAlignment, with the padding / sorting / rank_X assembly done on the GPU.

Reference: emo_rank_tts/fastspeech2/dataset.py
* ``FastSpeech2Dataset`` -- :11-58: one ``.npz`` per utterance listed in ``fs2_{mode}.txt``
  with keys mel (n_mels, T), pitch (T), energy (T), durations (T_phon), phones (T_phon strings),
  speaker, emotion, transcript, audio_path;
* ``TextMelCollateWithAlignment`` -- :62-133: sort by phoneme length (descending), zero-pad
  phonemes / durations (B, Tp), mel (B, n_mels, Tm) returned as ``permute(0, 2, 1)``, pitch /
  energy (B, Tm), rank_X (B, n_mels + 2, Tm) = cat(mel, pitch, energy), lengths, speakers,
  emotions, labels, wav paths.
* ``phoneme2sequence`` -- fastspeech2/util.py:11-12,30-32: index into
  ['@'] + speechbrain's ARPAbet ``valid_symbols`` + ['sil', 'spn', 'sp', ''].

``GpuCollate`` keeps the reference's call signature and 12-tuple.  The host only computes the
sort order (the same ``torch.sort`` call as the reference, so ties resolve identically) and
concatenates the items into packed buffers; one upload, then ``fs2_collate_phonemes`` /
``fs2_collate_frames`` write every padded tensor on the device.  ``mel`` comes back contiguous
(B, Tm, n_mels) (the reference's is a permuted view with the same values).

The .npz files are read with ``allow_pickle=False`` (the reference passes True); string fields
are stored by numpy as unicode arrays and load without pickling.
"""

import os

import numpy as np
import torch

from . import _native as N
from . import ops

# speechbrain.utils.text_to_sequence.valid_symbols (the CMUdict ARPAbet set of keithito's
# tacotron, 84 symbols), as util.py:12 builds VALID_TOKENS from it
_ARPABET = [
    "AA", "AA0", "AA1", "AA2", "AE", "AE0", "AE1", "AE2", "AH", "AH0", "AH1", "AH2", "AO",
    "AO0", "AO1", "AO2", "AW", "AW0", "AW1", "AW2", "AY", "AY0", "AY1", "AY2", "B", "CH", "D",
    "DH", "EH", "EH0", "EH1", "EH2", "ER", "ER0", "ER1", "ER2", "EY", "EY0", "EY1", "EY2", "F",
    "G", "HH", "IH", "IH0", "IH1", "IH2", "IY", "IY0", "IY1", "IY2", "JH", "K", "L", "M", "N",
    "NG", "OW", "OW0", "OW1", "OW2", "OY", "OY0", "OY1", "OY2", "P", "R", "S", "SH", "T", "TH",
    "UH", "UH0", "UH1", "UH2", "UW", "UW0", "UW1", "UW2", "V", "W", "Y", "Z", "ZH"]
SIL_PHONES = ["sil", "spn", "sp", ""]
VALID_TOKENS = ["@"] + _ARPABET + SIL_PHONES


def phoneme2sequence(phoneme):
    """util.py:30-32."""
    return [VALID_TOKENS.index(token) for token in phoneme]


def load_item(data_path, noise_symbol, speakers, emotions):
    """FastSpeech2Dataset.__getitem__ (dataset.py:28-58) for one .npz path."""
    data = np.load(data_path, allow_pickle=False)
    text = str(data["transcript"].item()).replace(noise_symbol.strip(), "").strip()
    return {
        "mel": torch.FloatTensor(data["mel"]),
        "pitch": torch.FloatTensor(data["pitch"]),
        "energy": torch.FloatTensor(data["energy"]),
        "duration": torch.LongTensor(data["durations"]),
        "phoneme": torch.LongTensor(phoneme2sequence([str(p) for p in data["phones"].tolist()])),
        "speaker": torch.tensor(speakers.index(str(data["speaker"].item())), dtype=torch.long),
        "emotion": torch.tensor(emotions.index(str(data["emotion"].item())), dtype=torch.long),
        "text": text,
        "audio_path": str(data["audio_path"].item()),
    }


class FastSpeech2Dataset(torch.utils.data.Dataset):
    """dataset.py:11-58 (same constructor and item dict)."""

    def __init__(self, preprocessed_path, noise_symbol, speakers, emotions, mode="train"):
        super().__init__()
        self.preprocessed_path = preprocessed_path
        self.noise_symbol = noise_symbol
        self.speakers = speakers
        self.emotions = emotions
        with open(os.path.join(preprocessed_path, f"fs2_{mode}.txt")) as f:
            self.data_paths = [line.strip() for line in f.readlines()]

    def __len__(self):
        return len(self.data_paths)

    def __getitem__(self, idx):
        return load_item(self.data_paths[idx], self.noise_symbol, self.speakers, self.emotions)


class GpuCollate:
    """Drop-in for TextMelCollateWithAlignment (dataset.py:62-133) producing device tensors."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)

    def __call__(self, batch):
        N.load()
        B = len(batch)
        input_lengths, ids_sorted_decreasing = torch.sort(
            torch.LongTensor([len(x["phoneme"]) for x in batch]), dim=0, descending=True)
        Tp = int(input_lengths[0])
        n_mels = batch[0]["mel"].size(0)
        frames = [int(x["mel"].size(1)) for x in batch]
        Tm = max(frames)
        poff = np.zeros(B + 1, dtype=np.int64)
        poff[1:] = np.cumsum([len(x["phoneme"]) for x in batch])
        foff = np.zeros(B + 1, dtype=np.int64)
        foff[1:] = np.cumsum(frames)
        # one packed host buffer per dtype -> one upload each
        ints = torch.cat([ids_sorted_decreasing.to(torch.int64), torch.from_numpy(poff),
                          torch.from_numpy(foff)] + [x["phoneme"].long() for x in batch]
                         + [x["duration"].long() for x in batch])
        flts = torch.cat([x["mel"].float().reshape(-1) for x in batch]
                         + [x["pitch"].float().reshape(-1) for x in batch]
                         + [x["energy"].float().reshape(-1) for x in batch])
        pin = self.device.type == "cuda"
        ints_d = (ints.pin_memory() if pin else ints).to(self.device, non_blocking=True)
        flts_d = (flts.pin_memory() if pin else flts).to(self.device, non_blocking=True)
        order = ints_d[:B].to(torch.int32)
        poff_d = ints_d[B:2 * B + 1]
        foff_d = ints_d[2 * B + 1:3 * B + 2]
        nph = int(poff[-1])
        phon_d = ints_d[3 * B + 2:3 * B + 2 + nph]
        dur_d = ints_d[3 * B + 2 + nph:3 * B + 2 + 2 * nph]
        nfr = int(foff[-1])
        mel_d = flts_d[:nfr * n_mels]
        pitch_d = flts_d[nfr * n_mels:nfr * (n_mels + 1)]
        energy_d = flts_d[nfr * (n_mels + 1):]
        dev = self.device
        phoneme_padded = torch.empty(B, Tp, dtype=torch.int64, device=dev)
        duration_padded = torch.empty(B, Tp, dtype=torch.int64, device=dev)
        in_len = torch.empty(B, dtype=torch.int64, device=dev)
        ops.collate_phonemes(order, poff_d, phon_d, dur_d, B, Tp, phoneme_padded,
                             duration_padded, in_len)
        mel_padded = torch.empty(B, Tm, n_mels, dtype=torch.float32, device=dev)
        pitch_padded = torch.empty(B, Tm, dtype=torch.float32, device=dev)
        energy_padded = torch.empty(B, Tm, dtype=torch.float32, device=dev)
        rank_x = torch.empty(B, n_mels + 2, Tm, dtype=torch.float32, device=dev)
        out_len = torch.empty(B, dtype=torch.int64, device=dev)
        ops.collate_frames(order, foff_d, mel_d, pitch_d, energy_d, B, Tm, n_mels, mel_padded,
                           pitch_padded, energy_padded, rank_x, out_len)
        idx = ids_sorted_decreasing.tolist()
        speakers = torch.LongTensor([int(batch[i]["speaker"]) for i in idx]).to(dev)
        emotions = torch.LongTensor([int(batch[i]["emotion"]) for i in idx]).to(dev)
        labels = [batch[i]["text"] for i in idx]
        wavs = [batch[i]["audio_path"] for i in idx]
        return (phoneme_padded, speakers, in_len, mel_padded, pitch_padded, energy_padded,
                duration_padded, out_len, labels, wavs, rank_x, emotions)
