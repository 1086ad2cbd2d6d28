"""CPU oracle for the frozen IntensityExtractor forward and the phoneme averaging of the
FastSpeech2 train step.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this file; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker.

What it restates (op for op, PyTorch-CPU fp32, written out without nn.MultiheadAttention /
nn.TransformerEncoder so that it is an independent statement of the algorithm):

* ``IntensityExtractor.forward``  -- /root/reference/emo_rank_tts/rank_model/model.py:96-109
  (mask :84-93, input projection :100, FFT block :101 = nn.TransformerEncoder over
  ``ConvTransformerEncoderLayer`` :32-50, emotion embedding add :103-104, masked_fill :106,
  classifier :107);
* ``get_intensity_representation``  -- /root/reference/emo_rank_tts/fastspeech2/train.py:16-51
  (per-utterance ``repeat_interleave`` + ``index_add_`` segment sum, ``/ clamp(d, 1)``;
  ``oracle.fs2_oracle.phoneme_average_intensity``), with the reference's ``rank_X`` layout
  defect fixed explicitly: the collate builds ``(B, 82, T)``
  (fastspeech2/dataset.py:94,116-117) while the extractor reads ``(B, T, 82)``
  (rank_model/model.py:86,100); ``layout="BCT"`` transposes first.

Parity status: **pinned**.  ``rank_model/model.py`` imports and runs in the dev container
(torch only), so ``tests/golden/make_golden_intensity.py`` runs the real reference module on
seeded weights and inputs and commits the outputs (``tests/golden/intensity_ref.npz``);
``tests/test_oracle.py`` checks this restatement against them.  The averaging step lives in
``fastspeech2/train.py``, which cannot be imported (speechbrain, tensorboard), so its expected
values come from two independent restatements of train.py:33-49 (the torch one in
fs2_oracle.py and the numpy loop ``phoneme_average_np`` below).
"""

import math

import numpy as np
import torch
import torch.nn.functional as F

from .fs2_oracle import phoneme_average_intensity  # noqa: F401  (train.py:16-51)


def prepare_mask(length, T):
    """rank_model/model.py:84-93: True at padded frames (t >= length[b])."""
    return torch.arange(T).unsqueeze(0).expand(length.shape[0], T) >= length.unsqueeze(1)


def _mha(x, key_pad, in_w, in_b, out_w, out_b, n_heads):
    """torch nn.MultiheadAttention(batch_first=True) eval forward with key_padding_mask only
    (rank_model/model.py:20,35): packed in-projection, per-head softmax(QK^T/sqrt(dh)) with
    padded keys at -inf, PV, out-projection."""
    B, T, D = x.shape
    dh = D // n_heads
    qkv = x @ in_w.t() + in_b
    q, k, v = qkv.split(D, dim=-1)
    q = q.reshape(B, T, n_heads, dh).transpose(1, 2)
    k = k.reshape(B, T, n_heads, dh).transpose(1, 2)
    v = v.reshape(B, T, n_heads, dh).transpose(1, 2)
    s = (q / math.sqrt(dh)) @ k.transpose(-1, -2)
    s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = (p @ v).transpose(1, 2).reshape(B, T, D)
    return o @ out_w.t() + out_b


def _conv_same_zero(x, w, b):
    """nn.Conv1d(padding=k//2) (zero padding) over (B, T, C) -> (B, T, O)."""
    k = w.shape[-1]
    return F.conv1d(x.transpose(1, 2), w, b, padding=k // 2).transpose(1, 2)


def extractor_forward(sd, x, length, emotions, n_heads, n_layers, layout="BTC"):
    """IntensityExtractor forward (rank_model/model.py:96-109) from a state dict with the
    reference's keys; x (B, T, n_mels+2) or, with layout="BCT", the collate's (B, n_mels+2, T).
    Returns I (B, T, n_emotions), fp32.  Eval mode: dropout is identity."""
    x = x.float()
    if layout == "BCT":
        x = x.transpose(1, 2)
    B, T, _ = x.shape
    g = lambda k: sd[k].float()
    mask = prepare_mask(length.cpu(), T)
    h = x @ g("input_proj.weight").t() + g("input_proj.bias")
    D = h.shape[-1]
    for i in range(n_layers):
        p = f"fft_block.layers.{i}."
        a = _mha(h, mask, g(p + "self_attn.in_proj_weight"), g(p + "self_attn.in_proj_bias"),
                 g(p + "self_attn.out_proj.weight"), g(p + "self_attn.out_proj.bias"), n_heads)
        h = F.layer_norm(h + a, (D,), g(p + "norm1.weight"), g(p + "norm1.bias"), 1e-5)
        y = F.gelu(_conv_same_zero(h, g(p + "conv1.weight"), g(p + "conv1.bias")))
        y = _conv_same_zero(y, g(p + "conv2.weight"), g(p + "conv2.bias"))
        h = F.layer_norm(h + y, (D,), g(p + "norm2.weight"), g(p + "norm2.bias"), 1e-5)
    i_ = h + g("emotion_embedding.weight")[emotions.long()].unsqueeze(1)
    i_ = i_.masked_fill(mask.unsqueeze(-1), 0.0)
    return i_ @ g("classifier.weight").t() + g("classifier.bias")


def phoneme_average_np(I, durations, phon_len):
    """train.py:29-51 in plain numpy loops (fp64 sums): the frames of phoneme p are
    [sum(d[:p]), sum(d[:p+1])), divided by clamp(d, 1); zeros past phon_len."""
    I = np.asarray(I, dtype=np.float64)
    durations = np.asarray(durations)
    B, Tp = durations.shape
    out = np.zeros((B, Tp, I.shape[-1]), dtype=np.float64)
    for b in range(B):
        t = 0
        for p in range(int(phon_len[b])):
            d = int(durations[b, p])
            if d > 0:
                out[b, p] = I[b, t:t + d].sum(0) / d
            t += d
    return out.astype(np.float32)


def extractor_flops_per_frame(hidden, n_layers, kernel, T, n_in=82, n_emo=5):
    """Algorithmic forward FLOPs per frame at padded length T: input projection, per layer
    QKV + out-projection (8 D^2), scores + context (4 T D), the two k-tap convs
    (2 * 2 k D 4D); classifier."""
    D, F4 = hidden, 4 * hidden
    per_layer = 8 * D * D + 4 * T * D + 2 * 2 * kernel * D * F4
    return 2 * n_in * D + n_layers * per_layer + 2 * D * n_emo
