"""Drop-in ``Loss`` (emo_rank_tts/fastspeech2/loss.py:6-186) on the fused HIP loss kernel.

``Loss(**config['loss'])(predictions, targets, current_epoch)`` returns the same dict of
seven scalars as the reference (loss.py:176-186).  Forward and the gradient of
``total_loss`` are computed together by ``fs2_loss_fwd_bwd`` (per-utterance masked MSE
terms, log1p duration targets, the [:mel_len]-on-phoneme-axis pitch/energy slicing, SB
SSIM with masked min-max normalisation and [0,1] clamp); ``backward`` only scales the
stored gradients by the upstream gradient.  Only ``total_loss`` is differentiable, which is
what the reference train step uses (train.py:80).
"""

import torch
import torch.nn as nn

from . import _native as N
from . import ops

LOSS_KEYS = ("total_loss", "ssim_loss", "mel_loss", "postnet_mel_loss", "dur_loss",
             "pitch_loss", "energy_loss")


def fused_loss(mel_out, postnet_out, log_dur, pitch_pred, energy_pred, mel_tgt, dur_tgt,
               pitch_avg, energy_avg, mel_len, phon_len, weights, need_grads=True):
    """Run fs2_loss_fwd_bwd.  Returns (loss_vec[8] fp32 device tensor, grads tuple)."""
    B, Tm, NM = mel_out.shape
    Tp = log_dur.shape[1]
    dt = N.dtype_code(mel_out.dtype)
    if mel_tgt.shape[1] != Tm:
        raise ValueError(f"mel target frames {mel_tgt.shape[1]} != predicted frames {Tm}; the "
                         f"reference SSIM needs equal lengths (durations must sum to mel length)")
    dev = mel_out.device
    d = N.LossDesc()
    d.B, d.Tm, d.Tp, d.NM, d.dtype = B, Tm, Tp, NM, dt
    keep = []

    def c(t, dtype=None):
        t = t.to(device=dev, dtype=dtype or t.dtype).contiguous()
        keep.append(t)
        return t.data_ptr()

    d.mel_out, d.postnet_out = c(mel_out), c(postnet_out)
    d.log_dur, d.pitch_pred, d.energy_pred = c(log_dur), c(pitch_pred), c(energy_pred)
    d.mel_tgt = c(mel_tgt, torch.float32)
    d.dur_tgt = c(dur_tgt, torch.int64)
    d.pitch_avg, d.energy_avg = c(pitch_avg, torch.float32), c(energy_avg, torch.float32)
    d.mel_len, d.phon_len = c(mel_len, torch.int64), c(phon_len, torch.int64)
    (d.w_ssim, d.w_mel, d.w_post, d.w_dur, d.w_pitch, d.w_energy) = weights
    loss = torch.empty(8, dtype=torch.float32, device=dev)
    g_mel = torch.empty_like(mel_out)
    g_post = torch.empty_like(mel_out)
    g_dur = torch.empty(B, Tp, dtype=mel_out.dtype, device=dev)
    g_pitch = torch.empty(B, Tp, dtype=mel_out.dtype, device=dev)
    g_energy = torch.empty(B, Tp, dtype=mel_out.dtype, device=dev)
    ws = torch.empty(int(ops.loss_ws(B, Tm, NM)) + 64, dtype=torch.float32, device=dev)
    d.loss_out = loss.data_ptr()
    d.d_mel_out, d.d_postnet_out = g_mel.data_ptr(), g_post.data_ptr()
    d.d_log_dur, d.d_pitch, d.d_energy = g_dur.data_ptr(), g_pitch.data_ptr(), g_energy.data_ptr()
    d.workspace = ws.data_ptr()
    ops.loss_fwd_bwd(d)
    return loss, (g_mel, g_post, g_dur, g_pitch, g_energy)


class _LossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mel_out, postnet_out, log_dur, pitch_pred, energy_pred, mel_tgt, dur_tgt,
                pitch_avg, energy_avg, mel_len, phon_len, weights):
        loss, grads = fused_loss(mel_out, postnet_out, log_dur, pitch_pred.squeeze(-1),
                                 energy_pred.squeeze(-1), mel_tgt, dur_tgt,
                                 pitch_avg.squeeze(-1), energy_avg.squeeze(-1), mel_len, phon_len,
                                 weights)
        ctx.grads = grads
        ctx.pshape = pitch_pred.shape
        ctx.set_materialize_grads(False)
        return tuple(loss[i] for i in range(7))

    @staticmethod
    def backward(ctx, g_total, *g_parts):
        if any(g is not None for g in g_parts):
            raise NotImplementedError("only total_loss is differentiable (train.py:80)")
        g_mel, g_post, g_dur, g_pitch, g_energy = ctx.grads
        ctx.grads = None
        if g_total is None:
            return (None,) * 12
        s = g_total.to(g_mel.dtype)
        return (g_mel * s, g_post * s, g_dur * s, (g_pitch * s).view(ctx.pshape),
                (g_energy * s).view(ctx.pshape), None, None, None, None, None, None, None)


class Loss(nn.Module):
    """loss.py:Loss -- same constructor and output dict."""

    def __init__(self, log_scale_durations, ssim_loss_weight, duration_loss_weight,
                 pitch_loss_weight, energy_loss_weight, mel_loss_weight, postnet_mel_loss_weight,
                 spn_loss_weight=1.0, spn_loss_max_epochs=8):
        super().__init__()
        if not log_scale_durations:
            raise NotImplementedError("reference trains with log_scale_durations=True "
                                      "(parameter.yaml:97); loss.py:108-124 is undefined otherwise")
        self.log_scale_durations = log_scale_durations
        self.ssim_loss_weight = ssim_loss_weight
        self.mel_loss_weight = mel_loss_weight
        self.postnet_mel_loss_weight = postnet_mel_loss_weight
        self.duration_loss_weight = duration_loss_weight
        self.pitch_loss_weight = pitch_loss_weight
        self.energy_loss_weight = energy_loss_weight
        self.spn_loss_weight = spn_loss_weight
        self.spn_loss_max_epochs = spn_loss_max_epochs

    @property
    def weights(self):
        return (float(self.ssim_loss_weight), float(self.mel_loss_weight),
                float(self.postnet_mel_loss_weight), float(self.duration_loss_weight),
                float(self.pitch_loss_weight), float(self.energy_loss_weight))

    def forward(self, predictions, targets, current_epoch):
        mel_target, target_durations, target_pitch, target_energy, mel_length, phon_len = targets
        assert len(mel_target.shape) == 3
        (mel_out, postnet_mel_out, log_durations, predicted_pitch, average_pitch,
         predicted_energy, average_energy, mel_lens) = predictions
        vals = _LossFunction.apply(mel_out, postnet_mel_out, log_durations, predicted_pitch,
                                   predicted_energy, mel_target, target_durations, average_pitch,
                                   average_energy, mel_length, phon_len, self.weights)
        return dict(zip(LOSS_KEYS, vals))
