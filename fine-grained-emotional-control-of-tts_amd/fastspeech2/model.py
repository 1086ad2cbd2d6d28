"""Drop-in ``FastSpeech2`` (emo_rank_tts/fastspeech2/model.py:32-441) on MI355X kernels.

Same constructor arguments (``FastSpeech2(**config['model']['fastspeech2'], n_speakers=N)``,
train.py:214), same ``forward`` signature and 8-tuple (model.py:279-441), same state_dict
keys as the speechbrain-based reference, so reference checkpoints load
with ``load_state_dict``.  The submodules below are parameter containers only: they mirror
the speechbrain lobes' attribute names and torch's default initialisation, but the forward
pass is the hand-written engine (``engine.FS2Engine``) over libfs2_hip.so.

Parameters live in ONE flat fp32 device buffer (``_flat``), gradients in another (``_gflat``),
both laid out in backward-completion order (PostNet -> decoder -> variance adaptor ->
conditioning -> encoder -> prenet) so data-parallel buckets are contiguous and can be
all-reduced while the rest of the backward is still running.
"""

import math
from dataclasses import dataclass, fields

import torch
import torch.nn as nn

# --------------------------------------------------------------------------- containers


class _Linear(nn.Module):            # speechbrain.nnet.linear.Linear  (.w)
    def __init__(self, n_neurons, input_size, bias=True):
        super().__init__()
        self.w = nn.Linear(input_size, n_neurons, bias=bias)


class _Embedding(nn.Module):         # speechbrain.nnet.embedding.Embedding  (.Embedding)
    def __init__(self, num_embeddings, embedding_dim):
        super().__init__()
        self.Embedding = nn.Embedding(num_embeddings, embedding_dim)


class _Conv1d(nn.Module):            # speechbrain.nnet.CNN.Conv1d  (.conv), reflect "same"
    def __init__(self, in_channels, out_channels, kernel_size):
        super().__init__()
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size)


class _LayerNorm(nn.Module):         # speechbrain.nnet.normalization.LayerNorm  (.norm)
    def __init__(self, size, eps=1e-5):
        super().__init__()
        self.norm = nn.LayerNorm(size, eps=eps)


class _MHA(nn.Module):               # speechbrain.nnet.attention.MultiheadAttention  (.att)
    def __init__(self, nhead, d_model, dropout, kdim, vdim):
        super().__init__()
        self.att = nn.MultiheadAttention(d_model, nhead, dropout=dropout, kdim=kdim, vdim=vdim)


class _FFTLayer(nn.Module):          # SB TransformerEncoderLayer(ffn_type='1dcnn')
    def __init__(self, d_ffn, nhead, d_model, kdim, vdim, dropout, ks):
        super().__init__()
        self.self_att = _MHA(nhead, d_model, dropout, kdim, vdim)
        self.pos_ffn = nn.Sequential(_Conv1d(d_model, d_ffn, ks[0]), nn.ReLU(),
                                     _Conv1d(d_ffn, d_model, ks[1]))
        self.norm1 = _LayerNorm(d_model, eps=1e-6)
        self.norm2 = _LayerNorm(d_model, eps=1e-6)


class _FFTStack(nn.Module):          # SB TransformerEncoder
    def __init__(self, num_layers, nhead, d_ffn, d_model, kdim, vdim, dropout, ks):
        super().__init__()
        self.layers = nn.ModuleList([_FFTLayer(d_ffn, nhead, d_model, kdim, vdim, dropout, ks)
                                     for _ in range(num_layers)])
        self.norm = _LayerNorm(d_model, eps=1e-6)


class _PositionalEncoding(nn.Module):  # SB PositionalEncoding(input_size, max_len=2500)
    def __init__(self, input_size, max_len=2500):
        super().__init__()
        pe = torch.zeros(max_len, input_size)
        positions = torch.arange(0, max_len).unsqueeze(1).float()
        denominator = torch.exp(torch.arange(0, input_size, 2).float()
                                * -(math.log(10000.0) / input_size))
        pe[:, 0::2] = torch.sin(positions * denominator)
        pe[:, 1::2] = torch.cos(positions * denominator)
        self.register_buffer("pe", pe.unsqueeze(0))


class _EncoderPreNet(nn.Module):     # SB EncoderPreNet (.token_embedding)
    def __init__(self, n_vocab, out_channels):
        super().__init__()
        self.token_embedding = _Embedding(n_vocab, out_channels)


class _DurationPredictor(nn.Module):  # SB DurationPredictor
    def __init__(self, channels, kernel_size):
        super().__init__()
        self.conv1 = _Conv1d(channels, channels, kernel_size)
        self.conv2 = _Conv1d(channels, channels, kernel_size)
        self.linear = _Linear(1, channels)
        self.ln1 = _LayerNorm(channels)
        self.ln2 = _LayerNorm(channels)


class _PostNet(nn.Module):           # SB PostNet
    def __init__(self, n_mels, dim, k, n_conv):
        super().__init__()
        self.conv_pre = _Conv1d(n_mels, dim, k)
        self.convs_intermedite = nn.ModuleList([_Conv1d(dim, dim, k) for _ in range(1, n_conv - 1)])
        self.conv_post = _Conv1d(dim, n_mels, k)
        self.ln1 = nn.LayerNorm(dim)
        self.ln2 = nn.LayerNorm(dim)
        self.ln3 = nn.LayerNorm(n_mels)


@dataclass
class FS2Config:
    enc_num_layers: int
    enc_num_head: int
    enc_d_model: int
    enc_ffn_dim: int
    enc_k_dim: int
    enc_v_dim: int
    enc_dropout: float
    dec_num_layers: int
    dec_num_head: int
    dec_d_model: int
    dec_ffn_dim: int
    dec_k_dim: int
    dec_v_dim: int
    dec_dropout: float
    normalize_before: bool
    ffn_type: str
    ffn_cnn_kernel_size_list: list
    n_char: int
    n_mels: int
    postnet_embedding_dim: int
    postnet_kernel_size: int
    postnet_n_convolutions: int
    postnet_dropout: float
    padding_idx: int
    dur_pred_kernel_size: int
    pitch_pred_kernel_size: int
    energy_pred_kernel_size: int
    variance_predictor_dropout: float
    n_speakers: int


def _group_key(name, n_dec, n_enc):
    """(group, order within group, layer) -- sorts parameters into backward-completion order."""
    if name.startswith("postnet."):
        return (0, 0, 0)
    if name.startswith("linear.") or name.startswith("decoder.norm."):
        return (1, 0, 0)
    if name.startswith("decoder.layers."):
        i = int(name.split(".")[2])
        return (2, n_dec - 1 - i, i)
    if name.split(".")[0] in ("energyEmbed", "energyPred", "pitchEmbed", "pitchPred", "durPred"):
        # the duration / pitch predictors' conv1 weights, then their biases, adjacent: the
        # engine runs the two conv1 layers (same input, model.py:366,379) as ONE conv with
        # 2 x 384 output channels over the contiguous [2O][KW][C] weights and [2O] biases
        sub = {"durPred.conv1.conv.weight": 0, "pitchPred.conv1.conv.weight": 1,
               "durPred.conv1.conv.bias": 2, "pitchPred.conv1.conv.bias": 3}.get(name, 4)
        return (3, sub, 0)
    if name.split(".")[0] in ("concat_proj", "speaker_emb") or name.startswith("encoder.norm."):
        return (4, 0, 0)
    if name.startswith("encoder.layers."):
        i = int(name.split(".")[2])
        return (5, n_enc - 1 - i, i)
    return (6, 0, 0)  # encPreNet


def _kw_major(name, shape):
    """Conv weights (O, C, KW>1) live in the flat buffer as [O][KW][C]."""
    return len(shape) == 3 and shape[2] > 1 and name.endswith("conv.weight")


def group_tag(key):
    g, _, layer = key
    return {0: "postnet", 1: "linear", 3: "variance", 4: "conditioning", 6: "prenet"}.get(
        g, None) or (f"decoder.layers.{layer}" if g == 2 else f"encoder.layers.{layer}")


class FastSpeech2(nn.Module):
    """emo_rank_tts/fastspeech2/model.py:FastSpeech2, MI355X-native."""

    def __init__(self, enc_num_layers, enc_num_head, enc_d_model, enc_ffn_dim, enc_k_dim,
                 enc_v_dim, enc_dropout, dec_num_layers, dec_num_head, dec_d_model, dec_ffn_dim,
                 dec_k_dim, dec_v_dim, dec_dropout, normalize_before, ffn_type,
                 ffn_cnn_kernel_size_list, n_char, n_mels, postnet_embedding_dim,
                 postnet_kernel_size, postnet_n_convolutions, postnet_dropout, padding_idx,
                 dur_pred_kernel_size, pitch_pred_kernel_size, energy_pred_kernel_size,
                 variance_predictor_dropout, n_speakers, act_dtype=torch.float32):
        super().__init__()
        self.cfg = FS2Config(**{f.name: v for f, v in zip(fields(FS2Config), [
            enc_num_layers, enc_num_head, enc_d_model, enc_ffn_dim, enc_k_dim, enc_v_dim,
            enc_dropout, dec_num_layers, dec_num_head, dec_d_model, dec_ffn_dim, dec_k_dim,
            dec_v_dim, dec_dropout, normalize_before, ffn_type, list(ffn_cnn_kernel_size_list),
            n_char, n_mels, postnet_embedding_dim, postnet_kernel_size, postnet_n_convolutions,
            postnet_dropout, padding_idx, dur_pred_kernel_size, pitch_pred_kernel_size,
            energy_pred_kernel_size, variance_predictor_dropout, n_speakers])})
        if normalize_before or ffn_type != "1dcnn":
            raise NotImplementedError("reference config is post-LN with ffn_type='1dcnn'")
        if enc_d_model != dec_d_model or enc_k_dim != enc_d_model or enc_v_dim != enc_d_model:
            raise ValueError("encoder/decoder widths must match (model.py:406-423)")
        self.enc_num_head = enc_num_head
        self.dec_num_head = dec_num_head
        self.padding_idx = padding_idx
        self.act_dtype = act_dtype
        # same construction order as model.py:187-276 -> identical state_dict order
        self.sinusoidal_positional_embed_encoder = _PositionalEncoding(enc_d_model)
        self.sinusoidal_positional_embed_decoder = _PositionalEncoding(dec_d_model)
        self.speaker_emb = _Embedding(n_speakers, enc_d_model)
        self.concat_proj = _Linear(enc_d_model, enc_d_model + enc_d_model + 5, bias=False)
        self.encPreNet = _EncoderPreNet(n_char, enc_d_model)
        self.durPred = _DurationPredictor(enc_d_model, dur_pred_kernel_size)
        self.pitchPred = _DurationPredictor(enc_d_model, dur_pred_kernel_size)
        self.energyPred = _DurationPredictor(enc_d_model, dur_pred_kernel_size)
        self.pitchEmbed = _Conv1d(1, enc_d_model, pitch_pred_kernel_size)
        self.energyEmbed = _Conv1d(1, enc_d_model, energy_pred_kernel_size)
        self.encoder = _FFTStack(enc_num_layers, enc_num_head, enc_ffn_dim, enc_d_model, enc_k_dim,
                                 enc_v_dim, enc_dropout, ffn_cnn_kernel_size_list)
        self.decoder = _FFTStack(dec_num_layers, dec_num_head, dec_ffn_dim, dec_d_model, dec_k_dim,
                                 dec_v_dim, dec_dropout, ffn_cnn_kernel_size_list)
        self.linear = _Linear(n_mels, dec_d_model)
        self.postnet = _PostNet(n_mels, postnet_embedding_dim, postnet_kernel_size,
                                postnet_n_convolutions)
        self._flat = None
        self._gflat = None
        self._grad_views = {}
        self._layout = []          # (name, offset, numel, shape, group_key)
        self._param_version = 0
        self._engine = None
        self._step_seed = 1234

    # ------------------------------------------------------------------ flat buffers
    def _ensure_packed(self):
        params = dict(self.named_parameters())
        if self._flat is not None:
            ok = all(params[n].data_ptr() == self._flat.data_ptr() + 4 * off
                     for n, off, _, _, _ in self._layout)
            if ok:
                return
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("FastSpeech2 (MI355X) runs on a HIP device: call .cuda() first")
        c = self.cfg
        order = sorted(params.keys(), key=lambda n: _group_key(n, c.dec_num_layers, c.enc_num_layers))
        layout, off = [], 0
        for n in order:
            p = params[n]
            layout.append((n, off, p.numel(), tuple(p.shape),
                           _group_key(n, c.dec_num_layers, c.enc_num_layers)))
            off += (p.numel() + 15) // 16 * 16
        flat = torch.zeros(off, dtype=torch.float32, device=dev)
        gflat = torch.zeros(off, dtype=torch.float32, device=dev)
        views = {}
        for n, o, k, shape, _ in layout:
            p = params[n]
            if _kw_major(n, shape):
                # conv weight (O, C, KW) stored [O][KW][C] so GEMM operand images and weight
                # gradients are contiguous; torch sees the same shape through a permuted view
                O, C, KW = shape
                flat[o:o + k].copy_(p.detach().permute(0, 2, 1).reshape(-1).float())
                p.data = flat[o:o + k].view(O, KW, C).permute(0, 2, 1)
                views[n] = gflat[o:o + k].view(O, KW, C).permute(0, 2, 1)
            else:
                flat[o:o + k].copy_(p.detach().reshape(-1).float())
                p.data = flat[o:o + k].view(shape)
                views[n] = gflat[o:o + k].view(shape)
        self._flat, self._gflat, self._grad_views, self._layout = flat, gflat, views, layout
        self._param_version += 1
        self._engine = None

    def group_ranges(self):
        """[(tag, start, end)] contiguous flat ranges per backward group, in completion order."""
        out = []
        for n, o, k, _, key in self._layout:
            tag = group_tag(key)
            end = o + (k + 15) // 16 * 16
            if out and out[-1][0] == tag:
                out[-1] = (tag, out[-1][1], end)
            else:
                out.append((tag, o, end))
        return out

    def engine(self):
        from .engine import FS2Engine
        self._ensure_packed()
        if self._engine is None or self._engine.adt != self.act_dtype:
            self._engine = FS2Engine(self, self.act_dtype)
        return self._engine

    def mark_params_updated(self):
        self._param_version += 1

    def _begin_backward(self):
        """zero + attach the flat gradient views unless gradients are being accumulated."""
        attached = all(p.grad is not None and p.grad.data_ptr() == self._grad_views[n].data_ptr()
                       for n, p in self.named_parameters())
        if not attached:
            self._gflat.zero_()
            for n, p in self.named_parameters():
                p.grad = self._grad_views[n]

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._param_version += 1
        return r

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self._flat = None
        self._engine = None
        return r

    # ------------------------------------------------------------------ forward
    def forward(self, tokens, speakers, durations=None, pitch=None, energy=None, pace=1.0,
                pitch_rate=1.0, energy_rate=1.0, intensity=None):
        """model.py:279-441; returns (mel_post, postnet_output, predict_durations, predict_pitch,
        avg_pitch, predict_energy, avg_energy, mel_lens)."""
        eng = self.engine()
        self._step_seed = (self._step_seed * 1103515245 + 12345) & 0x7fffffff
        args = (tokens, speakers, durations, pitch, energy, pace, pitch_rate, energy_rate,
                intensity)
        if torch.is_grad_enabled() and durations is not None and pitch is not None \
                and energy is not None:
            anchor = self.encPreNet.token_embedding.Embedding.weight
            return _FS2Function.apply(anchor, self, eng, self.training, self._step_seed, *args)
        with torch.no_grad():
            out, _ = eng.forward(*args, training=self.training, seed=self._step_seed)
        return out


class _FS2Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, model, eng, training, seed, tokens, speakers, durations, pitch,
                energy, pace, pitch_rate, energy_rate, intensity):
        out, ectx = eng.forward(tokens, speakers, durations, pitch, energy, pace, pitch_rate,
                                energy_rate, intensity, training=training, seed=seed)
        ctx.model, ctx.eng, ctx.ectx = model, eng, ectx
        mel, post, pd, pp, avg_p, pe, avg_e, mel_lens = out
        ctx.mark_non_differentiable(avg_p, avg_e, mel_lens)
        ctx.set_materialize_grads(False)
        ctx.shapes = (mel.shape, pd.shape, pp.shape, mel.dtype, mel.device)
        return mel, post, pd, pp, avg_p, pe, avg_e, mel_lens

    @staticmethod
    def backward(ctx, g_mel, g_post, g_pd, g_pp, g_avgp, g_pe, g_avge, g_len):
        mshape, pdshape, ppshape, dt, dev = ctx.shapes
        z = lambda g, s: g if g is not None else torch.zeros(s, dtype=dt, device=dev)
        ctx.model._begin_backward()
        ctx.eng.backward(ctx.ectx, z(g_mel, mshape), z(g_post, mshape), z(g_pd, pdshape),
                         z(g_pp, ppshape), z(g_pe, ppshape))
        ctx.ectx = None
        return (None,) * 14
