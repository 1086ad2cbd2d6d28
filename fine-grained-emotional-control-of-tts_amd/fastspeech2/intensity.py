"""Drop-in frozen ``IntensityExtractor`` forward and ``get_intensity_representation`` on the
MI355X kernels.

Reference:
* ``IntensityExtractor``  -- emo_rank_tts/rank_model/model.py:56-109 (input projection :71,
  ``nn.TransformerEncoder`` of ``ConvTransformerEncoderLayer`` :8-50 / :74-75, emotion
  embedding :78, classifier :81, mask :84-93, forward :96-109);
* ``RankModel`` container -- rank_model/model.py:115-135 (``rank_model.intensity_extractor`` is
  what fastspeech2/train.py:218-221 loads and freezes);
* ``get_intensity_representation`` -- fastspeech2/train.py:16-51.

The modules here are parameter containers with the reference's attribute names, so
``state_dict()`` keys equal the reference's and its checkpoints load with ``load_state_dict``.
The forward runs only through libfs2_hip.so:
  input staging (``fs2_intensity_input``) -> input projection GEMM -> per layer:
  QKV GEMM -> attention with plain key padding (``fs2_attn_fwd`` / ``fs2_softmax_fwd``,
  mask_mode 0) -> out-projection GEMM -> LN(x + attn) -> conv1 k=9 zero-padded implicit GEMM
  with a GELU epilogue (conv_mode 5, act 2) -> conv2 k=9 -> LN(x + ffn) -> emotion head
  (``fs2_intensity_head``) -> phoneme averaging (``fs2_phoneme_average``).
The extractor is frozen in the reference train step (``.eval().requires_grad_(False)`` and
``torch.no_grad()``, train.py:23,221): forward only, dropout off, no activations kept.

The reference passes the collate's ``rank_X`` of shape (B, n_mels+2, T)
(fastspeech2/dataset.py:94,116) to an extractor that reads (B, T, n_mels+2)
(rank_model/model.py:86,100), which raises unless T == 82.  Here the layout
is explicit: ``layout="BCT"`` (the collate's tensor, transposed inside the staging kernel) or
``layout="BTC"`` (what the extractor was trained on).
"""

import copy
import math

import torch
import torch.nn as nn

from . import _native as N
from . import ops
from .ops import round_up


class ConvTransformerEncoderLayer(nn.Module):
    """Parameter container of rank_model/model.py:8-50 (same attribute names)."""

    def __init__(self, n_heads, hidden_dim, kernel_size, dropout=0.1):
        super().__init__()
        self.self_attn = nn.MultiheadAttention(embed_dim=hidden_dim, num_heads=n_heads,
                                               dropout=dropout, batch_first=True)
        self.conv1 = nn.Conv1d(hidden_dim, hidden_dim * 4, kernel_size=kernel_size,
                               padding=kernel_size // 2)
        self.conv2 = nn.Conv1d(hidden_dim * 4, hidden_dim, kernel_size=kernel_size,
                               padding=kernel_size // 2)
        self.norm1 = nn.LayerNorm(hidden_dim)
        self.norm2 = nn.LayerNorm(hidden_dim)
        self.dropout = nn.Dropout(dropout)
        self.activation = nn.GELU()


class _FFTBlock(nn.Module):
    """``nn.TransformerEncoder(encoder_layer, n)``: ``n`` deep copies of ONE initialised layer
    (so all layers start identical, as in the reference), keys ``layers.{i}.*``, no final norm."""

    def __init__(self, layer, n):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(n)])


class IntensityExtractor(nn.Module):
    """Drop-in for rank_model/model.py:56-109: ``forward(x, length, emotions) -> (B, T, E)``."""

    def __init__(self, n_mels, n_heads, n_emotions, n_encoder_layers, hidden_dim, kernel_size,
                 dropout, act_dtype=torch.float32):
        super().__init__()
        self.input_proj = nn.Linear(n_mels + 2, hidden_dim)
        layer = ConvTransformerEncoderLayer(n_heads, hidden_dim, kernel_size, dropout)
        self.fft_block = _FFTBlock(layer, n_encoder_layers)
        self.emotion_embedding = nn.Embedding(n_emotions, hidden_dim)
        self.classifier = nn.Linear(hidden_dim, n_emotions)
        self.n_mels, self.n_heads, self.n_emotions = n_mels, n_heads, n_emotions
        self.n_layers, self.hidden, self.kernel = n_encoder_layers, hidden_dim, kernel_size
        self.act_dtype = act_dtype
        self._engine = None

    def prepare_mask(self, x, length):
        """rank_model/model.py:84-93 (True at padded frames)."""
        B, T, _ = x.size()
        return torch.arange(T, device=x.device).unsqueeze(0).expand(B, T) >= length.unsqueeze(1)

    def engine(self):
        if self._engine is None:
            self._engine = ExtractorEngine(self)
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        self._engine = None          # device / dtype moves invalidate the weight images
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        r = super().load_state_dict(*args, **kwargs)
        self._engine = None
        return r

    @torch.no_grad()
    def forward(self, x, length, emotions, layout="BTC"):
        """x (B, T, n_mels+2) with layout="BTC", or the collate's (B, n_mels+2, T) with
        layout="BCT"; length (B,) valid frames; emotions (B,) ids.  Returns I (B, T, E) fp32."""
        if x.device.type != "cuda":
            raise RuntimeError("IntensityExtractor runs only on the HIP device (libfs2_hip.so); "
                               "there is no CPU path")
        return self.engine().forward(x, length, emotions, layout)


class RankModel(nn.Module):
    """Parameter container of rank_model/model.py:115-135 so reference RankModel checkpoints load
    (``rank_model.load_state_dict(...)``, train.py:218-221).  Only ``.intensity_extractor`` is on
    the FastSpeech2 train path; the rank-model training forward is out of scope."""

    def __init__(self, n_mels, n_heads, n_emotions, n_encoder_layers, hidden_dim, kernel_size,
                 dropout, act_dtype=torch.float32, **kwargs):
        super().__init__()
        self.n_emotions = n_emotions
        self.intensity_extractor = IntensityExtractor(n_mels, n_heads, n_emotions,
                                                      n_encoder_layers, hidden_dim, kernel_size,
                                                      dropout, act_dtype=act_dtype)
        self.projector = nn.Linear(n_emotions, 1, bias=False)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("rank-model training is outside the FastSpeech2 train path "
                                  "(DESIGN.md section 7); use .intensity_extractor")


class ExtractorEngine:
    """Forward of the frozen extractor over libfs2_hip.so (no autograd, no saved activations)."""

    def __init__(self, ext):
        N.load()
        self.x = ext
        self.adt = ext.act_dtype
        self.dt = N.dtype_code(self.adt)
        self.epc = ops.EPC[self.dt]
        self.dev = ext.input_proj.weight.device
        D, KW = ext.hidden, ext.kernel
        if KW % 2 != 1:
            raise ValueError("kernel_size must be odd (padding=k//2 keeps the length only then)")
        self.specs = {"input_proj.weight": (D, ext.n_mels + 2, 1)}
        for i in range(ext.n_layers):
            p = f"fft_block.layers.{i}."
            self.specs[p + "self_attn.in_proj_weight"] = (3 * D, D, 1)
            self.specs[p + "self_attn.out_proj.weight"] = (D, D, 1)
            self.specs[p + "conv1.weight"] = (4 * D, D, KW)
            self.specs[p + "conv2.weight"] = (D, 4 * D, KW)
        self.w = {}
        self.p = {}
        self._ver = None
        self._ws = torch.empty(1 << 16, dtype=torch.float32, device=self.dev)

    def prepare(self):
        """fp32 torch-layout weights (O, C, KW) -> K-major GEMM images Wf[O][KW*C] in the
        activation dtype (rebuilt when a parameter changes)."""
        params = dict(self.x.named_parameters())
        ver = tuple(p._version for p in params.values())
        if self._ver == ver:
            return
        for name, (O, C, KW) in self.specs.items():
            ldf = round_up(KW * C, self.epc)
            if name not in self.w:
                self.w[name] = torch.empty(O, ldf, dtype=self.adt, device=self.dev)
            W = params[name].detach().float().contiguous()
            self.p[name] = W
            ops.weight_prep(W, O, C, KW, self.w[name], ldf, None, 0, dt=self.dt, w_okc=0)
        self.p.update({n: t.detach().float().contiguous() for n, t in params.items()
                       if n not in self.specs})
        self._ver = ver

    def empty(self, *shape, dtype=None):
        return torch.empty(*shape, dtype=dtype or self.adt, device=self.dev)

    def _gemm(self, X, ldx, M, T, wname, out, ldo, conv=False, **epi):
        O, C, KW = self.specs[wname]
        Wf = self.w[wname]
        K = Wf.shape[1]
        ops.gemm(M, O, K, X, ldx, Wf, K, out, ldo, dt=self.dt,
                 conv=(5, T, KW, C) if conv else None, **epi)

    def _attention(self, QKV, key_pad, B, T, D, H, out):
        dh = D // H
        scale = 1.0 / math.sqrt(dh)
        if self.dt == N.BF16 and ops.attn_supported(T, dh, self.dt):
            lse = torch.empty(B * H, T, dtype=torch.float32, device=self.dev)
            ops.attn_fwd(QKV, 3 * D, key_pad, B, H, T, dh, scale, 0.0, 0, 0, out, D, lse,
                         dt=self.dt, mask_mode=0)
            return
        ldt = round_up(T, 8)
        S = torch.empty(B * H, T, ldt, dtype=torch.float32, device=self.dev)
        ops.gemm(T, T, dh, QKV, 3 * D, QKV[:, D:], 3 * D, S, ldt, dt=self.dt, c_fp32=1,
                 batch=B * H, batch_div=H,
                 strides=(T * 3 * D, dh, T * 3 * D, dh, H * T * ldt, T * ldt, 0, 0))
        Pm = self.empty(B * H, T, ldt)
        ops.softmax_fwd(S, key_pad, B, H, T, T, ldt, scale, 0.0, 0, 0, Pm, None, dt=self.dt,
                        mask_mode=0)
        del S
        ops.gemm(T, dh, ldt, Pm, ldt, QKV[:, 2 * D:], 3 * D, out, D, dt=self.dt, b_kmajor=0,
                 kvalid=T, batch=B * H, batch_div=H,
                 strides=(H * T * ldt, T * ldt, T * 3 * D, dh, T * D, dh, 0, 0))

    def forward(self, x, length, emotions, layout="BTC"):
        ext = self.x
        self.prepare()
        D, H, E = ext.hidden, ext.n_heads, ext.n_emotions
        C = ext.n_mels + 2
        if layout not in ("BTC", "BCT"):
            raise ValueError(f"layout must be 'BTC' or 'BCT', got {layout!r}")
        x = x.to(device=self.dev, dtype=torch.float32).contiguous()
        if layout == "BTC":
            B, T, Cx = x.shape
        else:
            B, Cx, T = x.shape
        if Cx != C:
            raise RuntimeError(f"extractor input has {Cx} channels, expected n_mels + 2 = {C} "
                               f"(layout={layout})")
        length = length.to(device=self.dev, dtype=torch.int64).contiguous()
        emotions = emotions.to(device=self.dev, dtype=torch.int64).contiguous()
        M = B * T
        P = self.p
        ldx = round_up(C, self.epc)
        X0 = self.empty(M, ldx)
        ops.intensity_input(x, int(layout == "BCT"), B, T, C, X0, ldx, dt=self.dt)
        key_pad = torch.empty(M, dtype=torch.uint8, device=self.dev)
        ops.keypad_from_lengths(length, B, T, key_pad)                  # model.py:84-93
        X = self.empty(M, D)
        self._gemm(X0, ldx, M, T, "input_proj.weight", X, D, bias=P["input_proj.bias"])
        del X0
        mean = torch.empty(M, dtype=torch.float32, device=self.dev)
        rstd = torch.empty_like(mean)
        for i in range(ext.n_layers):
            p = f"fft_block.layers.{i}."
            QKV = self.empty(M, 3 * D)
            self._gemm(X, D, M, T, p + "self_attn.in_proj_weight", QKV, 3 * D,
                       bias=P[p + "self_attn.in_proj_bias"])
            Att = self.empty(M, D)
            self._attention(QKV, key_pad, B, T, D, H, Att)
            del QKV
            Ao = self.empty(M, D)
            self._gemm(Att, D, M, T, p + "self_attn.out_proj.weight", Ao, D,
                       bias=P[p + "self_attn.out_proj.bias"])
            X1 = self.empty(M, D)
            ops.ln_fwd(X, D, P[p + "norm1.weight"], P[p + "norm1.bias"], 1e-5, X1, D, mean, rstd,
                       M, D, dt=self.dt, r=Ao, ldr=D)                       # model.py:36-37
            Hc = self.empty(M, 4 * D)
            self._gemm(X1, D, M, T, p + "conv1.weight", Hc, 4 * D, conv=True,
                       bias=P[p + "conv1.bias"], relu=2)                     # :40-43 GELU
            Y = self.empty(M, D)
            self._gemm(Hc, 4 * D, M, T, p + "conv2.weight", Y, D, conv=True,
                       bias=P[p + "conv2.bias"])                             # :44-46
            del Hc
            X = self.empty(M, D)
            ops.ln_fwd(X1, D, P[p + "norm2.weight"], P[p + "norm2.bias"], 1e-5, X, D, mean, rstd,
                       M, D, dt=self.dt, r=Y, ldr=D)                        # :48-49
        I = torch.empty(B, T, E, dtype=torch.float32, device=self.dev)
        ops.intensity_head(X, D, P["emotion_embedding.weight"], emotions, length,
                           P["classifier.weight"], P["classifier.bias"], B, T, D, E, I,
                           dt=self.dt)                                      # :103-107
        return I


def phoneme_average(I, durations, phon_len):
    """train.py:29-49: per-phoneme mean of I over each phoneme's frames (denominator
    clamp(d, 1)), zeros past phon_len.  I (B, T, E) fp32 on the HIP device -> (B, T_phon, E)."""
    I = I.float().contiguous()
    B, T, E = I.shape
    durations = durations.to(device=I.device, dtype=torch.int64).contiguous()
    phon_len = phon_len.to(device=I.device, dtype=torch.int64).contiguous()
    Tp = durations.shape[1]
    out = torch.empty(B, Tp, E, dtype=torch.float32, device=I.device)
    ops.phoneme_average(I, T, E, durations, phon_len, B, Tp, out)
    return out


@torch.no_grad()
def get_intensity_representation(intensity_extractor, batch, device=None, layout="BCT"):
    """fastspeech2/train.py:16-51 on the HIP device.  ``batch`` is the collate's 12-tuple
    (phoneme, _, phon_len, _, _, _, duration_tgt, mel_len, _, _, rank_X, emo_ids); ``rank_X``
    is the collate's (B, n_mels+2, T) tensor, hence ``layout="BCT"``."""
    (phoneme, _, phon_len, _, _, _, duration_tgt, mel_len, _, _, rank_X, emo_ids) = batch
    I = intensity_extractor(rank_X, mel_len, emo_ids, layout=layout)
    return phoneme_average(I, duration_tgt, phon_len)
