"""HiFi-GAN generator forward on the MI355X kernels (BASELINE config 5's vocoder).

The reference decodes with speechbrain's pretrained ``HIFIGAN.from_hparams(source=
"speechbrain/tts-hifigan-libritts-16kHz")`` (fastspeech2/train.py:225, inference.py:60-63,
``vocoder.decode_batch(mel)`` at :85).  Neither speechbrain nor the hub weights exist here, so
this module rebuilds the generator architecture (SB 1.0.x ``HifiganGenerator`` with ``ResBlock1``
and the LibriTTS-16 kHz hyper-parameters, as restated in oracle/vocoder_oracle.py) with
weight-norm parameters; random-initialised unless a state dict with the same names is loaded.
Parity: against the restatement only ("parity unpinned").

Compute path (libfs2_hip.so only):
* ``fs2_vocoder_input``: (B, 80, T) mel -> rows with 5 replicated frames each side;
* every "same" conv (conv_pre, resblock convs with dilation 1/3/5, conv_post) is an implicit
  reflect-padded conv GEMM (conv_mode 1, ``conv_dil``) with bias, leaky-ReLU / tanh and the
  resblock residual add fused in the epilogue;
* every ConvTranspose1d(k = 2u, stride u, padding u/2) is ONE GEMM: the u output phases of
  output step q only read input steps q-1, q, q+1, so the layer is a 3-tap zero-padded conv
  (conv_mode 5) whose N = u * C_out columns are the phases; the GEMM output [B*L][u*C_out] is
  the upsampled sequence [B*L*u][C_out] in place;
* ``fs2_leaky_relu`` (ResBlock1's input activation) and ``fs2_mean3_leaky_relu`` (the mean of
  the three resblocks + the next stage's leaky ReLU).
The weight-norm reparameterisation (W = g v / ||v||) and the polyphase weight layout are
computed once per parameter update on the device when the weights are prepared.
"""

import torch
import torch.nn as nn

from . import _native as N
from . import ops
from .ops import round_up

HPARAMS = dict(in_channels=80, upsample_initial_channel=512, upsample_factors=(8, 8, 2, 2),
               upsample_kernel_sizes=(16, 16, 4, 4), resblock_kernel_sizes=(3, 7, 11),
               resblock_dilation_sizes=((1, 3, 5), (1, 3, 5), (1, 3, 5)), inference_padding=5)
LRELU_SLOPE = 0.1


class _WNConv(nn.Module):
    """weight-norm conv parameters: weight_g (dim-0 norms), weight_v, bias."""

    def __init__(self, shape, bias_n, std=0.01):
        super().__init__()
        v = torch.randn(*shape) * std
        self.weight_v = nn.Parameter(v)
        self.weight_g = nn.Parameter(v.flatten(1).norm(dim=1).reshape(-1, *([1] * (len(shape) - 1))))
        self.bias = nn.Parameter(torch.zeros(bias_n))


class _ResBlock1(nn.Module):
    def __init__(self, ch, k, dils):
        super().__init__()
        self.convs1 = nn.ModuleList([_WNConv((ch, ch, k), ch) for _ in dils])
        self.convs2 = nn.ModuleList([_WNConv((ch, ch, k), ch) for _ in dils])


class HifiganGenerator(nn.Module):
    """Generator parameters + ``decode_batch(mel (B, n_mels, T)) -> wav (B, 1, 256 (T + 10))``."""

    def __init__(self, act_dtype=torch.float32, hparams=None):
        super().__init__()
        hp = dict(HPARAMS, **(hparams or {}))
        self.hp = hp
        c0 = hp["upsample_initial_channel"]
        self.conv_pre = _WNConv((c0, hp["in_channels"], 7), c0)
        self.ups = nn.ModuleList()
        self.resblocks = nn.ModuleList()
        ch = c0
        for u, k in zip(hp["upsample_factors"], hp["upsample_kernel_sizes"]):
            assert k == 2 * u and u % 2 == 0, "polyphase form needs kernel = 2 x stride, even stride"
            self.ups.append(_WNConv((ch, ch // 2, k), ch // 2))
            ch //= 2
            for kr, dils in zip(hp["resblock_kernel_sizes"], hp["resblock_dilation_sizes"]):
                self.resblocks.append(_ResBlock1(ch, kr, dils))
        self.conv_post = _WNConv((1, ch, 7), 1)
        self.act_dtype = act_dtype
        self._engine = None

    def _apply(self, fn, *args, **kwargs):
        self._engine = None
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        r = super().load_state_dict(*args, **kwargs)
        self._engine = None
        return r

    @torch.no_grad()
    def decode_batch(self, mel):
        if mel.device.type != "cuda":
            raise RuntimeError("HifiganGenerator runs only on the HIP device (libfs2_hip.so)")
        if self._engine is None:
            self._engine = VocoderEngine(self)
        return self._engine.forward(mel)


def polyphase_weights(W, u):
    """ConvTranspose1d weight (C, O, 2u) with stride u, padding u/2 -> the 3-tap conv weight
    W3 [(r, o)][tap][c] of its polyphase form: output step q, phase r reads input step
    q + tap - 1 through kernel index j = r + u/2 + (1 - tap) u (zero where j is outside
    [0, 2u)).  Returned as (u*O, 3*C), i.e. [O'][KW][C]."""
    C, O, k = W.shape
    W3 = torch.zeros(u, O, 3, C, device=W.device, dtype=torch.float32)
    for r in range(u):
        a = r + u // 2
        for tap in range(3):
            j = a + (1 - tap) * u
            if 0 <= j < k:
                W3[r, :, tap, :] = W[:, :, j].t().float()
    return W3.reshape(u * O, 3 * C).contiguous()


def _wn(m):
    v, g = m.weight_v.detach().float(), m.weight_g.detach().float()
    return g * v / v.flatten(1).norm(dim=1).reshape(-1, *([1] * (v.dim() - 1)))


class VocoderEngine:
    def __init__(self, gen):
        N.load()
        self.g = gen
        self.adt = gen.act_dtype
        self.dt = N.dtype_code(self.adt)
        self.epc = ops.EPC[self.dt]
        self.dev = gen.conv_pre.weight_v.device
        self._ver = None
        self.w = {}

    def _prep_conv(self, name, m):
        """Conv1d (O, C, k) -> Wf [O][k*C] (activation dtype), fp32 bias."""
        W = _wn(m).contiguous()
        O, C, k = W.shape
        ldf = round_up(k * C, self.epc)
        Wf = torch.empty(O, ldf, dtype=self.adt, device=self.dev)
        ops.weight_prep(W, O, C, k, Wf, ldf, None, 0, dt=self.dt, w_okc=0)
        self.w[name] = (Wf, m.bias.detach().float().contiguous(), O, C, k)

    def _prep_up(self, name, m, u):
        """ConvTranspose1d (C, O, 2u), stride u, padding u/2 -> 3-tap polyphase conv weights
        W3[(r, o)][tap][c]: phase r reads input step q + tap - 1 with kernel index
        j = r + u/2 + (1 - tap) * u (taps whose j falls outside [0, 2u) are zero)."""
        W = _wn(m)                                  # (C, O, 2u)
        C, O, k = W.shape
        W3 = polyphase_weights(W, u)
        ldf = round_up(3 * C, self.epc)
        Wf = torch.empty(u * O, ldf, dtype=self.adt, device=self.dev)
        ops.weight_prep(W3, u * O, C, 3, Wf, ldf, None, 0, dt=self.dt, w_okc=1)
        bias = m.bias.detach().float().repeat(u).contiguous()
        self.w[name] = (Wf, bias, u * O, C, 3)

    def prepare(self):
        ver = tuple(p._version for p in self.g.parameters())
        if ver == self._ver:
            return
        g = self.g
        self._prep_conv("conv_pre", g.conv_pre)
        for i, (u, m) in enumerate(zip(g.hp["upsample_factors"], g.ups)):
            self._prep_up(f"ups.{i}", m, u)
        for bi, rb in enumerate(g.resblocks):
            for n in range(len(rb.convs1)):
                self._prep_conv(f"resblocks.{bi}.convs1.{n}", rb.convs1[n])
                self._prep_conv(f"resblocks.{bi}.convs2.{n}", rb.convs2[n])
        self._prep_conv("conv_post", g.conv_post)
        self._ver = ver

    def empty(self, *shape, dtype=None):
        return torch.empty(*shape, dtype=dtype or self.adt, device=self.dev)

    def _conv(self, name, X, M, T, out, ldo, mode=1, dil=1, act=0, residual=None, c_fp32=0):
        Wf, bias, O, C, k = self.w[name]
        K = Wf.shape[1]
        ops.gemm(M, O, K, X, X.shape[1], Wf, K, out, ldo, dt=self.dt, conv=(mode, T, k, C),
                 conv_dil=dil, bias=bias, relu=act, residual=residual,
                 ldr=residual.shape[1] if residual is not None else 0, c_fp32=c_fp32)

    def forward(self, mel):
        self.prepare()
        hp = self.g.hp
        mel = mel.to(device=self.dev, dtype=torch.float32).contiguous()
        B, NM, T0 = mel.shape
        pad = hp["inference_padding"]
        T = T0 + 2 * pad
        ldx = round_up(NM, self.epc)
        X0 = self.empty(B * T, ldx)
        ops.vocoder_input(mel, B, NM, T0, pad, X0, ldx, dt=self.dt)
        c0 = hp["upsample_initial_channel"]
        o = self.empty(B * T, c0)
        # conv_pre, then the first upsample's leaky ReLU (fused: o is only read through it)
        self._conv("conv_pre", X0, B * T, T, o, c0, act=3)
        del X0
        nk = len(hp["resblock_kernel_sizes"])
        ch = c0
        L = T
        n_up = len(hp["upsample_factors"])
        for i, u in enumerate(hp["upsample_factors"]):
            cout = ch // 2
            up = self.empty(B * L, u * cout)
            self._conv(f"ups.{i}", o, B * L, L, up, u * cout, mode=5)
            L *= u
            ch = cout
            x = up.view(B * L, ch)
            outs = []
            for j, dils in enumerate(hp["resblock_dilation_sizes"]):
                bi = i * nk + j
                xr = x
                for n, d in enumerate(dils):
                    xa = self.empty(B * L, ch)
                    ops.leaky_relu(xr, xa, B * L * ch, LRELU_SLOPE, dt=self.dt)
                    h = self.empty(B * L, ch)
                    self._conv(f"resblocks.{bi}.convs1.{n}", xa, B * L, L, h, ch, dil=d, act=3)
                    xn = self.empty(B * L, ch)
                    self._conv(f"resblocks.{bi}.convs2.{n}", h, B * L, L, xn, ch, residual=xr)
                    xr = xn
                outs.append(xr)
            # mean of the resblocks + the next leaky ReLU (0.1 before an upsample, F.leaky_relu's
            # default 0.01 before conv_post)
            o = self.empty(B * L, ch)
            ops.mean3_leaky_relu(outs[0], outs[1], outs[2], o, B * L * ch,
                                 LRELU_SLOPE if i + 1 < n_up else 0.01, dt=self.dt)
        wav = torch.empty(B * L, 1, dtype=torch.float32, device=self.dev)
        self._conv("conv_post", o, B * L, L, wav, 1, act=4, c_fp32=1)
        return wav.view(B, 1, L)
