"""CPU oracle for the HiFi-GAN generator forward.  TEST INFRASTRUCTURE ONLY: used
by tests/ as the checker, never by the product package.

The reference decodes mels with speechbrain's ``HIFIGAN.from_hparams(source="speechbrain/
tts-hifigan-libritts-16kHz")`` (fastspeech2/train.py:225, inference.py:60-63,85):
``vocoder.decode_batch(mel (B, n_mels, T))``.  speechbrain is not installed here and the hub
weights cannot be fetched, so this is a restatement of the generator as recalled from SB 1.0.x
``speechbrain/lobes/models/HifiGAN.py`` (``HifiganGenerator``, ``ResBlock1``) with the
LibriTTS-16 kHz hyper-parameters (in 80, upsample factors 8 8 2 2 = hop 256, upsample kernels
16 16 4 4, initial channels 512, resblock kernels 3 7 11 with dilations 1 3 5, inference
padding 5 replicated frames):

  x = replicate-pad(mel, 5) ; o = conv_pre(x)                        Conv1d(80, 512, 7, same)
  for each upsample i:  o = ups[i](leaky_relu(o, 0.1))              ConvTranspose1d(k=2u, u, p=u/2)
                        o = mean_j resblock[i, j](o)                 ResBlock1, kernels 3 / 7 / 11
  o = tanh(conv_post(leaky_relu(o)))                                 slope 0.01; Conv1d(C, 1, 7, same)
  ResBlock1(x): for d in (1, 3, 5): x = x + c2(lrelu(c1_d(lrelu(x, .1)), .1))   (c1 dilation d)

"same" convs pad reflectively (SB Conv1d's default padding_mode), dilation-aware
(pad = d (k-1) / 2 per side).  Weight norm (SB ``weight_norm=True``): W = g * v / ||v|| with the
norm over every dim except dim 0 (output channels for Conv1d, input channels for
ConvTranspose1d, torch's default).

Parity status: **unpinned** -- neither the SB source nor the weights are available here; the
restatement fixes the arithmetic the HIP path must reproduce, not the reference's bits.
"""

import torch
import torch.nn.functional as F

HPARAMS = dict(in_channels=80, upsample_initial_channel=512, upsample_factors=(8, 8, 2, 2),
               upsample_kernel_sizes=(16, 16, 4, 4), resblock_kernel_sizes=(3, 7, 11),
               resblock_dilation_sizes=((1, 3, 5), (1, 3, 5), (1, 3, 5)), inference_padding=5)
LRELU_SLOPE = 0.1


def wn(g, v):
    """torch weight_norm (dim 0): g * v / ||v|| over all other dims."""
    norm = v.flatten(1).norm(dim=1).reshape(-1, *([1] * (v.dim() - 1)))
    return g * v / norm


def conv_same(x, w, b, dilation=1):
    """(B, C, T) reflect-padded 'same' conv (SB Conv1d, stride 1)."""
    k = w.shape[-1]
    pad = dilation * (k - 1) // 2
    return F.conv1d(F.pad(x, (pad, pad), mode="reflect"), w, b, dilation=dilation)


def generator_forward(params, mel, hp=HPARAMS):
    """params: dict name -> tensor with the generator's weight-norm parameters (see
    fastspeech2.vocoder.HifiganGenerator for the names); mel (B, n_mels, T) -> (B, 1, 256 (T+10))."""
    P = {k: v.float() for k, v in params.items()}
    x = F.pad(mel.float(), (hp["inference_padding"],) * 2, mode="replicate")
    o = conv_same(x, wn(P["conv_pre.weight_g"], P["conv_pre.weight_v"]), P["conv_pre.bias"])
    nk = len(hp["resblock_kernel_sizes"])
    for i, (u, k) in enumerate(zip(hp["upsample_factors"], hp["upsample_kernel_sizes"])):
        o = F.leaky_relu(o, LRELU_SLOPE)
        w = wn(P[f"ups.{i}.weight_g"], P[f"ups.{i}.weight_v"])
        o = F.conv_transpose1d(o, w, P[f"ups.{i}.bias"], stride=u, padding=(k - u) // 2)
        z = None
        for j, (kr, dils) in enumerate(zip(hp["resblock_kernel_sizes"],
                                           hp["resblock_dilation_sizes"])):
            r = f"resblocks.{i * nk + j}."
            xr = o
            for n, d in enumerate(dils):
                xt = F.leaky_relu(xr, LRELU_SLOPE)
                xt = conv_same(xt, wn(P[r + f"convs1.{n}.weight_g"], P[r + f"convs1.{n}.weight_v"]),
                               P[r + f"convs1.{n}.bias"], d)
                xt = F.leaky_relu(xt, LRELU_SLOPE)
                xt = conv_same(xt, wn(P[r + f"convs2.{n}.weight_g"], P[r + f"convs2.{n}.weight_v"]),
                               P[r + f"convs2.{n}.bias"], 1)
                xr = xt + xr
            z = xr if z is None else z + xr
        o = z / nk
    o = F.leaky_relu(o)
    o = conv_same(o, wn(P["conv_post.weight_g"], P["conv_post.weight_v"]), P["conv_post.bias"])
    return torch.tanh(o)
