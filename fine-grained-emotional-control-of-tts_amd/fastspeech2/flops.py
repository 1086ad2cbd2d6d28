"""Algorithmic FLOP counts of the train step over the padded (B, T_max, hidden) layout
(SURVEY.md section 8d): per FFT layer 8TD^2 + 4T^2D + 2TDF(k0+k1) forward, predictors,
concat projection, mel linear, PostNet; train = 3x forward (backward = 2x forward)."""


def fft_layer_flops(T, D, F, ks):
    return 8 * T * D * D + 4 * T * T * D + 2 * T * D * F * (ks[0] + ks[1])


def forward_flops(cfg, B, Tp, Tm):
    c = cfg
    D = c.enc_d_model
    ks = c.ffn_cnn_kernel_size_list
    f = c.enc_num_layers * fft_layer_flops(Tp, D, c.enc_ffn_dim, ks)
    f += c.dec_num_layers * fft_layer_flops(Tm, D, c.dec_ffn_dim, ks)
    k = c.dur_pred_kernel_size
    f += 3 * (2 * 2 * Tp * D * k * D + 2 * Tp * D)
    f += 2 * Tp * (2 * D + 5) * D
    f += 2 * Tm * D * c.n_mels
    E, KP, NC = c.postnet_embedding_dim, c.postnet_kernel_size, c.postnet_n_convolutions
    f += 2 * Tm * KP * (c.n_mels * E + (NC - 2) * E * E + E * c.n_mels)
    return B * f


def train_flops(cfg, B, Tp, Tm):
    return 3 * forward_flops(cfg, B, Tp, Tm)


def extractor_flops(B, T, hidden, n_layers, kernel, n_in=82, n_emo=5):
    """Frozen IntensityExtractor forward (rank_model/model.py:96-109) over the padded (B, T)
    frames: input projection, per layer QKV + out projection 8TD^2, scores + context 4T^2D,
    two k-tap convs D<->4D 2*2*k*T*D*4D; classifier."""
    D = hidden
    per_layer = 8 * T * D * D + 4 * T * T * D + 2 * 2 * kernel * T * D * 4 * D
    return B * (2 * T * n_in * D + n_layers * per_layer + 2 * T * D * n_emo)


def vocoder_flops(B, T_frames, hp=None):
    """HiFi-GAN generator forward (fastspeech2.vocoder) over B utterances of T_frames mel frames
    (plus the 2 x inference_padding replicated frames): conv_pre, the polyphase upsampling
    GEMMs (3 taps, including their structural zero taps), 3 ResBlock1 x 3 x 2 convs per stage,
    conv_post."""
    from .vocoder import HPARAMS
    hp = hp or HPARAMS
    L = T_frames + 2 * hp["inference_padding"]
    c = hp["upsample_initial_channel"]
    f = 2 * L * 7 * hp["in_channels"] * c
    for u in hp["upsample_factors"]:
        f += 2 * L * 3 * c * (u * (c // 2))
        L *= u
        c //= 2
        for k, dils in zip(hp["resblock_kernel_sizes"], hp["resblock_dilation_sizes"]):
            f += len(dils) * 2 * 2 * L * k * c * c
    f += 2 * L * 7 * c
    return B * f
