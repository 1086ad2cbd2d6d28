"""CPU oracle for the FastSpeech2-with-emotion-intensity train step.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this file;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker / CPU baseline.

What it is
----------
An op-for-op PyTorch-CPU fp32 restatement of the reference hot path

* ``FastSpeech2.__init__``/``forward``  -- /root/reference/emo_rank_tts/fastspeech2/model.py:149-441
* ``Loss.forward``                        -- /root/reference/emo_rank_tts/fastspeech2/loss.py:31-186
* the train step                          -- /root/reference/emo_rank_tts/fastspeech2/train.py:72-81, 232

The reference delegates almost all arithmetic to ``speechbrain`` (SB 1.0.x), which is
NOT present in this container (``ModuleNotFoundError``), so the
SB layers are restated here from their published semantics,
on top of the same torch primitives SB wraps (``nn.MultiheadAttention``,
``nn.LayerNorm``, ``nn.Conv1d`` with reflect "same" padding, ``nn.Linear``,
``nn.Embedding``).  Parity status: **partially unpinned** -- the SB layer semantics
cannot be checked against SB source here.  What *is* pinned:

* the attention-mask construction and its head-major tiling quirk are computed with
  the reference's own expression (model.py:338-343) fed to torch's real
  ``nn.MultiheadAttention`` -- the exact call SB makes;
* the docstring shape example (model.py:133-146) -- shapes only;
* the LengthRegulator integer expansion follows ``repeat_interleave`` semantics and is
  checked bit-exactly against ``oracle/lr_oracle.py`` (numpy) and the C restatement.

State-dict keys follow SB naming so that weights
interchange with the product model and with reference checkpoints.
"""

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# SB lobes, restated
# --------------------------------------------------------------------------

class SBLinear(nn.Module):
    """speechbrain.nnet.linear.Linear -> nn.Linear at attribute ``w`` (App. A.13)."""

    def __init__(self, n_neurons, input_size, bias=True):
        super().__init__()
        self.w = nn.Linear(input_size, n_neurons, bias=bias)

    def forward(self, x):
        return self.w(x)


class SBEmbedding(nn.Module):
    """speechbrain.nnet.embedding.Embedding -> nn.Embedding at ``Embedding`` (App. A.6)."""

    def __init__(self, num_embeddings, embedding_dim):
        super().__init__()
        self.Embedding = nn.Embedding(num_embeddings, embedding_dim)

    def forward(self, x):
        return self.Embedding(x.long())


class SBConv1d(nn.Module):
    """speechbrain.nnet.CNN.Conv1d, padding="same", padding_mode="reflect" (App. A.1).

    Input (B, T, C) (transposed internally) unless ``skip_transpose``; pads
    floor((k-1)/2) frames each side with *reflect* then runs a padding-free conv.
    """

    def __init__(self, in_channels, out_channels, kernel_size, skip_transpose=False, bias=True):
        super().__init__()
        self.kernel_size = kernel_size
        self.skip_transpose = skip_transpose
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size, bias=bias)

    def forward(self, x):
        if not self.skip_transpose:
            x = x.transpose(1, -1)
        p = (self.kernel_size - 1) // 2
        if p > 0:
            x = F.pad(x, (p, p), mode="reflect")
        y = self.conv(x)
        if not self.skip_transpose:
            y = y.transpose(1, -1)
        return y


class SBLayerNorm(nn.Module):
    """speechbrain.nnet.normalization.LayerNorm -> nn.LayerNorm at ``norm``."""

    def __init__(self, input_size, eps=1e-5):
        super().__init__()
        self.norm = nn.LayerNorm(input_size, eps=eps)

    def forward(self, x):
        return self.norm(x)


class SBMultiheadAttention(nn.Module):
    """speechbrain.nnet.attention.MultiheadAttention (App. A.4).

    Wraps torch's nn.MultiheadAttention at attribute ``att``; inputs (B,T,D) are
    permuted to (T,B,D) and the call uses need_weights=True.
    """

    def __init__(self, nhead, d_model, dropout=0.0, kdim=None, vdim=None):
        super().__init__()
        self.att = nn.MultiheadAttention(d_model, nhead, dropout=dropout, bias=True,
                                         kdim=kdim, vdim=vdim)

    def forward(self, q, k, v, attn_mask=None, key_padding_mask=None):
        q, k, v = q.permute(1, 0, 2), k.permute(1, 0, 2), v.permute(1, 0, 2)
        out, att = self.att(q, k, v, attn_mask=attn_mask, key_padding_mask=key_padding_mask,
                            need_weights=True)
        return out.permute(1, 0, 2), att


class SBTransformerEncoderLayer(nn.Module):
    """SB TransformerEncoderLayer, ffn_type='1dcnn', post-LN (App. A.2)."""

    def __init__(self, d_ffn, nhead, d_model, kdim, vdim, dropout, kernel_sizes):
        super().__init__()
        self.self_att = SBMultiheadAttention(nhead, d_model, dropout, kdim, vdim)
        self.pos_ffn = nn.Sequential(
            SBConv1d(d_model, d_ffn, kernel_sizes[0]),
            nn.ReLU(),
            SBConv1d(d_ffn, d_model, kernel_sizes[1]),
        )
        self.norm1 = SBLayerNorm(d_model, eps=1e-6)
        self.norm2 = SBLayerNorm(d_model, eps=1e-6)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)

    def forward(self, src, src_mask=None, src_key_padding_mask=None):
        output, att = self.self_att(src, src, src, attn_mask=src_mask,
                                    key_padding_mask=src_key_padding_mask)
        src = self.norm1(src + self.dropout1(output))
        output = self.pos_ffn(src)
        output = self.norm2(src + self.dropout2(output))
        return output, att


class SBTransformerEncoder(nn.Module):
    """SB TransformerEncoder: layers then a final LayerNorm(eps=1e-6) (App. A.3)."""

    def __init__(self, num_layers, nhead, d_ffn, d_model, kdim, vdim, dropout, kernel_sizes):
        super().__init__()
        self.layers = nn.ModuleList([
            SBTransformerEncoderLayer(d_ffn, nhead, d_model, kdim, vdim, dropout, kernel_sizes)
            for _ in range(num_layers)
        ])
        self.norm = SBLayerNorm(d_model, eps=1e-6)

    def forward(self, src, src_mask=None, src_key_padding_mask=None):
        out = src
        atts = []
        for layer in self.layers:
            out, att = layer(out, src_mask=src_mask, src_key_padding_mask=src_key_padding_mask)
            atts.append(att)
        return self.norm(out), atts


class SBPositionalEncoding(nn.Module):
    """SB PositionalEncoding(input_size, max_len=2500) (App. A.5)."""

    def __init__(self, input_size, max_len=2500):
        super().__init__()
        pe = torch.zeros(max_len, input_size)
        positions = torch.arange(0, max_len).unsqueeze(1).float()
        denominator = torch.exp(torch.arange(0, input_size, 2).float()
                                * -(math.log(10000.0) / input_size))
        pe[:, 0::2] = torch.sin(positions * denominator)
        pe[:, 1::2] = torch.cos(positions * denominator)
        self.register_buffer("pe", pe.unsqueeze(0))

    def forward(self, x):
        return self.pe[:, : x.size(1)].clone().detach()


class SBEncoderPreNet(nn.Module):
    """SB EncoderPreNet -> token_embedding (SBEmbedding, no padding_idx) (App. A.6)."""

    def __init__(self, n_vocab, blank_id, out_channels):
        super().__init__()
        self.token_embedding = SBEmbedding(n_vocab, out_channels)

    def forward(self, x):
        return self.token_embedding(x)


class SBDurationPredictor(nn.Module):
    """SB DurationPredictor (App. A.7): [mask->conv->relu->LN(1e-5)->drop]x2 -> mask->linear."""

    def __init__(self, in_channels, out_channels, kernel_size, dropout=0.0):
        super().__init__()
        self.conv1 = SBConv1d(in_channels, out_channels, kernel_size)
        self.conv2 = SBConv1d(out_channels, out_channels, kernel_size)
        self.linear = SBLinear(1, out_channels)
        self.ln1 = SBLayerNorm(out_channels)
        self.ln2 = SBLayerNorm(out_channels)
        self.relu = nn.ReLU()
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)

    def forward(self, x, x_mask):
        x = self.relu(self.conv1(x * x_mask))
        x = self.dropout1(self.ln1(x))
        x = self.relu(self.conv2(x * x_mask))
        x = self.dropout2(self.ln2(x))
        return self.linear(x * x_mask)


class SBPostNet(nn.Module):
    """SB PostNet (App. A.8): note the 3 intermediate convs run back-to-back."""

    def __init__(self, n_mel_channels=80, postnet_embedding_dim=512, postnet_kernel_size=5,
                 postnet_n_convolutions=5, postnet_dropout=0.5):
        super().__init__()
        self.conv_pre = SBConv1d(n_mel_channels, postnet_embedding_dim, postnet_kernel_size)
        self.convs_intermedite = nn.ModuleList([
            SBConv1d(postnet_embedding_dim, postnet_embedding_dim, postnet_kernel_size)
            for _ in range(1, postnet_n_convolutions - 1)
        ])
        self.conv_post = SBConv1d(postnet_embedding_dim, n_mel_channels, postnet_kernel_size)
        self.tanh = nn.Tanh()
        self.ln1 = nn.LayerNorm(postnet_embedding_dim)
        self.ln2 = nn.LayerNorm(postnet_embedding_dim)
        self.ln3 = nn.LayerNorm(n_mel_channels)
        self.dropout1 = nn.Dropout(postnet_dropout)
        self.dropout2 = nn.Dropout(postnet_dropout)
        self.dropout3 = nn.Dropout(postnet_dropout)

    def forward(self, x):
        x = self.conv_pre(x)
        x = self.dropout1(self.tanh(self.ln1(x)))
        for conv in self.convs_intermedite:
            x = conv(x)
        x = self.dropout2(self.tanh(self.ln2(x)))
        x = self.conv_post(x)
        x = self.dropout3(self.ln3(x))
        return x


def get_key_padding_mask(tokens, pad_idx):
    """SB get_key_padding_mask for 2-D input (App. A.11)."""
    return tokens.eq(pad_idx)


def get_mask_from_lengths(lengths):
    """SB get_mask_from_lengths (App. A.11): True = padded."""
    max_len = int(torch.max(lengths).item())
    ids = torch.arange(0, max_len, device=lengths.device, dtype=lengths.dtype)
    return ~(ids < lengths.unsqueeze(1))


def upsample(feats, durs, pace=1.0, padding_value=0.0):
    """SB upsample (App. A.9): per-utterance repeat_interleave by (pace*d).long()."""
    ups = [torch.repeat_interleave(feats[i], (pace * durs[i]).long(), dim=0)
           for i in range(len(durs))]
    mel_lens = [u.shape[0] for u in ups]
    return nn.utils.rnn.pad_sequence(ups, batch_first=True, padding_value=padding_value), mel_lens


def average_over_durations(values, durs):
    """SB average_over_durations (App. A.10): cumsum/gather, mean over NON-ZERO frames."""
    durs_cums_ends = torch.cumsum(durs, dim=1).long()
    durs_cums_starts = F.pad(durs_cums_ends[:, :-1], (1, 0))
    values_nonzero_cums = F.pad(torch.cumsum(values != 0.0, dim=2), (1, 0))
    values_cums = F.pad(torch.cumsum(values, dim=2), (1, 0))
    bs, length = durs_cums_ends.size()
    n_formants = values.size(1)
    dcs = durs_cums_starts[:, None, :].expand(bs, n_formants, length)
    dce = durs_cums_ends[:, None, :].expand(bs, n_formants, length)
    values_sums = (torch.gather(values_cums, 2, dce) - torch.gather(values_cums, 2, dcs)).float()
    values_nelems = (torch.gather(values_nonzero_cums, 2, dce)
                     - torch.gather(values_nonzero_cums, 2, dcs)).float()
    return torch.where(values_nelems == 0.0, values_nelems, values_sums / values_nelems)


# --------------------------------------------------------------------------
# FastSpeech2 (model.py:32-441)
# --------------------------------------------------------------------------

class FastSpeech2Oracle(nn.Module):
    """Restatement of emo_rank_tts/fastspeech2/model.py:FastSpeech2."""

    def __init__(self, enc_num_layers, enc_num_head, enc_d_model, enc_ffn_dim, enc_k_dim,
                 enc_v_dim, enc_dropout, dec_num_layers, dec_num_head, dec_d_model, dec_ffn_dim,
                 dec_k_dim, dec_v_dim, dec_dropout, normalize_before, ffn_type,
                 ffn_cnn_kernel_size_list, n_char, n_mels, postnet_embedding_dim,
                 postnet_kernel_size, postnet_n_convolutions, postnet_dropout, padding_idx,
                 dur_pred_kernel_size, pitch_pred_kernel_size, energy_pred_kernel_size,
                 variance_predictor_dropout, n_speakers):
        super().__init__()
        assert not normalize_before and ffn_type == "1dcnn"
        self.enc_num_head = enc_num_head
        self.dec_num_head = dec_num_head
        self.padding_idx = padding_idx
        self.sinusoidal_positional_embed_encoder = SBPositionalEncoding(enc_d_model)
        self.sinusoidal_positional_embed_decoder = SBPositionalEncoding(dec_d_model)
        self.speaker_emb = SBEmbedding(n_speakers, enc_d_model)                        # :194-198
        self.concat_proj = SBLinear(enc_d_model, enc_d_model + enc_d_model + 5, bias=False)  # :199-203
        self.encPreNet = SBEncoderPreNet(n_char, padding_idx, enc_d_model)
        # all three predictors use dur_pred_kernel_size (model.py:211,217,223; App. B-10)
        self.durPred = SBDurationPredictor(enc_d_model, enc_d_model, dur_pred_kernel_size,
                                           variance_predictor_dropout)
        self.pitchPred = SBDurationPredictor(enc_d_model, enc_d_model, dur_pred_kernel_size,
                                             variance_predictor_dropout)
        self.energyPred = SBDurationPredictor(enc_d_model, enc_d_model, dur_pred_kernel_size,
                                              variance_predictor_dropout)
        self.pitchEmbed = SBConv1d(1, enc_d_model, pitch_pred_kernel_size, skip_transpose=True)
        self.energyEmbed = SBConv1d(1, enc_d_model, energy_pred_kernel_size, skip_transpose=True)
        self.encoder = SBTransformerEncoder(enc_num_layers, enc_num_head, enc_ffn_dim, enc_d_model,
                                            enc_k_dim, enc_v_dim, enc_dropout,
                                            ffn_cnn_kernel_size_list)
        self.decoder = SBTransformerEncoder(dec_num_layers, dec_num_head, dec_ffn_dim, dec_d_model,
                                            dec_k_dim, dec_v_dim, dec_dropout,
                                            ffn_cnn_kernel_size_list)
        self.linear = SBLinear(n_mels, dec_d_model)
        self.postnet = SBPostNet(n_mels, postnet_embedding_dim, postnet_kernel_size,
                                 postnet_n_convolutions, postnet_dropout)

    @staticmethod
    def head_major_attn_mask(srcmask, nhead, T):
        """The reference's attention-mask expression (model.py:338-343 / 414-419).

        ``.repeat(nhead, 1, T)`` lays the (B*nhead) masks out head-major, while torch
        reads them batch-major -- the head-major tiling quirk.
        """
        return srcmask.unsqueeze(-1).repeat(nhead, 1, T).permute(0, 2, 1).bool()

    def forward(self, tokens, speakers, durations=None, pitch=None, energy=None, pace=1.0,
                pitch_rate=1.0, energy_rate=1.0, intensity=None):
        srcmask = get_key_padding_mask(tokens, pad_idx=self.padding_idx)          # :331
        srcmask_inverted = (~srcmask).unsqueeze(-1)                              # :332
        token_feats = self.encPreNet(tokens)                                     # :335
        pos = self.sinusoidal_positional_embed_encoder(token_feats)
        token_feats = torch.add(token_feats, pos) * srcmask_inverted             # :337
        attn_mask = self.head_major_attn_mask(srcmask, self.enc_num_head, token_feats.shape[1])
        token_feats, _ = self.encoder(token_feats, src_mask=attn_mask,
                                      src_key_padding_mask=srcmask)             # :344-346
        token_feats = token_feats * srcmask_inverted                             # :347

        B, T, D = token_feats.shape                                              # :352-360
        speaker_emb = self.speaker_emb(speakers).unsqueeze(1).expand(-1, T, -1)
        x = torch.cat([token_feats, speaker_emb, intensity], dim=-1)
        token_feats = self.concat_proj(x) * srcmask_inverted

        predict_durations = self.durPred(token_feats, srcmask_inverted).squeeze(-1)  # :366
        if predict_durations.dim() == 1:
            predict_durations = predict_durations.unsqueeze(0)
        if durations is None:
            dur_pred_reverse_log = torch.clamp(torch.special.expm1(predict_durations), 0)

        avg_pitch = None                                                         # :378-389
        predict_pitch = self.pitchPred(token_feats, srcmask_inverted) * pitch_rate
        if pitch is not None:
            avg_pitch = average_over_durations(pitch.unsqueeze(1), durations)
            pitch = self.pitchEmbed(avg_pitch)
            avg_pitch = avg_pitch.permute(0, 2, 1)
        else:
            pitch = self.pitchEmbed(predict_pitch.permute(0, 2, 1))
        token_feats = token_feats.add(pitch.permute(0, 2, 1))

        avg_energy = None                                                        # :392-403
        predict_energy = self.energyPred(token_feats, srcmask_inverted) * energy_rate
        if energy is not None:
            avg_energy = average_over_durations(energy.unsqueeze(1), durations)
            energy = self.energyEmbed(avg_energy)
            avg_energy = avg_energy.permute(0, 2, 1)
        else:
            energy = self.energyEmbed(predict_energy.permute(0, 2, 1))
        token_feats = token_feats.add(energy.permute(0, 2, 1))

        spec_feats, mel_lens = upsample(                                         # :406-410
            token_feats, durations if durations is not None else dur_pred_reverse_log, pace=pace)
        srcmask = get_mask_from_lengths(torch.tensor(mel_lens)).to(spec_feats.device)
        srcmask_inverted = (~srcmask).unsqueeze(-1)
        attn_mask = self.head_major_attn_mask(srcmask, self.dec_num_head, spec_feats.shape[1])
        pos = self.sinusoidal_positional_embed_decoder(spec_feats)              # :422-423
        spec_feats = torch.add(spec_feats, pos) * srcmask_inverted
        output_mel_feats, _ = self.decoder(spec_feats, src_mask=attn_mask,
                                           src_key_padding_mask=srcmask)        # :425-427
        mel_post = self.linear(output_mel_feats) * srcmask_inverted              # :430
        postnet_output = self.postnet(mel_post) + mel_post                       # :431
        return (mel_post, postnet_output, predict_durations, predict_pitch, avg_pitch,
                predict_energy, avg_energy, torch.tensor(mel_lens))


# --------------------------------------------------------------------------
# SSIM (SB SSIMLoss, Coqui/piq-derived; App. A.12)
# --------------------------------------------------------------------------

def gaussian_filter(kernel_size=11, sigma=1.5, dtype=torch.float32):
    coords = torch.arange(kernel_size, dtype=dtype)
    coords -= (kernel_size - 1) / 2.0
    g = coords ** 2
    g = (-(g.unsqueeze(0) + g.unsqueeze(1)) / (2 * sigma ** 2)).exp()
    g /= g.sum()
    return g.unsqueeze(0)


def _ssim_per_channel(x, y, kernel, k1=0.01, k2=0.03):
    # valid ("padding=0") 2-D Gaussian filtering, as in piq's _ssim_per_channel
    c1, c2 = k1 ** 2, k2 ** 2
    n_channels = x.size(1)
    mu_x = F.conv2d(x, weight=kernel, stride=1, padding=0, groups=n_channels)
    mu_y = F.conv2d(y, weight=kernel, stride=1, padding=0, groups=n_channels)
    mu_xx, mu_yy, mu_xy = mu_x ** 2, mu_y ** 2, mu_x * mu_y
    sigma_xx = F.conv2d(x ** 2, weight=kernel, stride=1, padding=0, groups=n_channels) - mu_xx
    sigma_yy = F.conv2d(y ** 2, weight=kernel, stride=1, padding=0, groups=n_channels) - mu_yy
    sigma_xy = F.conv2d(x * y, weight=kernel, stride=1, padding=0, groups=n_channels) - mu_xy
    cs = (2.0 * sigma_xy + c2) / (sigma_xx + sigma_yy + c2)
    ss = (2.0 * mu_xy + c1) / (mu_xx + mu_yy + c1) * cs
    return ss.mean(dim=(-1, -2)), cs.mean(dim=(-1, -2))


def ssim(x, y, kernel_size=11, kernel_sigma=1.5, data_range=1.0, k1=0.01, k2=0.03):
    x = x / float(data_range)
    y = y / float(data_range)
    f = max(1, round(min(x.size()[-2:]) / 256))
    if f > 1:
        x = F.avg_pool2d(x, kernel_size=f)
        y = F.avg_pool2d(y, kernel_size=f)
    kernel = gaussian_filter(kernel_size, kernel_sigma, dtype=x.dtype).repeat(x.size(1), 1, 1, 1)
    ssim_map, _ = _ssim_per_channel(x, y, kernel, k1, k2)
    return ssim_map.mean(1).mean()


class SSIMLoss(nn.Module):
    """SB SSIMLoss: masked per-sample min-max normalisation, then 1 - SSIM, clamped."""

    @staticmethod
    def sequence_mask(sequence_length, max_len):
        seq_range = torch.arange(max_len, dtype=sequence_length.dtype)
        return seq_range.unsqueeze(0) < sequence_length.unsqueeze(1)

    @staticmethod
    def sample_wise_min_max(x, mask):
        maximum = torch.amax(x.masked_fill(~mask, 0), dim=(1, 2), keepdim=True)
        minimum = torch.amin(x.masked_fill(~mask, math.inf), dim=(1, 2), keepdim=True)
        return (x - minimum) / (maximum - minimum + 1e-8)

    def forward(self, y_hat, y, length):
        mask = self.sequence_mask(length, y.size(1)).unsqueeze(2)
        y_norm = self.sample_wise_min_max(y, mask)
        y_hat_norm = self.sample_wise_min_max(y_hat, mask)
        loss = 1.0 - ssim((y_norm * mask).unsqueeze(1), (y_hat_norm * mask).unsqueeze(1))
        if loss.item() > 1.0:
            loss = torch.tensor(1.0)
        if loss.item() < 0.0:
            loss = torch.tensor(0.0)
        return loss


class LossOracle(nn.Module):
    """Restatement of emo_rank_tts/fastspeech2/loss.py:Loss."""

    def __init__(self, log_scale_durations, ssim_loss_weight, duration_loss_weight,
                 pitch_loss_weight, energy_loss_weight, mel_loss_weight, postnet_mel_loss_weight,
                 spn_loss_weight=1.0, spn_loss_max_epochs=8):
        super().__init__()
        self.ssim_loss = SSIMLoss()
        self.mse = nn.MSELoss()
        self.log_scale_durations = log_scale_durations
        self.w = dict(ssim=ssim_loss_weight, mel=mel_loss_weight, post=postnet_mel_loss_weight,
                      dur=duration_loss_weight, pitch=pitch_loss_weight, energy=energy_loss_weight)

    def forward(self, predictions, targets, current_epoch):
        mel_target, target_durations, target_pitch, target_energy, mel_length, phon_len = targets
        assert len(mel_target.shape) == 3
        (mel_out, postnet_mel_out, log_durations, predicted_pitch, average_pitch,
         predicted_energy, average_energy, mel_lens) = predictions
        predicted_pitch = predicted_pitch.squeeze(-1)                 # loss.py:101-105
        predicted_energy = predicted_energy.squeeze(-1)
        target_pitch = average_pitch.squeeze(-1)
        target_energy = average_energy.squeeze(-1)
        log_durations = log_durations.squeeze(-1)
        log_target_durations = torch.log1p(target_durations.float())  # :108-109
        B = mel_target.shape[0]
        for i in range(B):                                            # :112-154
            L, P = int(mel_length[i]), int(phon_len[i])
            m = self.mse(mel_out[i, :L, :], mel_target[i, :L, :])
            pm = self.mse(postnet_mel_out[i, :L, :], mel_target[i, :L, :])
            d = self.mse(log_durations[i, :P], log_target_durations[i, :P].to(torch.float32))
            # pitch/energy are phoneme-level but sliced by the MEL length (App. B-3)
            p = self.mse(predicted_pitch[i, :L], target_pitch[i, :L].to(torch.float32))
            e = self.mse(predicted_energy[i, :L], target_energy[i, :L].to(torch.float32))
            if i == 0:
                mel_loss, post_loss, dur_loss, pitch_loss, energy_loss = m, pm, d, p, e
            else:
                mel_loss, post_loss = mel_loss + m, post_loss + pm
                dur_loss, pitch_loss, energy_loss = dur_loss + d, pitch_loss + p, energy_loss + e
        ssim_loss = self.ssim_loss(mel_out, mel_target, mel_length)   # :155 (pre-postnet mel)
        mel_loss, post_loss = mel_loss / B, post_loss / B
        dur_loss, pitch_loss, energy_loss = dur_loss / B, pitch_loss / B, energy_loss / B
        w = self.w
        total = (ssim_loss * w["ssim"] + mel_loss * w["mel"] + post_loss * w["post"]
                 + dur_loss * w["dur"] + pitch_loss * w["pitch"] + energy_loss * w["energy"])
        return {"total_loss": total, "ssim_loss": ssim_loss * w["ssim"],
                "mel_loss": mel_loss * w["mel"], "postnet_mel_loss": post_loss * w["post"],
                "dur_loss": dur_loss * w["dur"], "pitch_loss": pitch_loss * w["pitch"],
                "energy_loss": energy_loss * w["energy"]}


# --------------------------------------------------------------------------
# train step (train.py:72-81) and intensity averaging (train.py:16-51)
# --------------------------------------------------------------------------

def train_step(model, criterion, optim, batch, intensity, epoch=0):
    """One reference train step: forward -> loss -> zero_grad -> backward -> AdamW.step."""
    (phoneme, spk_ids, phon_len, mel_tgt, pitch_tgt, energy_tgt, duration_tgt, mel_len) = batch[:8]
    predictions = model(phoneme, spk_ids, duration_tgt, pitch_tgt, energy_tgt, intensity=intensity)
    targets = (mel_tgt, duration_tgt, pitch_tgt, energy_tgt, mel_len, phon_len)
    loss = criterion(predictions, targets, epoch)
    optim.zero_grad()
    loss["total_loss"].backward()
    optim.step()
    return predictions, loss


def phoneme_average_intensity(I, duration_tgt, phon_len):
    """train.py:16-51 per-utterance segment mean of frame-level intensity logits.

    Denominator is clamp(d, 1) and zero frames are included (unlike
    average_over_durations).  I: (B, T_mel, E) -> (B, T_phon_max, E).
    """
    B, Tp = duration_tgt.shape
    E = I.shape[-1]
    out = torch.zeros(B, Tp, E)
    for b in range(B):
        P = int(phon_len[b])
        d = duration_tgt[b].long()[:P]
        Tm = int(d.sum())
        idx = torch.repeat_interleave(torch.arange(P), d)
        s = torch.zeros(P, E)
        s.index_add_(0, idx, I[b, :Tm, :])
        out[b, :P, :] = s / d.unsqueeze(1).float().clamp(min=1.0)
    return out
