"""Generates the committed golden fixtures under tests/golden/ (run in the dev container).

    python tests/golden/make_golden.py

Fixtures (all self-generated from the oracle / torch in this container; parity status of
each is stated in DESIGN.md "Oracle and parity"):
  mask_tiling.npz   torch nn.MultiheadAttention fed the reference's attention-mask
                    expression (model.py:338-343) + key_padding_mask, B=3 T=6 nh=2 lens
                    [6,4,2]: pins the head-major tiling quirk
  lr_kat.npz        LengthRegulator integer expansion, incl. zero durations and pace 1.1/0.7
  avg_kat.npz       average_over_durations with unvoiced (zero) frames and zero durations
  oracle_tiny.pt    oracle forward outputs, loss dict and all parameter gradients of a tiny
                    FastSpeech2 (D=32, 2+2 layers, 16 mels) on a B=2 batch, dropout off
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))

from oracle.fs2_oracle import FastSpeech2Oracle, LossOracle, get_key_padding_mask  # noqa: E402
from oracle.lr_oracle import lr_index_np, avg_over_durations_np  # noqa: E402
from fastspeech2.synthetic import make_batch, as_tuple  # noqa: E402

TINY = dict(enc_num_layers=2, enc_num_head=2, enc_d_model=32, enc_ffn_dim=64, enc_k_dim=32,
            enc_v_dim=32, enc_dropout=0.1, dec_num_layers=2, dec_num_head=2, dec_d_model=32,
            dec_ffn_dim=64, dec_k_dim=32, dec_v_dim=32, dec_dropout=0.1, normalize_before=False,
            ffn_type="1dcnn", ffn_cnn_kernel_size_list=[9, 1], n_char=20, n_mels=16,
            postnet_embedding_dim=32, postnet_kernel_size=5, postnet_n_convolutions=5,
            postnet_dropout=0.5, padding_idx=0, dur_pred_kernel_size=3, pitch_pred_kernel_size=3,
            energy_pred_kernel_size=3, variance_predictor_dropout=0.5)
LOSS = dict(log_scale_durations=True, ssim_loss_weight=1.0, duration_loss_weight=1.0,
            pitch_loss_weight=1.0, energy_loss_weight=1.0, mel_loss_weight=1.0,
            postnet_mel_loss_weight=1.0)


def mask_tiling():
    torch.manual_seed(0)
    B, T, D, nh = 3, 6, 8, 2
    lens = [6, 4, 2]
    tokens = torch.zeros(B, T, dtype=torch.long)
    for b, L in enumerate(lens):
        tokens[b, :L] = torch.arange(1, L + 1)
    x = torch.randn(B, T, D)
    mha = torch.nn.MultiheadAttention(D, nh)
    srcmask = get_key_padding_mask(tokens, 0)
    attn_mask = srcmask.unsqueeze(-1).repeat(nh, 1, T).permute(0, 2, 1).bool()  # model.py:338-343
    q = x.permute(1, 0, 2)
    with torch.no_grad():
        out, _ = mha(q, q, q, attn_mask=attn_mask, key_padding_mask=srcmask, need_weights=True)
    out = out.permute(1, 0, 2)
    sd = {k: v.numpy() for k, v in mha.state_dict().items()}
    np.savez(os.path.join(HERE, "mask_tiling.npz"), x=x.numpy(), tokens=tokens.numpy(),
             out=out.numpy(), lens=np.array(lens), nhead=nh,
             in_proj_weight=sd["in_proj_weight"], in_proj_bias=sd["in_proj_bias"],
             out_proj_weight=sd["out_proj.weight"], out_proj_bias=sd["out_proj.bias"])


def lr_kat():
    rng = np.random.default_rng(1)
    d = rng.integers(0, 10, (5, 17)).astype(np.int64)
    d[0, 3] = 0
    d[2, 10:] = 0          # ragged utterance
    d[4, :] = 0
    d[4, 0] = 7            # single voiced phoneme
    out = {"durs": d}
    for pace in (1.0, 1.1, 0.7):
        ml, fs = lr_index_np(d, pace)
        out[f"mel_len_{pace}"] = ml
        out[f"frame_src_{pace}"] = fs
    df = (rng.random((3, 9)) * 6).astype(np.float32)   # predicted (float) durations
    ml, fs = lr_index_np(df, 1.0)
    out.update(durs_f=df, mel_len_f=ml, frame_src_f=fs)
    np.savez(os.path.join(HERE, "lr_kat.npz"), **out)


def avg_kat():
    rng = np.random.default_rng(2)
    d = rng.integers(0, 6, (4, 11)).astype(np.int64)
    d[1, 7:] = 0
    Tm = int(d.sum(1).max()) + 3
    v = rng.standard_normal((4, Tm)).astype(np.float32)
    v[rng.random((4, Tm)) < 0.3] = 0.0
    np.savez(os.path.join(HERE, "avg_kat.npz"), values=v, durs=d, avg=avg_over_durations_np(v, d))


def oracle_tiny():
    torch.manual_seed(3)
    m = FastSpeech2Oracle(**TINY, n_speakers=4).eval()
    crit = LossOracle(**LOSS)
    b = make_batch(B=2, tp_min=12, tp_max=16, t_mel_cap=80, n_mels=16, n_char=20, seed=5)
    bt, inten = as_tuple(b)
    pred = m(bt[0], bt[1], bt[6], bt[4], bt[5], intensity=inten)
    loss = crit(pred, (bt[3], bt[6], bt[4], bt[5], bt[7], bt[2]), 0)
    loss["total_loss"].backward()
    torch.save({
        "config": TINY, "loss_config": LOSS,
        "state_dict": {k: v.clone() for k, v in m.state_dict().items()
                       if not k.startswith("sinusoidal")},   # PE tables are rebuilt
        "batch": {k: v.clone() for k, v in b.items()},
        "outputs": [None if x is None else x.detach().clone() for x in pred],
        "loss": {k: v.detach().clone() for k, v in loss.items()},
        "grads": {n: p.grad.clone() for n, p in m.named_parameters()},
    }, os.path.join(HERE, "oracle_tiny.pt"))


if __name__ == "__main__":
    mask_tiling()
    lr_kat()
    avg_kat()
    oracle_tiny()
    print("golden fixtures written to", HERE)
