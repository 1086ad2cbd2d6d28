"""CPU: the oracle against the committed golden fixtures and known-answer tests.

These pin the oracle before it is trusted as the parity checker (DESIGN.md "Oracle"):
  * mask tiling: the reference's mask expression (model.py:338-343) through torch's real
    nn.MultiheadAttention equals the rule "key k masked for (b, h) iff pad[b][k] or
    pad[(b*nh+h) % B][k]" that the HIP softmax implements;
  * LengthRegulator: numpy, C and torch ``repeat_interleave`` expansions agree bit-exactly;
  * average_over_durations: numpy, C and the oracle's torch restatement agree bit-exactly;
  * the oracle's tiny-model forward / loss / gradients reproduce the committed fixture;
  * the reference docstring's shape example (model.py:133-146).
"""
import os

import numpy as np
import pytest
import torch

from oracle.fs2_oracle import (FastSpeech2Oracle, LossOracle, average_over_durations,
                               upsample, phoneme_average_intensity)
from oracle.lr_oracle import (avg_over_durations_np, avg_over_durations_c, lr_index_np,
                              lr_index_c)


def _masked_mha_rule(x, tokens, nh, w_in, b_in, w_out, b_out, quirk=True):
    """Explicit numpy attention with the head-major-quirk key mask."""
    B, T, D = x.shape
    dh = D // nh
    pad = tokens == 0
    qkv = x @ w_in.T + b_in
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    out = np.zeros((B, T, D), np.float64)
    for b in range(B):
        for h in range(nh):
            b2 = (b * nh + h) % B if quirk else b
            m = pad[b] | pad[b2]
            s = (q[b, :, h * dh:(h + 1) * dh] / np.sqrt(dh)) @ k[b, :, h * dh:(h + 1) * dh].T
            s = np.where(m[None, :], -np.inf, s)
            p = np.exp(s - s.max(1, keepdims=True))
            p /= p.sum(1, keepdims=True)
            out[b, :, h * dh:(h + 1) * dh] = p @ v[b, :, h * dh:(h + 1) * dh]
    return out @ w_out.T + b_out


def test_mask_tiling_rule_matches_torch_mha(golden_dir):
    g = np.load(os.path.join(golden_dir, "mask_tiling.npz"))
    ours = _masked_mha_rule(g["x"].astype(np.float64), g["tokens"], int(g["nhead"]),
                            g["in_proj_weight"], g["in_proj_bias"], g["out_proj_weight"],
                            g["out_proj_bias"])
    np.testing.assert_allclose(ours, g["out"], rtol=1e-5, atol=1e-6)
    # and the quirk is real: plain key padding gives a different answer
    plain = _masked_mha_rule(g["x"].astype(np.float64), g["tokens"], int(g["nhead"]),
                             g["in_proj_weight"], g["in_proj_bias"], g["out_proj_weight"],
                             g["out_proj_bias"], quirk=False)
    assert np.abs(plain - g["out"]).max() > 1e-3


@pytest.mark.parametrize("pace", [1.0, 1.1, 0.7])
def test_lr_index_golden_and_restatements(golden_dir, pace):
    g = np.load(os.path.join(golden_dir, "lr_kat.npz"))
    d = g["durs"]
    ml, fs = lr_index_np(d, pace)
    np.testing.assert_array_equal(ml, g[f"mel_len_{pace}"])
    np.testing.assert_array_equal(fs, g[f"frame_src_{pace}"])
    ml2, fs2 = lr_index_c(d, pace)
    np.testing.assert_array_equal(ml2, ml)
    np.testing.assert_array_equal(fs2, fs)
    # torch repeat_interleave (SB upsample as restated in the oracle)
    feats = torch.arange(d.shape[1], dtype=torch.float32).view(1, -1, 1).expand(d.shape[0], -1, 1)
    up, lens = upsample(feats, torch.from_numpy(d), pace=pace)
    assert lens == ml.tolist()
    for b in range(d.shape[0]):
        np.testing.assert_array_equal(up[b, :lens[b], 0].numpy().astype(np.int32), fs[b, :lens[b]])


def test_lr_index_float_durations(golden_dir):
    g = np.load(os.path.join(golden_dir, "lr_kat.npz"))
    ml, fs = lr_index_np(g["durs_f"], 1.0)
    np.testing.assert_array_equal(ml, g["mel_len_f"])
    np.testing.assert_array_equal(fs, g["frame_src_f"])
    ml2, fs2 = lr_index_c(g["durs_f"], 1.0)
    np.testing.assert_array_equal(fs2, fs)


def test_avg_over_durations_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "avg_kat.npz"))
    np.testing.assert_array_equal(avg_over_durations_np(g["values"], g["durs"]), g["avg"])
    np.testing.assert_array_equal(avg_over_durations_c(g["values"], g["durs"]), g["avg"])
    t = average_over_durations(torch.from_numpy(g["values"]).unsqueeze(1),
                               torch.from_numpy(g["durs"])).squeeze(1).numpy()
    np.testing.assert_array_equal(t, g["avg"])
    # semantics: mean over NON-ZERO frames, 0 where none
    v, d = g["values"], g["durs"]
    s = 0
    for p in range(d.shape[1]):
        seg = v[0, s:s + d[0, p]]
        nz = seg[seg != 0]
        exp = nz.mean() if len(nz) else 0.0
        assert abs(g["avg"][0, p] - exp) <= 1e-5 * max(1.0, abs(exp))
        s += d[0, p]


def test_oracle_tiny_fixture(golden_dir):
    fx = torch.load(os.path.join(golden_dir, "oracle_tiny.pt"), weights_only=True)
    m = FastSpeech2Oracle(**fx["config"], n_speakers=4).eval()
    m.load_state_dict(fx["state_dict"], strict=False)
    crit = LossOracle(**fx["loss_config"])
    b = fx["batch"]
    pred = m(b["phoneme"], b["speakers"], b["duration"], b["pitch"], b["energy"],
             intensity=b["intensity"])
    for got, exp in zip(pred, fx["outputs"]):
        torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-6)
    loss = crit(pred, (b["mel"], b["duration"], b["pitch"], b["energy"], b["mel_len"],
                       b["phon_len"]), 0)
    for k, v in fx["loss"].items():
        torch.testing.assert_close(loss[k], v, rtol=1e-5, atol=1e-6)
    loss["total_loss"].backward()
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.grad, fx["grads"][n], rtol=1e-4, atol=1e-6)


def test_docstring_shapes():
    """model.py:133-146: mel_post (2,15,80), predict_durations (2,5), predict_pitch (2,5,1)."""
    torch.manual_seed(0)
    m = FastSpeech2Oracle(enc_num_layers=1, enc_num_head=2, enc_d_model=32, enc_ffn_dim=64,
                          enc_k_dim=32, enc_v_dim=32, enc_dropout=0.1, dec_num_layers=1,
                          dec_num_head=2, dec_d_model=32, dec_ffn_dim=64, dec_k_dim=32,
                          dec_v_dim=32, dec_dropout=0.1, normalize_before=False, ffn_type="1dcnn",
                          ffn_cnn_kernel_size_list=[3, 1], n_char=40, n_mels=80,
                          postnet_embedding_dim=32, postnet_kernel_size=5,
                          postnet_n_convolutions=5, postnet_dropout=0.5, padding_idx=0,
                          dur_pred_kernel_size=3, pitch_pred_kernel_size=3,
                          energy_pred_kernel_size=3, variance_predictor_dropout=0.5,
                          n_speakers=1).eval()
    tokens = torch.tensor([[13, 12, 31, 14, 19], [31, 16, 30, 31, 0]])
    durations = torch.tensor([[2, 4, 1, 5, 3], [1, 2, 4, 3, 0]])
    pitch = torch.randn(2, 15)
    energy = torch.randn(2, 15)
    out = m(tokens, torch.zeros(2, dtype=torch.long), durations, pitch, energy,
            intensity=torch.zeros(2, 5, 5))
    assert out[0].shape == (2, 15, 80) and out[2].shape == (2, 5)
    assert out[3].shape == (2, 5, 1) and out[5].shape == (2, 5, 1)
    assert out[7].tolist() == [15, 10]   # 2+4+1+5+3, 1+2+4+3 (docstring shape claims hold)


def test_phoneme_average_intensity():
    """train.py:16-51: denominator clamp(d,1), zero frames included, zeros in padding."""
    I = torch.randn(2, 12, 5)
    d = torch.tensor([[3, 0, 4, 2], [5, 1, 0, 0]])
    out = phoneme_average_intensity(I, d, torch.tensor([4, 2]))
    torch.testing.assert_close(out[0, 0], I[0, 0:3].mean(0))
    assert torch.all(out[0, 1] == 0)
    torch.testing.assert_close(out[0, 2], I[0, 3:7].mean(0))
    torch.testing.assert_close(out[1, 1], I[1, 5])
    assert torch.all(out[1, 2:] == 0)


def _intensity_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "intensity_ref.npz"))
    cfg = {k: v for k, v in zip(z["cfg_keys"].tolist(), z["cfg_vals"].tolist())}
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")}
    return z, cfg, sd


def test_intensity_extractor_oracle_matches_reference(golden_dir):
    """oracle/intensity_oracle.py vs outputs of the REFERENCE IntensityExtractor
    (rank_model/model.py:96-109) on seeded weights, both input layouts (App. B-2 fix)."""
    from oracle.intensity_oracle import extractor_forward
    z, cfg, sd = _intensity_golden(golden_dir)
    x = torch.from_numpy(z["x"])
    args = (torch.from_numpy(z["lengths"]), torch.from_numpy(z["emotions"]),
            int(cfg["n_heads"]), int(cfg["n_encoder_layers"]))
    I = extractor_forward(sd, x, *args)
    np.testing.assert_allclose(I.numpy(), z["I"], rtol=1e-5, atol=1e-5)
    I2 = extractor_forward(sd, x.transpose(1, 2).contiguous(), *args, layout="BCT")
    np.testing.assert_allclose(I2.numpy(), z["I"], rtol=1e-5, atol=1e-5)


def test_phoneme_average_matches_reference(golden_dir):
    """Both restatements of train.py:29-49 vs the reference function's own output."""
    from oracle.intensity_oracle import phoneme_average_np
    z, _, _ = _intensity_golden(golden_dir)
    I, d, pl = torch.from_numpy(z["I"]), torch.from_numpy(z["duration"]), torch.from_numpy(z["phon_len"])
    np.testing.assert_allclose(phoneme_average_intensity(I, d, pl).numpy(), z["rep"], rtol=1e-6,
                               atol=1e-6)
    np.testing.assert_allclose(phoneme_average_np(z["I"], z["duration"], z["phon_len"]), z["rep"],
                               rtol=1e-5, atol=1e-6)


def test_intensity_container_keys_match_reference(golden_dir):
    """The drop-in IntensityExtractor / RankModel containers carry the reference's state_dict
    keys and shapes, so reference checkpoints load (train.py:218-221)."""
    from fastspeech2.intensity import IntensityExtractor, RankModel
    z, cfg, sd = _intensity_golden(golden_dir)
    kw = {k: (v if k == "dropout" else int(v)) for k, v in cfg.items()}
    m = IntensityExtractor(**kw)
    ours = m.state_dict()
    assert list(ours) == list(sd)
    for k in sd:
        assert ours[k].shape == sd[k].shape, k
    m.load_state_dict(sd)
    rm = RankModel(**kw)
    assert set(rm.state_dict()) == {"intensity_extractor." + k for k in sd} | {"projector.weight"}


def test_collate_oracle_matches_reference(golden_dir):
    """oracle/collate_oracle.py vs the reference TextMelCollateWithAlignment's own output
    (dataset.py:62-133, run by make_golden_collate.py), bit-exact incl. tie order."""
    from oracle.collate_oracle import collate_np, items_from_golden
    z = np.load(os.path.join(golden_dir, "collate_ref.npz"))
    out = collate_np(items_from_golden(z))
    for k, v in out.items():
        ref = z["out_" + k]
        if k in ("labels", "wavs"):
            assert list(v) == [str(s) for s in ref.tolist()], k
        else:
            assert np.array_equal(np.asarray(v), ref), k
