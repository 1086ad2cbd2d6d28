"""GPU: the frozen IntensityExtractor forward + phoneme averaging through
libfs2_hip.so against the reference's own outputs (tests/golden/intensity_ref.npz, made by
make_golden_intensity.py from rank_model/model.py and train.py:16-51) and against the oracle
(oracle/intensity_oracle.py, pinned to those outputs in test_oracle.py) at full width.

Tolerances: fp32 activations rel 1e-4 (GEMM-class reassociation); bf16 activations rel 3e-2
against the fp32 oracle (bf16 storage of every activation over 6 layers); phoneme averaging
rel 1e-5 (fp32 sequential sums vs float64).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = torch.as_tensor(a).float().cpu(), torch.as_tensor(b).float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


def _golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "intensity_ref.npz"))
    cfg = {k: v for k, v in zip(z["cfg_keys"].tolist(), z["cfg_vals"].tolist())}
    kw = {k: (v if k == "dropout" else int(v)) for k, v in cfg.items()}
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")}
    return z, kw, sd


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
def test_extractor_matches_reference_golden(cuda, golden_dir, dt, tol):
    from fastspeech2.intensity import IntensityExtractor, get_intensity_representation
    z, kw, sd = _golden(golden_dir)
    m = IntensityExtractor(**kw, act_dtype=dt)
    m.load_state_dict(sd)
    m = m.to(cuda)
    x = torch.from_numpy(z["x"]).to(cuda)
    lengths = torch.from_numpy(z["lengths"]).to(cuda)
    emo = torch.from_numpy(z["emotions"]).to(cuda)
    I = m(x, lengths, emo)
    assert I.shape == z["I"].shape and I.dtype == torch.float32
    assert rel(I, z["I"]) < tol
    # the collate's (B, n_mels+2, T) tensor with the explicit layout fix (App. B-2)
    I2 = m(x.transpose(1, 2).contiguous(), lengths, emo, layout="BCT")
    assert rel(I2, z["I"]) < tol
    d = torch.from_numpy(z["duration"]).to(cuda)
    pl = torch.from_numpy(z["phon_len"]).to(cuda)
    batch = (None, None, pl, None, None, None, d, lengths, None, None,
             x.transpose(1, 2).contiguous(), emo)
    rep = get_intensity_representation(m, batch, cuda)
    assert rep.shape == z["rep"].shape
    assert rel(rep, z["rep"]) < tol


def _full_case(B=4, T=300, seed=0):
    g = torch.Generator().manual_seed(seed)
    lengths = torch.tensor([T, T - 37, T - 150, 61][:B])
    x = torch.randn(B, 82, T, generator=g)
    for b in range(B):
        x[b, :, int(lengths[b]):] = 0.0
    emo = torch.randint(0, 5, (B,), generator=g)
    return x, lengths, emo


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-3), (torch.bfloat16, 3e-2)])
def test_extractor_full_width_vs_oracle(cuda, cfg_all, dt, tol):
    """Reference config (parameter.yaml model.rank_model: 6 layers, hidden 384, 2 heads, k=9):
    the bf16 run takes the fused attention kernel (dh=192) with mask_mode 0."""
    from fastspeech2.intensity import IntensityExtractor
    from oracle.intensity_oracle import extractor_forward
    rc = cfg_all["model"]["rank_model"]
    torch.manual_seed(1)
    m = IntensityExtractor(80, rc["n_heads"], 5, rc["n_encoder_layers"], rc["hidden_dim"],
                           rc["kernel_size"], rc["dropout"], act_dtype=dt)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(cuda)
    x, lengths, emo = _full_case()
    I = m(x.to(cuda), lengths.to(cuda), emo.to(cuda), layout="BCT")
    ref = extractor_forward(sd, x, lengths, emo, rc["n_heads"], rc["n_encoder_layers"],
                            layout="BCT")
    assert rel(I, ref) < tol
    # padded frames carry exactly the classifier bias (masked_fill before the classifier)
    b = 3
    L = int(lengths[b])
    torch.testing.assert_close(I[b, L:].cpu(), sd["classifier.bias"].expand(I.shape[1] - L, 5),
                               rtol=0, atol=0)


def test_phoneme_average_full_size(cuda):
    """B=32, T_phon<=200, T_mel<=1000 synthetic collate: HIP segment mean vs numpy float64."""
    from fastspeech2.intensity import phoneme_average
    from fastspeech2.synthetic import make_batch
    from oracle.intensity_oracle import phoneme_average_np
    b = make_batch(B=32, seed=7)
    d = b["duration"].clone()
    d[0, 5] = 0                                   # zero-duration phoneme: 0 / clamp(0, 1) = 0
    I = torch.randn(32, b["mel"].shape[1], 5)
    out = phoneme_average(I.to(cuda), d.to(cuda), b["phon_len"].to(cuda))
    ref = phoneme_average_np(I.numpy(), d.numpy(), b["phon_len"].numpy())
    assert rel(out, ref) < 1e-5
    assert torch.all(out[0, 5] == 0)
    for i in range(32):
        assert torch.all(out[i, int(b["phon_len"][i]):] == 0)


@pytest.mark.parametrize("code,tol", [(0, 1e-5), (1, 2e-2)])
def test_softmax_plain_key_padding(cuda, code, tol):
    """fs2_softmax_fwd mask_mode 0 = nn.MultiheadAttention key_padding_mask only."""
    from fastspeech2 import ops
    dt = torch.float32 if code == 0 else torch.bfloat16
    B, H, T = 3, 2, 37
    ldt = ops.round_up(T, 8)
    S = torch.randn(B * H, T, ldt, device=cuda)
    lens = torch.tensor([37, 20, 9], device=cuda)
    kp = torch.empty(B * T, dtype=torch.uint8, device=cuda)
    ops.keypad_from_lengths(lens, B, T, kp)
    P = torch.empty(B * H, T, ldt, device=cuda, dtype=dt)
    ops.softmax_fwd(S, kp, B, H, T, T, ldt, 0.5, 0.0, 0, 1, P, None, dt=code, mask_mode=0)
    mask = (torch.arange(T, device=cuda)[None, :] >= lens[:, None]).repeat_interleave(H, 0)
    ref = torch.softmax((S[..., :T] * 0.5).masked_fill(mask[:, None, :], float("-inf")), -1)
    assert rel(P[..., :T], ref) < tol
