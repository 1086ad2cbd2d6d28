"""GPU: whole-model parity of the HIP train path against the oracle (fp32, dropout off),
bf16 behaviour, the drop-in API, and size-independent properties at BASELINE's full size.

Tolerances (north_star: mel/variance tensors within 1e-3 relative fp32, LengthRegulator
bit-exact):
  fp32 outputs       max|a-b| / max|b| <= 1e-3   (observed ~2e-6)
  fp32 losses        rel 1e-4
  fp32 param grads   max|a-b| / max|b| <= 1e-2 per tensor, median <= 1e-4
  bf16 outputs       <= 5e-2; bf16 grads: cosine similarity >= 0.99 per tensor
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


def _pair(cfg_all, dt=torch.float32, seed=0):
    from fastspeech2.model import FastSpeech2
    from oracle.fs2_oracle import FastSpeech2Oracle
    kw = cfg_all["model"]["fastspeech2"]
    torch.manual_seed(seed)
    o = FastSpeech2Oracle(**kw, n_speakers=4).eval()
    torch.manual_seed(seed)
    m = FastSpeech2(**kw, n_speakers=4, act_dtype=dt).cuda().eval()
    return o, m


def _run_both(o, m, cfg_all, b):
    from fastspeech2.loss import Loss
    from oracle.fs2_oracle import LossOracle
    from fastspeech2.synthetic import as_tuple
    bt, inten = as_tuple(b)
    po = o(bt[0], bt[1], bt[6], bt[4], bt[5], intensity=inten)
    lo = LossOracle(**cfg_all["loss"])(po, (bt[3], bt[6], bt[4], bt[5], bt[7], bt[2]), 0)
    lo["total_loss"].backward()
    g = [t.cuda() for t in bt]
    pm = m(g[0], g[1], g[6], g[4], g[5], intensity=inten.cuda())
    lm = Loss(**cfg_all["loss"])(pm, (g[3], g[6], g[4], g[5], g[7], g[2]), 0)
    lm["total_loss"].backward()
    torch.cuda.synchronize()
    return po, lo, pm, lm


def test_tiny_model_matches_committed_oracle_fixture(cuda, golden_dir):
    from fastspeech2.model import FastSpeech2
    from fastspeech2.loss import Loss
    fx = torch.load(os.path.join(golden_dir, "oracle_tiny.pt"), weights_only=True)
    m = FastSpeech2(**fx["config"], n_speakers=4).cuda().eval()
    m.load_state_dict(fx["state_dict"], strict=False)
    b = {k: v.cuda() for k, v in fx["batch"].items()}
    pm = m(b["phoneme"], b["speakers"], b["duration"], b["pitch"], b["energy"],
           intensity=b["intensity"])
    for got, exp in zip(pm, fx["outputs"]):
        assert rel(got, exp) <= 1e-3
    lm = Loss(**fx["loss_config"])(pm, (b["mel"], b["duration"], b["pitch"], b["energy"],
                                        b["mel_len"], b["phon_len"]), 0)
    for k, v in fx["loss"].items():
        assert abs(lm[k].item() - v.item()) <= 1e-4 * max(1.0, abs(v.item())), k
    lm["total_loss"].backward()
    errs = [rel(p.grad, fx["grads"][n]) for n, p in m.named_parameters()]
    assert max(errs) <= 1e-2 and float(np.median(errs)) <= 1e-4


@pytest.mark.parametrize("emotion", [False, True])
def test_full_model_fp32_matches_oracle(cuda, cfg_all, emotion):
    """Default dims (D=384, 6+6 layers), BASELINE config 1 shape: B=2, T_phon=50."""
    from fastspeech2.synthetic import make_batch
    o, m = _pair(cfg_all)
    b = make_batch(B=2, tp_min=50, tp_max=50, seed=0, emotion=emotion)
    po, lo, pm, lm = _run_both(o, m, cfg_all, b)
    for i, (a, r) in enumerate(zip(pm, po)):
        if i == 7:
            assert torch.equal(a.cpu(), r)                    # mel_lens, integer
        else:
            assert rel(a, r) <= 1e-3, i
    for k in lo:
        assert abs(lm[k].item() - lo[k].item()) <= 1e-4 * max(1.0, abs(lo[k].item())), k
    go = dict(o.named_parameters())
    errs = {n: rel(p.grad, go[n].grad) for n, p in m.named_parameters()}
    assert max(errs.values()) <= 1e-2, max(errs.items(), key=lambda kv: kv[1])
    assert float(np.median(list(errs.values()))) <= 1e-4


def test_ragged_batch_and_zero_durations_fp32(cuda, cfg_all):
    """Ragged utterances (padding inside the batch) and a zero-duration phoneme."""
    from fastspeech2.synthetic import make_batch
    o, m = _pair(cfg_all, seed=1)
    b = make_batch(B=3, tp_min=20, tp_max=40, seed=7, t_mel_cap=150)
    b["duration"][0, 3] = 0            # a phoneme with no frames
    b["mel_len"] = b["duration"].sum(1)
    Tm = int(b["mel_len"].max())
    b["mel"], b["pitch"], b["energy"] = b["mel"][:, :Tm], b["pitch"][:, :Tm], b["energy"][:, :Tm]
    for i in range(3):
        L = int(b["mel_len"][i])
        b["mel"][i, L:] = 0
        b["pitch"][i, L:] = 0
        b["energy"][i, L:] = 0
    po, lo, pm, lm = _run_both(o, m, cfg_all, b)
    for i in range(7):
        assert rel(pm[i], po[i]) <= 1e-3, i
    assert abs(lm["total_loss"].item() - lo["total_loss"].item()) <= 1e-4 * abs(lo["total_loss"].item())


def test_full_model_bf16_close_to_oracle(cuda, cfg_all):
    from fastspeech2.synthetic import make_batch
    o, m = _pair(cfg_all, dt=torch.bfloat16)
    b = make_batch(B=2, tp_min=50, tp_max=50, seed=0)
    po, lo, pm, lm = _run_both(o, m, cfg_all, b)
    for i in range(7):
        assert rel(pm[i], po[i]) <= 5e-2, i
    assert abs(lm["total_loss"].item() - lo["total_loss"].item()) <= 2e-2 * abs(lo["total_loss"].item())
    go = dict(o.named_parameters())
    for n, p in m.named_parameters():
        a, r = p.grad.float().cpu().flatten(), go[n].grad.flatten()
        cos = torch.nn.functional.cosine_similarity(a, r, dim=0).item()
        assert cos >= 0.99, (n, cos)


def test_dropin_train_step_torch_adamw_equals_fused_trainer(cuda, cfg_all):
    """train.py:72-81 with torch.optim.AdamW == FusedTrainer (fused loss + fused AdamW), fp32."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.loss import Loss
    from fastspeech2.train import train_step, FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    kw = cfg_all["model"]["fastspeech2"]
    b = make_batch(B=2, tp_min=30, tp_max=40, seed=3, device="cuda")
    bt, inten = as_tuple(b)
    torch.manual_seed(0)
    m1 = FastSpeech2(**kw, n_speakers=4).cuda().eval()
    torch.manual_seed(0)
    m2 = FastSpeech2(**kw, n_speakers=4).cuda().eval()
    opt = torch.optim.AdamW(m1.parameters(), lr=1e-4)
    _, l1 = train_step(m1, Loss(**cfg_all["loss"]), opt, bt, inten)
    tr = FusedTrainer(m2, lr=1e-4)
    # FusedTrainer always trains with dropout; compare on the deterministic p=0 path
    for k in ("enc_dropout", "dec_dropout", "postnet_dropout", "variance_predictor_dropout"):
        setattr(m2.cfg, k, 0.0)
    l2 = tr.step(bt, inten)
    torch.cuda.synchronize()
    assert abs(l1["total_loss"].item() - l2[0].item()) <= 1e-4 * abs(l2[0].item())
    # the first Adam step is ~lr*sign(g): elements whose exact gradient is 0 (e.g. the key
    # bias, softmax shift invariance) move by +-lr on rounding noise, so allow |dp| <= 2 lr
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        d = (p2.detach() - p1.detach()).abs().max().item()
        assert d <= 2e-4 + 1e-3 * p1.detach().abs().max().item(), (n, d)


def test_inference_branch_predicted_durations(cuda, cfg_all):
    """durations=None: clamp(expm1(pred), 0) -> .long() truncation (model.py:372-375, 408)."""
    from fastspeech2.synthetic import make_batch
    o, m = _pair(cfg_all, seed=2)
    with torch.no_grad():   # push predicted log-durations to ~log(1+5) so frames exist
        for mod in (o, m):
            mod.durPred.linear.w.weight.mul_(0.05)
            mod.durPred.linear.w.bias.fill_(1.8)
    b = make_batch(B=2, tp_min=20, tp_max=30, seed=9)
    with torch.no_grad():
        po = o(b["phoneme"], b["speakers"], intensity=b["intensity"])
        pm = m(b["phoneme"].cuda(), b["speakers"].cuda(), intensity=b["intensity"].cuda())
    assert torch.equal(pm[7].cpu(), po[7])
    assert rel(pm[2], po[2]) <= 1e-3
    if int(po[7].max()) > 0:
        assert rel(pm[0], po[0]) <= 1e-3


def test_full_size_train_properties_bf16(cuda, cfg_all):
    """BASELINE size (B=32, T_phon<=200, T_mel<=1000): size-independent properties.

    * LengthRegulator index expansion bit-exact vs the numpy oracle;
    * mel_len == sum(durations); decoder padding rows of mel_post are exactly zero;
    * loss finite and decreasing over a few fused steps (dropout on).
    """
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    from fastspeech2 import ops
    from oracle.lr_oracle import lr_index_np
    kw = cfg_all["model"]["fastspeech2"]
    b = make_batch(B=32, seed=11, device="cuda")
    bt, inten = as_tuple(b)
    d = b["duration"]
    B, Tp = d.shape
    Tm = b["mel"].shape[1]
    ml = torch.empty(B, dtype=torch.int64, device="cuda")
    cum = torch.empty(B, Tp, dtype=torch.int32, device="cuda")
    fs = torch.empty(B, Tm, dtype=torch.int32, device="cuda")
    ops.lr_index(d, 0, 1.0, B, Tp, Tm, ml, cum, fs)
    ml_ref, fs_ref = lr_index_np(d.cpu().numpy(), 1.0, Tm)
    np.testing.assert_array_equal(fs.cpu().numpy(), fs_ref)
    assert torch.equal(ml, b["mel_len"])
    torch.manual_seed(0)
    m = FastSpeech2(**kw, n_speakers=4, act_dtype=torch.bfloat16).cuda().train()
    tr = FusedTrainer(m, lr=3e-4)
    losses = [tr.step(bt, inten)[0].item() for _ in range(6)]
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0]
    with torch.no_grad():
        out = m(bt[0], bt[1], bt[6], bt[4], bt[5], intensity=inten)
    mel = out[0].float()
    for i in range(B):
        assert torch.all(mel[i, int(b["mel_len"][i]):] == 0)


def test_scaled_config4_fp32_matches_oracle(cuda, cfg_all):
    """BASELINE config 4 width (hidden 512, FFN 2048; dh = 256 in the fused attention on the
    bf16 path) -- 2+2 layers keep the fp32 oracle fast; B=2, T_phon=40."""
    import copy
    from fastspeech2.model import FastSpeech2
    from fastspeech2.synthetic import make_batch
    from oracle.fs2_oracle import FastSpeech2Oracle
    kw = copy.deepcopy(cfg_all["model"]["fastspeech2"])
    for k in ("enc_d_model", "enc_k_dim", "enc_v_dim", "dec_d_model", "dec_k_dim", "dec_v_dim"):
        kw[k] = 512
    kw.update(enc_ffn_dim=2048, dec_ffn_dim=2048, enc_num_layers=2, dec_num_layers=2)
    torch.manual_seed(6)
    o = FastSpeech2Oracle(**kw, n_speakers=4).eval()
    torch.manual_seed(6)
    m = FastSpeech2(**kw, n_speakers=4).cuda().eval()
    b = make_batch(B=2, tp_min=40, tp_max=40, seed=11)
    po, lo, pm, lm = _run_both(o, m, cfg_all, b)
    for i in range(7):
        assert rel(pm[i], po[i]) <= 1e-3, i
    assert abs(lm["total_loss"].item() - lo["total_loss"].item()) <= 1e-4 * abs(lo["total_loss"].item())
    go = dict(o.named_parameters())
    errs = [rel(p.grad, go[n].grad) for n, p in m.named_parameters()]
    assert max(errs) <= 1e-2 and float(np.median(errs)) <= 1e-4
    # bf16: fused attention at dh = 256
    torch.manual_seed(6)
    mb = FastSpeech2(**kw, n_speakers=4, act_dtype=torch.bfloat16).cuda().eval()
    from fastspeech2.synthetic import as_tuple
    bt, inten = as_tuple(b)
    g = [t.cuda() for t in bt]
    with torch.no_grad():
        pb = mb(g[0], g[1], g[6], g[4], g[5], intensity=inten.cuda())
    assert rel(pb[0], po[0]) <= 5e-2


def test_bf16_stream_overlap_matches_single_stream(cuda, cfg_all):
    """The bf16 step runs weight gradients on a side stream and the duration / pitch predictor
    chains on an aux stream.  Same model, batch and (dropout-off) inputs with both extra streams
    disabled must give the same outputs (bit-exact: the forward arithmetic is unchanged) and the
    same parameter gradients up to the summation order of the predictor input gradient and the
    split-K atomics (max rel 2e-2 per tensor, cosine >= 0.999): a missing stream dependency shows
    up as stale or garbage gradients here."""
    from fastspeech2.loss import Loss
    from fastspeech2.synthetic import make_batch, as_tuple
    _, m = _pair(cfg_all, dt=torch.bfloat16)
    b = make_batch(B=4, tp_min=60, tp_max=90, seed=3)
    bt, inten = as_tuple(b)
    g = [t.cuda() for t in bt]

    def run():
        for p in m.parameters():
            p.grad = None
        pm = m(g[0], g[1], g[6], g[4], g[5], intensity=inten.cuda())
        lm = Loss(**cfg_all["loss"])(pm, (g[3], g[6], g[4], g[5], g[7], g[2]), 0)
        lm["total_loss"].backward()
        torch.cuda.synchronize()
        return [t.detach().clone() for t in pm[:7]], {n: p.grad.detach().clone()
                                                       for n, p in m.named_parameters()}
    eng = m.engine()
    assert eng._side is not None and eng._aux is not None
    out_a, grad_a = run()
    side, aux = eng._side, eng._aux
    eng._side, eng._aux = None, None
    try:
        out_b, grad_b = run()
    finally:
        eng._side, eng._aux = side, aux
    for x, y in zip(out_a, out_b):
        assert torch.equal(x, y)
    for n in grad_a:
        a, r = grad_a[n].float(), grad_b[n].float()
        assert rel(a, r) <= 2e-2, n
        cos = torch.nn.functional.cosine_similarity(a.flatten(), r.flatten(), dim=0).item()
        assert cos >= 0.999, (n, cos)


def test_graph_replayed_step_equals_eager_step(cuda, cfg_all):
    """FusedTrainer's captured HIP-graph step (one capture per batch shape, dropout seed in the
    kernels' device-resident seed base) against the eager step on the same initial weights and
    batch, dropout on: the first step's loss is bit-identical (same kernels, same masks), later
    steps within 1e-4 (weight-gradient split-K atomics perturb the weights at fp32 rounding),
    and the weights after three steps agree except where a gradient is rounding noise."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
    b = make_batch(B=8, tp_min=60, tp_max=90, seed=21, device="cuda")
    bt, inten = as_tuple(b)
    res = {}
    for graph in (False, True):
        torch.manual_seed(0)
        m = FastSpeech2(**kw, n_speakers=4, act_dtype=torch.bfloat16).cuda().train()
        tr = FusedTrainer(m, lr=1e-4, graph=graph)
        losses = [tr.step(bt, inten).clone() for _ in range(3)]
        torch.cuda.synchronize()
        res[graph] = (torch.stack(losses).cpu(), m._flat.cpu())
        if graph:
            assert len(tr._graphs) == 1
    (le, pe), (lg, pg) = res[False], res[True]
    assert torch.equal(le[0], lg[0])
    assert torch.allclose(le, lg, rtol=1e-4, atol=0)
    assert not torch.equal(le[1], le[2])            # masks / weights do change per step
    dp = (pe - pg).abs()
    assert dp.max().item() <= 3 * 2.1e-4
    assert (dp > 1e-6).float().mean().item() <= 1e-3


@pytest.mark.parametrize("dtname", ["bfloat16", "float32"])
def test_fused_adamw_writes_the_weight_images(cuda, cfg_all, dtname, monkeypatch):
    """fs2_adamw_prep (AdamW fused with the GEMM weight images) == fs2_adamw followed by the
    separate fs2_weight_prep_batched pass, bit for bit: parameters, both moments and every
    Wf / Wb image; the next forward then skips its weight-prep pass."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.optim import FusedAdamW
    from fastspeech2 import optim as optim_mod
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=1, dec_num_layers=1)
    dt = getattr(torch, dtname)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(optim_mod, "_NO_FUSED", not fused)
        torch.manual_seed(0)
        m = FastSpeech2(**kw, n_speakers=4, act_dtype=dt).cuda()
        eng = m.engine()
        eng.prepare_weights()
        g = torch.Generator(device="cuda").manual_seed(5)
        m._gflat.copy_(torch.randn(m._gflat.shape, device="cuda", generator=g) * 1e-3)
        opt = FusedAdamW(m, lr=1e-3)
        for _ in range(2):
            opt.step(grad_scale=0.5)
        eng.prepare_weights()              # unfused: rebuilds the images; fused: already current
        torch.cuda.synchronize()
        res.append((m._flat.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(),
                    {k: (a.clone(), b.clone()) for k, (a, b) in eng.w.items()},
                    eng._prepared_version == (m._param_version, m._flat._version)))
    (p1, m1, v1, w1, ok1), (p2, m2, v2, w2, ok2) = res
    assert ok1 and ok2
    assert torch.equal(p1, p2) and torch.equal(m1, m2) and torch.equal(v1, v2)
    for k in w1:
        assert torch.equal(w1[k][0], w2[k][0]), k
        assert torch.equal(w1[k][1], w2[k][1]), k



def _fresh_grads(cfg_kw, flat, batch, inten, seed):
    """loss and flat gradient of one forward + loss + backward on a NEW model / engine holding
    the weights ``flat`` (no cached images, workspaces or weight tables from earlier steps)"""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    m = FastSpeech2(**cfg_kw, n_speakers=4, act_dtype=torch.bfloat16).cuda().train()
    m._ensure_packed()
    m._flat.copy_(flat)
    m.mark_params_updated()
    tr = FusedTrainer(m, lr=1e-4, graph=False)
    loss = tr.forward_backward(batch, inten, seed=seed)
    torch.cuda.synchronize()
    return loss.cpu(), m._gflat.cpu(), m._layout


@pytest.mark.parametrize("graph", [False, True])
def test_shape_changing_steps_match_fresh_engine(cuda, cfg_all, parity_log, graph):
    """Real training changes (B, T_mel,max) every batch (dataset.py:62-133 pads per batch).
    FusedTrainer steps over batches that grow, shrink after a grow, and come back, so the
    engine's per-layer zero-padded dY images (_dy_image) and the K-major weight-gradient
    images (_km_image) are re-laid-out, grown and re-guarded between steps -- eager, and with
    HIP-graph replay (one captured graph per shape, several resident).  Every step's loss and
    every parameter gradient must equal those of a freshly constructed engine on the same
    weights, batch and dropout seed: bit-exact, except the split-K fp32-atomic weight
    gradients, whose summation order varies (<= 1e-6 of the tensor's max, observed 2.1e-7; values go
    to parity_observed.json).  The caches stay
    bounded: one dY image per layer, one K-major image per (operand, channels)."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
    shapes = [(8, 60, 90, 31), (6, 30, 50, 32), (8, 70, 110, 33), (6, 30, 50, 32), (8, 60, 90, 31)]
    batches = []
    for B, lo, hi, sd in shapes:
        bt, inten = as_tuple(make_batch(B=B, tp_min=lo, tp_max=hi, seed=sd, device="cuda"))
        batches.append((bt, inten))
    tms = [bt[3].shape[1] for bt, _ in batches]
    assert tms[2] > tms[0] > tms[1] and tms[3] == tms[1]       # grow, shrink after a grow
    torch.manual_seed(0)
    m = FastSpeech2(**kw, n_speakers=4, act_dtype=torch.bfloat16).cuda().train()
    tr = FusedTrainer(m, lr=1e-4, graph=graph)
    worst = 0.0
    for i, (bt, inten) in enumerate(batches):
        w0 = m._flat.clone()
        loss = tr.step(bt, inten)                 # forward + loss + backward + AdamW
        torch.cuda.synchronize()
        g_long = m._gflat.cpu()                   # this step's gradients (AdamW leaves them)
        l_f, g_f, layout = _fresh_grads(kw, w0, bt, inten, tr.seed)
        assert torch.equal(loss.cpu(), l_f), (i, loss.cpu(), l_f)
        for name, off, k, _, _ in layout:
            a, b = g_long[off:off + k], g_f[off:off + k]
            if torch.equal(a, b):
                continue
            r = ((a - b).abs().max() / b.abs().max().clamp(min=1e-30)).item()
            worst = max(worst, r)
            assert r <= 1e-6, (i, name, r)
    eng = m.engine()
    L = kw["enc_num_layers"] + kw["dec_num_layers"]
    assert len(eng._img) == L, sorted(eng._img)
    assert len(eng._km) <= 6, sorted(eng._km)
    if graph:
        assert len(tr._graphs) == 3               # one per distinct shape, all resident
    parity_log[f"shape_changing_steps_graph{int(graph)}_max_grad_rel"] = worst


def test_split_adamw_equals_single_update(cuda, cfg_all):
    """FusedTrainer's split AdamW (the decoder / mel-linear / PostNet parameters on the aux
    stream during the encoder backward, the rest after it; engine._adam_launch_late +
    adamw_step_split) against ONE fs2_adamw_prep over everything (engine.adamw_step), bf16, on
    fixed random gradients: parameters, both moments and every Wf / Wb weight image
    bit-identical.  The two range tables are disjoint and together cover every non-GEMM
    parameter; the two weight tables partition the GEMM weights."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.optim import FusedAdamW
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
    res = []
    for split in (False, True):
        torch.manual_seed(0)
        m = FastSpeech2(**kw, n_speakers=4, act_dtype=torch.bfloat16).cuda()
        eng = m.engine()
        eng.prepare_weights()
        opt = FusedAdamW(m, lr=1e-3)
        g = torch.Generator(device="cuda").manual_seed(7)
        for _ in range(2):
            m._gflat.copy_(torch.randn(m._gflat.shape, device="cuda", generator=g) * 1e-3)
            scal = opt.begin_step(0.5)
            if split:
                eng.adam_split = (opt, scal)
                eng._adam_launch_late()
                eng.adam_split = None
                eng.adamw_step_split(opt, scal)
            else:
                eng.adamw_step(opt, *scal)
        torch.cuda.synchronize()
        res.append((m._flat.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(),
                    {k: (a.clone(), b.clone()) for k, (a, b) in eng.w.items()}))
        if split:
            n = m._flat.numel()
            cover = {}
            for late in (False, True):
                mask = torch.zeros(n, dtype=torch.bool)
                for st, ln in eng._adam_range_list(late):
                    mask[st:st + ln] = True
                cover[late] = mask
            assert not (cover[False] & cover[True]).any()
            for name, off, k, _, _ in m._layout:
                if name in eng._gemm_params:
                    continue
                assert bool((cover[False] | cover[True])[off:off + k].all()), name
                assert bool(cover[eng._adam_late(name)][off:off + k].all()), name
            late_w = {nm for nm in eng._wspecs if eng._adam_late(nm)}
            early_w = set(eng._wspecs) - late_w
            assert late_w and early_w and set(eng._wentries) == late_w | early_w
    (p1, m1, v1, w1), (p2, m2, v2, w2) = res
    assert torch.equal(p1, p2) and torch.equal(m1, m2) and torch.equal(v1, v2)
    for k in w1:
        assert torch.equal(w1[k][0], w2[k][0]), k
        assert torch.equal(w1[k][1], w2[k][1]), k


def test_failed_split_step_is_not_half_applied_silently(cuda, cfg_all, monkeypatch):
    """A step whose backward raises: before the late AdamW half was launched the
    optimizer is untouched (step count restored) and the step can be retried; after it, the
    trainer refuses further steps instead of running on a half-updated optimizer."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    kw = dict(cfg_all["model"]["fastspeech2"], enc_num_layers=1, dec_num_layers=1)
    bt, inten = as_tuple(make_batch(B=4, tp_min=30, tp_max=40, seed=5, device="cuda"))
    torch.manual_seed(0)
    m = FastSpeech2(**kw, n_speakers=4, act_dtype=torch.bfloat16).cuda().train()
    tr = FusedTrainer(m, lr=1e-4, graph=False)
    tr.step(bt, inten)
    eng = m.engine()
    assert tr.opt.step_count == 1

    def boom(*a, **k):
        raise RuntimeError("injected")
    monkeypatch.setattr(eng, "backward", boom)
    with pytest.raises(RuntimeError, match="injected"):
        tr.step(bt, inten)
    assert tr.opt.step_count == 1 and not eng._adam_late_done and eng.adam_split is None
    monkeypatch.undo()
    tr.step(bt, inten)                        # retried: a normal step
    assert tr.opt.step_count == 2
    late = eng._adam_launch_late

    def late_then_boom():
        late()
        raise RuntimeError("injected late")
    monkeypatch.setattr(eng, "_adam_launch_late", late_then_boom)
    with pytest.raises(RuntimeError, match="injected late"):
        tr.step(bt, inten)
    monkeypatch.undo()
    with pytest.raises(RuntimeError, match="inconsistent"):
        tr.step(bt, inten)
    torch.cuda.synchronize()
