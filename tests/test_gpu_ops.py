"""GPU: op-level parity of the HIP kernels (through the C ABI) against torch fp32 references
and the oracle's golden fixtures.  Tolerances: fp32 mode rel 1e-4 (GEMM-class) / exact for
integer paths; bf16 mode rel 2e-2 against the fp32 reference of the same bf16 inputs.
"""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DT = [(torch.float32, 0, 1e-4), (torch.bfloat16, 1, 2e-2)]


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


@pytest.mark.parametrize("dt,code,tol", DT)
def test_gemm_epilogue(cuda, dt, code, tol):
    from fastspeech2 import ops
    torch.manual_seed(0)
    M, N, K = 300, 200, 256
    A = torch.randn(M, K, device=cuda).to(dt)
    W = torch.randn(N, K, device=cuda).to(dt)
    bias = torch.randn(N, device=cuda)
    gate = torch.randn(M, N, device=cuda).to(dt)
    res = torch.randn(M, N, device=cuda).to(dt)
    rs = (torch.rand(M, device=cuda) > 0.3).float()
    rs2 = torch.rand(M, device=cuda)
    C = torch.empty(M, N, device=cuda, dtype=dt)
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=code, bias=bias, relu=1, gate=gate, ldg=N, row_scale=rs,
             residual=res, ldr=N, row_scale_post=rs2)
    ref = torch.relu(A.float() @ W.float().t() + bias) * (gate.float() > 0)
    ref = (ref * rs[:, None] + res.float()) * rs2[:, None]
    assert rel(C, ref) < tol


@pytest.mark.parametrize("dt,code,tol", DT)
@pytest.mark.parametrize("KW", [9, 5, 3])
def test_gemm_implicit_conv_fwd_dgrad_wgrad(cuda, dt, code, tol, KW):
    from fastspeech2 import ops
    torch.manual_seed(KW)
    Bn, T, Cin, O = 3, 37, 64, 96
    P = (KW - 1) // 2
    X = torch.randn(Bn, T, Cin, device=cuda).to(dt)
    Wt = torch.randn(O, Cin, KW, device=cuda).to(dt).float()
    Wf = Wt.permute(0, 2, 1).contiguous().to(dt)     # [O][KW][C]
    Wb = Wt.permute(1, 2, 0).contiguous().to(dt)     # [C][KW][O]
    Xr = X.float().clone().requires_grad_(True)
    Wr = Wt.clone().requires_grad_(True)
    out = F.conv1d(F.pad(Xr.transpose(1, 2), (P, P), mode="reflect"), Wr).transpose(1, 2)
    G = torch.randn(out.shape, device=cuda).to(dt).contiguous()
    out.backward(G.float())
    Y = torch.empty(Bn * T, O, device=cuda, dtype=dt)
    ops.gemm(Bn * T, O, KW * Cin, X, Cin, Wf, KW * Cin, Y, O, dt=code, conv=(1, T, KW, Cin))
    assert rel(Y, out.detach().reshape(-1, O)) < tol
    dX = torch.empty(Bn * T, Cin, device=cuda, dtype=dt)
    ops.gemm(Bn * T, Cin, KW * O, G, O, Wb, KW * O, dX, Cin, dt=code, conv=(2, T, KW, O))
    assert rel(dX, Xr.grad.reshape(-1, Cin)) < tol
    dW = torch.zeros(O, Cin, KW, device=cuda)
    K = ops.round_up(Bn * T, 8)
    ops.gemm(O, KW * Cin, K, G, O, X, Cin, dW, Cin * KW, dt=code, a_kmajor=0, b_kmajor=0,
             conv=(3, T, KW, Cin), c_fp32=1, c_conv_kw=KW, kvalid=Bn * T, accumulate=1, split_k=3)
    assert rel(dW, Wr.grad) < tol


@pytest.mark.parametrize("dt,code,tol", DT)
def test_gemm_batched_attention_shapes(cuda, dt, code, tol):
    """S = Q K^T, O = P V, dV = P^T dO, dK = dS^T Q over the packed (B,T,3D) QKV layout."""
    from fastspeech2 import ops
    torch.manual_seed(1)
    B, H, T, dh = 3, 2, 45, 32
    D = H * dh
    ldt = ops.round_up(T, 8)
    QKV = torch.randn(B * T, 3 * D, device=cuda).to(dt)
    q = QKV[:, :D].float().view(B, T, H, dh).permute(0, 2, 1, 3)
    k = QKV[:, D:2 * D].float().view(B, T, H, dh).permute(0, 2, 1, 3)
    v = QKV[:, 2 * D:].float().view(B, T, H, dh).permute(0, 2, 1, 3)
    S = torch.empty(B * H, T, ldt, device=cuda)
    ops.gemm(T, T, dh, QKV, 3 * D, QKV[:, D:], 3 * D, S, ldt, dt=code, c_fp32=1, batch=B * H,
             batch_div=H, strides=(T * 3 * D, dh, T * 3 * D, dh, H * T * ldt, T * ldt, 0, 0))
    assert rel(S[:, :, :T], (q @ k.transpose(-1, -2)).reshape(B * H, T, T)) < tol
    Pm = torch.zeros(B * H, T, ldt, device=cuda, dtype=dt)
    Pm[:, :, :T] = torch.softmax(S[:, :, :T], -1).to(dt)
    O = torch.empty(B * T, D, device=cuda, dtype=dt)
    ops.gemm(T, dh, ldt, Pm, ldt, QKV[:, 2 * D:], 3 * D, O, D, dt=code, b_kmajor=0, kvalid=T,
             batch=B * H, batch_div=H, strides=(H * T * ldt, T * ldt, T * 3 * D, dh, T * D, dh, 0, 0))
    ref = (Pm[:, :, :T].float().view(B, H, T, T) @ v).permute(0, 2, 1, 3).reshape(B * T, D)
    assert rel(O, ref) < tol
    dO = torch.randn(B * T, D, device=cuda).to(dt)
    dQKV = torch.zeros(B * T, 3 * D, device=cuda, dtype=dt)
    ops.gemm(ldt, dh, ldt, Pm, ldt, dO, D, dQKV[:, 2 * D:], 3 * D, dt=code, a_kmajor=0, b_kmajor=0,
             kvalid=T, mvalid=T, batch=B * H, batch_div=H,
             strides=(H * T * ldt, T * ldt, T * D, dh, T * 3 * D, dh, 0, 0))
    dOh = dO.float().view(B, T, H, dh).permute(0, 2, 1, 3)
    ref = (Pm[:, :, :T].float().view(B, H, T, T).transpose(-1, -2) @ dOh)
    assert rel(dQKV[:, 2 * D:], ref.permute(0, 2, 1, 3).reshape(B * T, D)) < tol
    assert torch.all(dQKV[:, :2 * D] == 0)     # mvalid: no spill into neighbouring columns/rows


@pytest.mark.parametrize("dt,code,tol", DT)
@pytest.mark.parametrize("D", [384, 90, 80, 512, 8, 64])
def test_layernorm_fwd_bwd(cuda, dt, code, tol, D):
    """D=384: 16-byte vector kernels; D=90: scalar kernels; bf16 D = 8 / 80 / 512: the rows
    kernels' DPP row sums with 1 / 10 / 64 lanes holding data.  dcol = fused column sum of the
    emitted gradient (the bias gradient of the layer that produced s)."""
    from fastspeech2 import ops
    torch.manual_seed(2)
    M = 300
    x = torch.randn(M, D, device=cuda).to(dt)
    r = torch.randn(M, D, device=cuda).to(dt)
    g = torch.randn(D, device=cuda)
    b = torch.randn(D, device=cuda)
    keep = (torch.rand(M, device=cuda) > 0.2).float()
    pa = torch.randn(M, D, device=cuda).to(dt)
    for tanh in (0, 1):
        y = torch.empty(M, D, device=cuda, dtype=dt)
        s = torch.empty(M, D, device=cuda, dtype=dt)
        mean = torch.empty(M, device=cuda)
        rstd = torch.empty(M, device=cuda)
        ops.ln_fwd(x, D, g, b, 1e-5, y, D, mean, rstd, M, D, dt=code, r=r, ldr=D, s_out=s,
                   do_tanh=tanh, row_mask=keep, post_add=pa, ldp=D)
        sr = (x.float() + r.float()).requires_grad_(True)
        gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
        o = F.layer_norm(sr, (D,), gr, br, 1e-5)
        if tanh:
            o = torch.tanh(o)
        o = o * keep[:, None] + pa.float()
        assert rel(y, o) < tol
        dy = torch.randn(M, D, device=cuda).to(dt)
        o.backward(dy.float())
        ds = torch.empty(M, D, device=cuda, dtype=dt)
        dg = torch.zeros(D, device=cuda)
        db = torch.zeros(D, device=cuda)
        dc = torch.full((D,), 1.0, device=cuda)
        ws = torch.empty(int(ops.ln_ws(M, D)), device=cuda)
        ops.ln_bwd(dy, D, s, D, mean, rstd, g, b, ds, D, M, D, dt=code, ws=ws, do_tanh=tanh,
                   row_mask=keep, dgamma=dg, dbeta=db, dcol=dc)
        assert rel(ds, sr.grad) < tol * 3
        assert rel(dg, gr.grad) < tol * 3
        assert rel(db, br.grad) < tol * 3
        assert rel(dc - 1.0, sr.grad.sum(0)) < tol * 3
        dc2 = torch.zeros(D, device=cuda)          # column sum alone (no gamma/beta)
        ops.ln_bwd(dy, D, s, D, mean, rstd, g, b, ds, D, M, D, dt=code, ws=ws, do_tanh=tanh,
                   row_mask=keep, dcol=dc2)
        assert rel(dc2, sr.grad.sum(0)) < tol * 3


def _keep_ln_np(seed, salt, idx, p):
    """The per-element LayerNorm dropout mask: fs2_keep (fs2_common.h), the pair hash restated by
    _keep_np below, evaluated per element (the attention probabilities draw fs2_attn_keep)."""
    return _keep_np(seed, salt, idx, p)


@pytest.mark.parametrize("M,D", [(300, 384), (1001, 384), (203, 256)])
def test_layernorm_bwd_dropout_gate(cuda, M, D):
    """bf16 LayerNorm backward with output dropout, the relu gate on the input, the
    dropout-masked residual-branch copy dr and all three partial sums (the multi-row kernel's
    cases: ragged row counts per wave, D below a full wave) against torch fp32 on the same
    masks (fs2_keep restated in numpy).  Tolerance rel 2e-2 (bf16 outputs)."""
    from fastspeech2 import ops
    torch.manual_seed(M + D)
    x = torch.randn(M, D, device=cuda).to(torch.bfloat16)
    g = torch.randn(D, device=cuda)
    b = torch.randn(D, device=cuda)
    keep = (torch.rand(M, device=cuda) > 0.2).float()
    y = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    mean = torch.empty(M, device=cuda)
    rstd = torch.empty(M, device=cuda)
    ops.ln_fwd(x, D, g, b, 1e-5, y, D, mean, rstd, M, D, dt=1)
    dy = torch.randn(M, D, device=cuda).to(torch.bfloat16)
    seed, so, sr, po, pr = 7, 3, 11, 0.1, 0.2
    idx = np.arange(M * D, dtype=np.uint64)
    ko = torch.from_numpy(_keep_ln_np(seed, so, idx, po).reshape(M, D)).to(cuda).float()
    kr = torch.from_numpy(_keep_ln_np(seed, sr, idx, pr).reshape(M, D)).to(cuda).float()
    xs = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    o = F.layer_norm(xs, (D,), gr, br, 1e-5)
    gg = dy.float() * keep[:, None] * ko / (1 - po)
    o.backward(gg)
    ds_ref = xs.grad * (x.float() > 0).float()
    dr_ref = ds_ref * kr / (1 - pr)
    ds = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    dr = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    dg = torch.zeros(D, device=cuda)
    db = torch.zeros(D, device=cuda)
    dc = torch.zeros(D, device=cuda)
    ws = torch.empty(int(ops.ln_ws(M, D)), device=cuda)
    ops.ln_bwd(dy, D, x, D, mean, rstd, g, b, ds, D, M, D, dt=1, ws=ws, seed=seed, p_o=po,
               salt_o=so, row_mask=keep, relu_gate_in=1, dr=dr, p_r=pr, salt_r=sr,
               dgamma=dg, dbeta=db, dcol=dc)
    assert rel(ds, ds_ref) < 2e-2
    assert rel(dr, dr_ref) < 2e-2
    assert rel(dg, gr.grad) < 2e-2
    assert rel(db, br.grad) < 2e-2
    assert rel(dc, dr_ref.sum(0)) < 2e-2


@pytest.mark.parametrize("M,npart", [(31264, 3), (6400, 3), (31264, 1), (2000, 2), (777, 3)])
def test_layernorm_bwd_partial_reduction(cuda, M, npart):
    """The bf16 LayerNorm backward's gamma / beta / column-sum reduction over per-block partial
    rows at the decoder's M = 31264 (763 partial rows) down to M = 777: the sums against torch
    fp32 (rel 1e-3 -- fp32 sums over M rows of bf16 inputs), added onto the outputs' previous
    values, with the workspace poisoned with NaN beforehand, and bit-identical over repeated
    calls (fixed summation order)."""
    from fastspeech2 import ops
    torch.manual_seed(M + npart)
    D = 384
    x = torch.randn(M, D, device=cuda).to(torch.bfloat16)
    g = torch.randn(D, device=cuda)
    b = torch.randn(D, device=cuda)
    y = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    mean = torch.empty(M, device=cuda)
    rstd = torch.empty(M, device=cuda)
    ops.ln_fwd(x, D, g, b, 1e-6, y, D, mean, rstd, M, D, dt=1)
    dy = torch.randn(M, D, device=cuda).to(torch.bfloat16)
    ws = torch.full((int(ops.ln_ws(M, D)),), float("nan"), device=cuda)
    ds = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    dr = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    outs = []
    for _ in range(3):
        dg = torch.full((D,), 0.5, device=cuda) if npart >= 2 else None
        db = torch.full((D,), -0.25, device=cuda) if npart >= 2 else None
        dc = torch.full((D,), 2.0, device=cuda) if npart != 2 else None
        ops.ln_bwd(dy, D, x, D, mean, rstd, g, b, ds, D, M, D, dt=1, ws=ws, seed=5, dr=dr,
                   p_r=0.1, salt_r=9, dgamma=dg, dbeta=db, dcol=dc)
        outs.append([t.clone() for t in (dg, db, dc) if t is not None])
    torch.cuda.synchronize()
    for o in outs[1:]:
        for a, c in zip(outs[0], o):
            assert torch.equal(a, c)
    xs = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.layer_norm(xs, (D,), gr, br, 1e-6).backward(dy.float())
    res = outs[0]
    if npart >= 2:
        assert rel(res[0] - 0.5, gr.grad) < 1e-3
        assert rel(res[1] + 0.25, br.grad) < 1e-3
    if npart != 2:        # the column sum of the fp32 dropout-masked gradient (before rounding)
        kr = _keep_ln_np(5, 9, np.arange(M * D, dtype=np.uint64), 0.1).reshape(M, D)
        dr_ref = xs.grad * torch.from_numpy(kr).to(cuda).float() / 0.9
        assert rel(res[-1] - 2.0, dr_ref.sum(0)) < 1e-3


def test_attention_mask_quirk_against_torch_mha(cuda, golden_dir):
    """The golden torch-MHA output (reference mask expression) through our kernels, fp32."""
    from fastspeech2 import ops
    g = np.load(os.path.join(golden_dir, "mask_tiling.npz"))
    x = torch.from_numpy(g["x"]).to(cuda)
    tokens = torch.from_numpy(g["tokens"]).to(cuda)
    B, T, D = x.shape
    H = int(g["nhead"])
    dh = D // H
    ldt = ops.round_up(T, 8)
    w_in = torch.from_numpy(g["in_proj_weight"]).to(cuda)
    b_in = torch.from_numpy(g["in_proj_bias"]).to(cuda)
    w_out = torch.from_numpy(g["out_proj_weight"]).to(cuda)
    b_out = torch.from_numpy(g["out_proj_bias"]).to(cuda)
    X = x.reshape(B * T, D).contiguous()
    QKV = torch.empty(B * T, 3 * D, device=cuda)
    ops.gemm(B * T, 3 * D, D, X, D, w_in, D, QKV, 3 * D, dt=0, bias=b_in)
    S = torch.empty(B * H, T, ldt, device=cuda)
    ops.gemm(T, T, dh, QKV, 3 * D, QKV[:, D:], 3 * D, S, ldt, dt=0, c_fp32=1, batch=B * H,
             batch_div=H, strides=(T * 3 * D, dh, T * 3 * D, dh, H * T * ldt, T * ldt, 0, 0))
    kp = torch.empty(B * T, dtype=torch.uint8, device=cuda)
    ops.keypad_from_tokens(tokens, 0, B * T, kp)
    P = torch.empty(B * H, T, ldt, device=cuda)
    ops.softmax_fwd(S, kp, B, H, T, T, ldt, 1.0 / math.sqrt(dh), 0.0, 0, 1, P, None, dt=0)
    Att = torch.empty(B * T, D, device=cuda)
    ops.gemm(T, dh, ldt, P, ldt, QKV[:, 2 * D:], 3 * D, Att, D, dt=0, b_kmajor=0, kvalid=T,
             batch=B * H, batch_div=H, strides=(H * T * ldt, T * ldt, T * 3 * D, dh, T * D, dh, 0, 0))
    out = torch.empty(B * T, D, device=cuda)
    ops.gemm(B * T, D, D, Att, D, w_out, D, out, D, dt=0, bias=b_out)
    torch.testing.assert_close(out.view(B, T, D).cpu(), torch.from_numpy(g["out"]), rtol=1e-4,
                               atol=1e-5)


@pytest.mark.parametrize("pace", [1.0, 1.1, 0.7])
def test_length_regulator_bit_exact(cuda, golden_dir, pace):
    from fastspeech2 import ops
    g = np.load(os.path.join(golden_dir, "lr_kat.npz"))
    d = torch.from_numpy(g["durs"]).to(cuda)
    B, Tp = d.shape
    exp_fs = g[f"frame_src_{pace}"]
    Tm = exp_fs.shape[1]
    ml = torch.empty(B, dtype=torch.int64, device=cuda)
    cum = torch.empty(B, Tp, dtype=torch.int32, device=cuda)
    fs = torch.empty(B, Tm, dtype=torch.int32, device=cuda)
    ops.lr_index(d, 0, pace, B, Tp, Tm, ml, cum, fs)
    np.testing.assert_array_equal(ml.cpu().numpy(), g[f"mel_len_{pace}"])
    np.testing.assert_array_equal(fs.cpu().numpy(), exp_fs)
    # gather + scatter round trip on integer-valued features: exact
    D = 16
    X = torch.arange(B * Tp * D, device=cuda, dtype=torch.float32).view(B * Tp, D) % 97
    pe = torch.zeros(Tm, D, device=cuda)
    Y = torch.empty(B * Tm, D, device=cuda)
    keep = torch.empty(B * Tm, device=cuda)
    ops.lr_gather(X, fs, pe, B, Tp, Tm, D, Y, keep, dt=0)
    ref = torch.zeros(B, Tm, D)
    fsc = torch.from_numpy(exp_fs).long()
    for b in range(B):
        v = fsc[b] >= 0
        ref[b, v] = X.cpu().view(B, Tp, D)[b, fsc[b, v]]
    assert torch.equal(Y.cpu().view(B, Tm, D), ref)
    dX = torch.empty(B * Tp, D, device=cuda)
    ops.lr_scatter(Y, cum, keep, B, Tp, Tm, D, dX, dt=0)
    counts = torch.zeros(B, Tp)
    n = (np.float32(pace) * g["durs"].astype(np.float32)).astype(np.int64)
    assert torch.equal(dX.cpu().view(B, Tp, D), X.cpu().view(B, Tp, D) * torch.from_numpy(n)[..., None].float())


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("B,Tp,D", [(32, 200, 384), (3, 1024, 1104), (2, 999, 20), (5, 7, 36)])
def test_length_regulator_rows(cuda, dt, code, B, Tp, D):
    """LengthRegulator index / gather / scatter at the bench shape and at the edges of the
    row-vector kernels: T_p = 1024 (four phonemes per scan thread) with rows of more than one
    64-lane column sweep (D = 1104), D = 20 (bf16: the element-wise fallback) and D = 36.
    lr_index against the oracle bit for bit; gather exact (a copy plus the fp32 positional
    row, rounded once); scatter against an fp32 segment sum in frame order (rel 1e-6 in fp32,
    one bf16 rounding in bf16)."""
    from fastspeech2 import ops
    from oracle.lr_oracle import lr_index_np
    g = torch.Generator().manual_seed(B * Tp + D)
    d = torch.randint(0, 9, (B, Tp), generator=g)
    d[0, Tp // 2:] = 0
    ml_ref, fs_ref = lr_index_np(d.numpy(), 1.0)
    Tm = fs_ref.shape[1]
    dc = d.to(cuda)
    ml = torch.empty(B, dtype=torch.int64, device=cuda)
    cum = torch.empty(B, Tp, dtype=torch.int32, device=cuda)
    fs = torch.empty(B, Tm, dtype=torch.int32, device=cuda)
    ops.lr_index(dc, 0, 1.0, B, Tp, Tm, ml, cum, fs)
    np.testing.assert_array_equal(ml.cpu().numpy(), ml_ref)
    np.testing.assert_array_equal(fs.cpu().numpy(), fs_ref)
    assert torch.equal(cum.cpu().long(), d.cumsum(1))
    X = torch.randn(B * Tp, D, generator=g).to(dt).to(cuda)
    pe = torch.randn(Tm, D, generator=g).to(cuda)
    Y = torch.empty(B * Tm, D, device=cuda, dtype=dt)
    keep = torch.empty(B * Tm, device=cuda)
    ops.lr_gather(X, fs, pe, B, Tp, Tm, D, Y, keep, dt=code)
    fsl = fs.long().view(B, Tm)
    valid = fsl >= 0
    src = (torch.arange(B, device=cuda)[:, None] * Tp + fsl.clamp(min=0)).view(-1)
    ref = ((X.float()[src].view(B, Tm, D) + pe[None]) * valid[..., None]).to(dt)
    assert torch.equal(Y.view(B, Tm, D), ref)
    assert torch.equal(keep.view(B, Tm), valid.float())
    dY = torch.randn(B * Tm, D, generator=g).to(dt).to(cuda)
    dX = torch.empty(B * Tp, D, device=cuda, dtype=dt)
    ops.lr_scatter(dY, cum, keep, B, Tp, Tm, D, dX, dt=code)
    seg = (torch.arange(B, device=cuda)[:, None] * Tp + fsl.clamp(min=0)).view(-1)
    w = (dY.float() * keep[:, None])[valid.view(-1)]
    ref = torch.zeros(B * Tp, D, device=cuda).index_add_(0, seg[valid.view(-1)], w)
    assert rel(dX, ref.to(dt)) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("B,T,D,E,ldc", [(32, 200, 384, 5, 776), (3, 17, 1104, 0, 2208),
                                         (2, 9, 20, 3, 48), (2, 9, 21, 2, 44)])
def test_concat_fwd(cuda, dt, code, B, T, D, E, ldc):
    """fs2_concat_fwd (model.py:352-358): cat = [feats, spk_emb[spk[b]], intensity, 0-pad] per
    row, exact.  Bench shape (ldc padded to a 16-element multiple), rows wider than one
    64-lane sweep, D = 20 (bf16: element-wise fallback) and D = 21 (odd: fallback in both)."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + D)
    feats = torch.randn(B * T, D, device=cuda).to(dt)
    table = torch.randn(4, D, device=cuda)
    spk = torch.randint(0, 4, (B,), device=cuda)
    inten = torch.rand(B * T, E, device=cuda) if E else None
    cat = torch.full((B * T, ldc), 7.0, device=cuda, dtype=dt)
    ops.concat_fwd(feats, table, spk, inten, B, T, D, E, cat, ldc, dt=code)
    ref = torch.zeros(B * T, ldc, device=cuda)
    ref[:, :D] = feats.float()
    ref[:, D:2 * D] = table[spk].repeat_interleave(T, 0)
    if E:
        ref[:, 2 * D:2 * D + E] = inten
    assert torch.equal(cat, ref.to(dt))


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("B,T,D,KW", [(32, 200, 384, 3), (3, 37, 1104, 5), (2, 9, 20, 8),
                                      (4, 5, 36, 1)])
def test_embed1d_fwd(cuda, dt, code, B, T, D, KW):
    """fs2_embed1d_fwd (pitch / energy embedding conv fused with the residual add, model.py:
    226-240,384-403) against torch's reflect-padded conv1d in fp32 (rel 1e-6 in fp32, one bf16
    rounding in bf16)."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + D + KW)
    a = torch.randn(B, T, device=cuda)
    base = torch.randn(B * T, D, device=cuda).to(dt)
    W = torch.randn(D, KW, device=cuda)
    bias = torch.randn(D, device=cuda)
    out = torch.empty(B * T, D, device=cuda, dtype=dt)
    ops.embed1d_fwd(base, a, W, bias, B, T, D, KW, out, dt=code)
    P = (KW - 1) // 2
    x = F.pad(a[:, None, :], (P, KW - 1 - P), mode="reflect") if KW > 1 else a[:, None, :]
    y = F.conv1d(x, W[:, None, :], bias).transpose(1, 2).reshape(B * T, D)
    assert rel(out, (base.float() + y).to(dt)) < (1e-6 if dt == torch.float32 else 1e-2)


def test_length_regulator_float_durations(cuda, golden_dir):
    from fastspeech2 import ops
    g = np.load(os.path.join(golden_dir, "lr_kat.npz"))
    d = torch.from_numpy(g["durs_f"]).to(cuda)
    B, Tp = d.shape
    Tm = g["frame_src_f"].shape[1]
    ml = torch.empty(B, dtype=torch.int64, device=cuda)
    cum = torch.empty(B, Tp, dtype=torch.int32, device=cuda)
    fs = torch.empty(B, Tm, dtype=torch.int32, device=cuda)
    ops.lr_index(d, 1, 1.0, B, Tp, Tm, ml, cum, fs)
    np.testing.assert_array_equal(fs.cpu().numpy(), g["frame_src_f"])


def test_avg_over_durations_bit_exact(cuda, golden_dir):
    from fastspeech2 import ops
    g = np.load(os.path.join(golden_dir, "avg_kat.npz"))
    v = torch.from_numpy(g["values"]).to(cuda)
    d = torch.from_numpy(g["durs"]).to(cuda)
    B, Tm = v.shape
    Tp = d.shape[1]
    out = torch.empty(B, Tp, device=cuda)
    ops.avg_over_durations(v, Tm, d, B, Tp, out, torch.empty(int(ops.avg_ws(B, Tm)), device=cuda))
    np.testing.assert_array_equal(out.cpu().numpy(), g["avg"])


@pytest.mark.parametrize("kind", ["pitch", "wide", "nonfinite", "zeros"])
def test_avg_over_durations_scan_paths(cuda, kind):
    """fs2_avg_over_durations at the bench shape (B = 32, T_mel = 1000, T_p = 200) against the
    oracle (oracle/lr_oracle.py, torch-CPU sequential double cumsum), bit for bit, through both
    scan paths: "pitch" (normalised values, ~30 % unvoiced zeros: the exactness-gated parallel
    scan), "wide" (rows mixing 1e30 and 1e-30: additions round, so the gate sends them to the
    sequential scan), "nonfinite" (an inf / nan row: sequential), "zeros" (all-zero rows)."""
    from fastspeech2 import ops
    from oracle.lr_oracle import avg_over_durations_np
    rng = np.random.default_rng({"pitch": 1, "wide": 2, "nonfinite": 3, "zeros": 4}[kind])
    B, Tm, Tp = 32, 1000, 200
    v = rng.standard_normal((B, Tm)).astype(np.float32)
    v[rng.random((B, Tm)) < 0.3] = 0.0
    if kind == "wide":
        v[::2, ::7] *= np.float32(1e30)
        v[::2, 3::7] *= np.float32(1e-30)
    elif kind == "nonfinite":
        v[3, 10] = np.inf
        v[5, 20] = np.nan
        v[7, 30], v[7, 31] = np.inf, -np.inf
    elif kind == "zeros":
        v[::3] = 0.0
    d = rng.integers(0, 9, (B, Tp)).astype(np.int64)
    d[1, 150:] = 0
    out = torch.empty(B, Tp, device=cuda)
    ops.avg_over_durations(torch.from_numpy(v).to(cuda), Tm, torch.from_numpy(d).to(cuda), B, Tp,
                           out, torch.empty(int(ops.avg_ws(B, Tm)), device=cuda))
    np.testing.assert_array_equal(out.cpu().numpy(), avg_over_durations_np(v, d))


@pytest.mark.parametrize("dt,B,Tp,ties", [(torch.float32, 3, 20, False), (torch.bfloat16, 3, 20, False),
                                          (torch.float32, 4, 60, True), (torch.bfloat16, 4, 60, True),
                                          (torch.float32, 300, 8, False)])
def test_fused_loss_vs_oracle(cuda, dt, B, Tp, ties):
    """fs2_loss_fwd_bwd vs LossOracle (loss.py:101-186).  ``ties``: predictions clamped so
    their max / min repeat many times across the min-max kernels' 16 chunks per utterance --
    the SSIM normalisation gradient is split over every tie (torch amax / amin semantics).
    B = 300: more utterances than one 256-thread finalize block (strided per-utterance sums)."""
    from fastspeech2.loss import fused_loss
    from oracle.fs2_oracle import LossOracle
    torch.manual_seed(4 + Tp)
    NM = 80
    d = torch.randint(1, 6, (B, Tp))
    d[1, Tp * 3 // 4:] = 0
    d[2, Tp // 2 - 1:] = 0
    mel_len = d.sum(1)
    Tm = int(mel_len.max())
    phon_len = (d > 0).sum(1)
    tgt = torch.randn(B, Tm, NM) * 2 - 4
    for b in range(B):
        tgt[b, mel_len[b]:] = 0
    mel = (torch.randn(B, Tm, NM) * 2 - 4)
    if ties:
        mel = mel.clamp(-6.0, -2.5)
    post = mel + 0.1 * torch.randn(B, Tm, NM)
    for b in range(B):
        mel[b, mel_len[b]:] = 0
    ld, pp, pe = torch.randn(B, Tp), torch.randn(B, Tp), torch.randn(B, Tp)
    ap, ae = torch.randn(B, Tp), torch.randn(B, Tp)
    mel, post, ld, pp, pe = [t.to(dt).float() for t in (mel, post, ld, pp, pe)]
    leaves = [t.clone().requires_grad_(True) for t in (mel, post, ld, pp, pe)]
    crit = LossOracle(True, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0)
    lo = crit((leaves[0], leaves[1], leaves[2], leaves[3].unsqueeze(-1), ap.unsqueeze(-1),
               leaves[4].unsqueeze(-1), ae.unsqueeze(-1), mel_len), (tgt, d, None, None, mel_len,
                                                                      phon_len), 0)
    lo["total_loss"].backward()
    c = lambda t: t.to(cuda)
    loss, grads = fused_loss(c(mel).to(dt), c(post).to(dt), c(ld).to(dt), c(pp).to(dt),
                             c(pe).to(dt), c(tgt), c(d), c(ap), c(ae), c(mel_len), c(phon_len),
                             (1.0,) * 6)
    keys = ["total_loss", "ssim_loss", "mel_loss", "postnet_mel_loss", "dur_loss", "pitch_loss",
            "energy_loss"]
    got = loss.cpu()
    for i, k in enumerate(keys):
        assert abs(got[i].item() - lo[k].item()) <= 1e-4 * max(1.0, abs(lo[k].item())), k
    gtol = 1e-4 if dt == torch.float32 else 2e-2
    for gg, leaf in zip(grads, leaves):
        assert rel(gg.cpu().reshape(leaf.shape), leaf.grad) < gtol


@pytest.mark.parametrize("n", [10000, 10003])
def test_adamw_matches_torch(cuda, n):
    """16-byte vector kernel over n // 4 groups + scalar tail (n = 10003)."""
    from fastspeech2 import ops
    torch.manual_seed(5)
    p0 = torch.randn(n, device=cuda)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, foreach=False)
    p, m, v = p0.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    for t in range(1, 4):
        g = torch.randn(n, device=cuda)
        ref.grad = g.clone()
        opt.step()
        b1, b2, lr, wd = 0.9, 0.999, 1e-3, 1e-2
        ops.adamw(p, g, m, v, n, 1 - lr * wd, 1 - b1, b2, 1 - b2, lr / (1 - b1 ** t),
                  (1 - b2 ** t) ** 0.5, 1e-8, 1.0)
    torch.testing.assert_close(p, ref.detach(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dt,code,tol", DT)
@pytest.mark.parametrize("KW,T", [(9, 37), (5, 6), (3, 2)])
@pytest.mark.parametrize("split", [1, 4])
def test_conv_dgrad_shift_plus_fold(cuda, dt, code, tol, KW, T, split):
    """conv_mode 4 (zero-padded shift conv over T+2P rows) + fs2_conv_fold == reflect-conv
    data gradient, with the fused epilogue ((dX * rs) + residual) * rs2.  split > 1: split-K
    partials stored to separate slices (a shortened split zeroes the unused ones; the slices
    start as NaN to prove it) and summed by the fold."""
    from fastspeech2 import ops
    torch.manual_seed(KW + T)
    Bn, Cin, O = 3, 64, 96
    P = (KW - 1) // 2
    Wt = torch.randn(O, Cin, KW, device=cuda).to(dt).float()
    Wb = Wt.permute(1, 2, 0).contiguous().to(dt)
    Xr = torch.randn(Bn, T, Cin, device=cuda).requires_grad_(True)
    out = F.conv1d(F.pad(Xr.transpose(1, 2), (P, P), mode="reflect"), Wt).transpose(1, 2)
    G = torch.randn(out.shape, device=cuda).to(dt).contiguous()
    out.backward(G.float())
    Mp = Bn * (T + 2 * P)
    Xpad = torch.full((split, Mp, Cin), float("nan"), device=cuda)
    ops.gemm(Mp, Cin, KW * O, G, O, Wb, KW * O, Xpad, Cin, dt=code, conv=(4, T, KW, O), c_fp32=1,
             split_k=split, split_stride=Mp * Cin if split > 1 else 0)
    res = torch.randn(Bn * T, Cin, device=cuda).to(dt)
    rs = (torch.rand(Bn * T, device=cuda) > 0.3).float()
    rs2 = torch.rand(Bn * T, device=cuda)
    dX = torch.empty(Bn * T, Cin, device=cuda, dtype=dt)
    ops.conv_fold(Xpad, Bn, T, P, Cin, dX, Cin, dt=code, residual=res, ldr=Cin, row_scale=rs,
                  row_scale_post=rs2, nsplit=split, split_stride=Mp * Cin)
    ref = (Xr.grad.reshape(-1, Cin) * rs[:, None] + res.float()) * rs2[:, None]
    assert rel(dX, ref) < tol


@pytest.mark.parametrize("split", [1, 3])
def test_conv_fold_vector_form_bit_exact(cuda, split):
    """the 8-channel, 16-byte-access bf16 fold (conv_fold8_kernel) equals the 4-channel form
    (taken when the output stride is not a multiple of 8) bit for bit, with residual and both
    row scales, at the decoder's T = 977 / P = 4"""
    from fastspeech2 import ops
    torch.manual_seed(11)
    Bn, T, P, C = 4, 977, 4, 384
    Mp = Bn * (T + 2 * P)
    Xpad = torch.randn(split, Mp, C, device=cuda)
    res = torch.randn(Bn * T, C + 8, device=cuda).to(torch.bfloat16)
    rs = (torch.rand(Bn * T, device=cuda) > 0.3).float()
    rs2 = torch.rand(Bn * T, device=cuda)
    a = torch.empty(Bn * T, C, device=cuda, dtype=torch.bfloat16)
    b = torch.empty(Bn * T, C + 4, device=cuda, dtype=torch.bfloat16)
    for out, ldo in ((a, C), (b, C + 4)):
        ops.conv_fold(Xpad, Bn, T, P, C, out, ldo, dt=1, residual=res, ldr=C + 8, row_scale=rs,
                      row_scale_post=rs2, nsplit=split, split_stride=Mp * C)
    assert torch.equal(a, b[:, :C])


@pytest.mark.parametrize("Bn,T", [(32, 640), (1, 640), (32, 200), (32, 977)])
def test_gemm_big_tile_paths_bf16(cuda, Bn, T):
    """BASELINE-sized GEMMs that take the 256x128 LDS-DMA kernel (gemm_big_kernel): implicit
    reflect conv k=9 forward with bias+ReLU, zero-padded shift-conv data gradient + fold, and
    the weight gradient into the [O][KW][C] layout -- split-K with atomics at Bn=32, the
    single-split vector accumulate epilogue at Bn=1; T=200 (encoder) takes the split-slice
    data gradient; T=977 is the bench's decoder shape (M = 31264: a partial last 256-row tile,
    utterance boundaries inside tiles).  bf16 inputs, fp32 reference on the same
    bf16 values, rel 2e-2."""
    from fastspeech2 import ops
    torch.manual_seed(Bn)
    Cin, O, KW = 384, 1536, 9
    P = (KW - 1) // 2
    M = Bn * T
    X = torch.randn(Bn, T, Cin, device=cuda).to(torch.bfloat16)
    Wt = (torch.randn(O, Cin, KW, device=cuda) * 0.05).to(torch.bfloat16).float()
    bias = torch.randn(O, device=cuda)
    Wf = Wt.permute(0, 2, 1).contiguous().to(torch.bfloat16)
    Wb = Wt.permute(1, 2, 0).contiguous().to(torch.bfloat16)
    Xr = X.float().clone().requires_grad_(True)
    Wr = Wt.clone().requires_grad_(True)
    pre = F.conv1d(F.pad(Xr.transpose(1, 2), (P, P), mode="reflect"), Wr, bias).transpose(1, 2)
    out = torch.relu(pre)
    G = torch.randn(out.shape, device=cuda).to(torch.bfloat16).contiguous()
    pre.backward(G.float())          # data/weight gradients of the conv itself (no ReLU gate)
    Y = torch.empty(M, O, device=cuda, dtype=torch.bfloat16)
    ops.gemm(M, O, KW * Cin, X, Cin, Wf, KW * Cin, Y, O, dt=1, conv=(1, T, KW, Cin), bias=bias,
             relu=1)
    assert rel(Y, out.detach().reshape(-1, O)) < 2e-2
    Mp = Bn * (T + 2 * P)
    from fastspeech2.engine import dgrad_split
    split = dgrad_split(Mp, Cin, KW * O, 1)
    Xpad = torch.empty(split, Mp, Cin, device=cuda)
    ops.gemm(Mp, Cin, KW * O, G, O, Wb, KW * O, Xpad, Cin, dt=1, conv=(4, T, KW, O), c_fp32=1,
             split_k=split, split_stride=Mp * Cin if split > 1 else 0)
    dX = torch.empty(M, Cin, device=cuda, dtype=torch.bfloat16)
    ops.conv_fold(Xpad, Bn, T, P, Cin, dX, Cin, dt=1, nsplit=split, split_stride=Mp * Cin)
    assert rel(dX, Xr.grad.reshape(-1, Cin)) < 2e-2
    dW = torch.full((O, KW, Cin), 0.5, device=cuda)        # accumulates onto existing values
    ops.gemm(O, KW * Cin, ops.round_up(M, 8), G, O, X, Cin, dW, KW * Cin, dt=1, a_kmajor=0,
             b_kmajor=0, conv=(3, T, KW, Cin), c_fp32=1, kvalid=M, accumulate=1)
    assert rel(dW - 0.5, Wr.grad.permute(0, 2, 1)) < 2e-2


@pytest.mark.parametrize("Bn,T,O,Cin,KW,ns", [(32, 977, 1536, 384, 9, 3), (32, 200, 1536, 384, 9, 2),
                                              (4, 77, 600, 72, 9, 1), (32, 977, 512, 512, 5, 2),
                                              (3, 130, 520, 128, 5, 3)])
def test_wgrad_conv3_slices(cuda, Bn, T, O, Cin, KW, ns):
    """Implicit-reflect-conv weight gradients written as split-K fp32 planes (split_stride, the
    engine's path for the large FFN / PostNet weights) -- the 256x256 MN-major kernel
    (gemm256_kernel<false, false, 0, 1>) at the decoder / encoder FFN conv1 shapes, a
    PostNet-like k=5 shape, and
    ragged ones (M, N not multiples of 256, utterance boundaries inside K-tiles, a slice count
    that leaves no plane empty and one plane (ns = 1)).  The summed planes equal the fp32
    reference of the same bf16 values (rel 2e-2); planes cover every output element exactly."""
    from fastspeech2 import ops
    torch.manual_seed(T + O)
    P = (KW - 1) // 2
    M = Bn * T
    X = torch.randn(Bn, T, Cin, device=cuda).to(torch.bfloat16)
    G = torch.randn(M, O, device=cuda).to(torch.bfloat16)
    cols = []
    idx = torch.arange(T, device=cuda)
    for j in range(KW):
        src = idx + j - P
        src = torch.where(src < 0, -src, src)
        src = torch.where(src >= T, 2 * (T - 1) - src, src)
        cols.append(X[:, src, :].float())
    Xcol = torch.cat(cols, dim=2).reshape(M, KW * Cin)
    ref = G.float().t() @ Xcol                              # [O][KW*C]
    K = ops.round_up(M, 8)
    stride = O * KW * Cin
    ws = torch.full((ns, O, KW * Cin), float("nan"), device=cuda)
    ops.gemm(O, KW * Cin, K, G, O, X, Cin, ws, KW * Cin, dt=1, a_kmajor=0, b_kmajor=0,
             conv=(3, T, KW, Cin), c_fp32=1, kvalid=M, nvalid=KW * Cin, split_k=ns,
             split_stride=stride if ns > 1 else 0)
    torch.cuda.synchronize()
    assert torch.isfinite(ws).all()
    assert rel(ws.sum(0), ref) < 2e-2


@pytest.mark.parametrize("Bn,T,O,Cin,KW,S", [(32, 977, 1536, 384, 9, 3), (32, 200, 1536, 384, 9, 3),
                                             (4, 77, 600, 72, 9, 1), (3, 130, 520, 128, 5, 2),
                                             (2, 50, 1024, 80, 5, 4)])
def test_wgrad_kmajor_padded_images(cuda, Bn, T, O, Cin, KW, S):
    """conv_mode 6 (the engine's FFN conv1 weight gradient): fs2_pad_transpose writes dY
    (zero pads) and X (reflect pads) channel-major over the padded token domain, exactly the
    torch construction, and dY's column sums (the fused bias gradient, rel 1e-5); the K-major GEMM over them (gemm_ps_kernel<0, 64, 0, 1>, tap j = a
    column shift j - P, 2-byte-aligned LDS-DMA sources, split-K fp32 slices) equals the fp32
    reference of the same bf16 values (rel 1e-3: both sum exact bf16 products in fp32).  Shapes:
    decoder / encoder FFN conv1, ragged M / N / K (tile edges, utterance boundaries inside
    K-tiles, odd T), one slice, four slices."""
    from fastspeech2 import ops
    torch.manual_seed(T + O + S)
    P = (KW - 1) // 2
    M = Bn * T
    Tp = T + 2 * P
    X = torch.randn(Bn, T, Cin, device=cuda).to(torch.bfloat16)
    G = torch.randn(M, O, device=cuda).to(torch.bfloat16)
    idx = torch.arange(T, device=cuda)
    cols = []
    for j in range(KW):
        src = idx + j - P
        src = torch.where(src < 0, -src, src)
        src = torch.where(src >= T, 2 * (T - 1) - src, src)
        cols.append(X[:, src, :].float())
    ref = G.float().t() @ torch.cat(cols, dim=2).reshape(M, KW * Cin)
    Kp = ops.round_up(Bn * Tp, 64 * S)
    # images with zeroed 64-element guards before row 0 and after the last row
    gy = torch.full((O * Kp + 128,), float("nan"), device=cuda).to(torch.bfloat16)
    gx = torch.zeros(Cin * Kp + 128, device=cuda).to(torch.bfloat16)
    dYT, XT = gy[64:64 + O * Kp], gx[64:64 + Cin * Kp]
    bias = torch.full((O,), 0.25, device=cuda)                # the fused column sum accumulates
    pws = torch.empty(ops.pad_transpose_ws(Kp, O), device=cuda)
    ops.pad_transpose(G, O, Bn, T, O, P, 0, dYT, Kp, Kp, dt=1, colsum=bias, ws=pws)
    assert rel(bias - 0.25, G.float().sum(0)) < 1e-5
    ops.pad_transpose(X, Cin, Bn, T, Cin, P, 1, XT, Kp, Kp, dt=1)
    ipad = torch.arange(-P, T + P, device=cuda)
    rpad = torch.where(ipad < 0, -ipad, ipad)
    rpad = torch.where(rpad >= T, 2 * (T - 1) - rpad, rpad)
    xi = torch.zeros(Cin, Kp, device=cuda, dtype=torch.bfloat16)
    xi[:, :Bn * Tp] = X[:, rpad, :].reshape(Bn * Tp, Cin).t()
    gi = torch.zeros(Bn, Tp, O, device=cuda, dtype=torch.bfloat16)
    gi[:, P:P + T] = G.reshape(Bn, T, O)
    yi = torch.zeros(O, Kp, device=cuda, dtype=torch.bfloat16)
    yi[:, :Bn * Tp] = gi.reshape(Bn * Tp, O).t()
    assert torch.equal(XT.reshape(Cin, Kp), xi)
    assert torch.equal(dYT.reshape(O, Kp), yi)
    stride = O * KW * Cin
    ws = torch.full((S, O, KW * Cin), float("nan"), device=cuda)
    ops.gemm(O, KW * Cin, Kp, dYT, Kp, XT, Kp, ws, KW * Cin, dt=1, conv=(6, T, KW, Cin),
             c_fp32=1, split_k=S, split_stride=stride if S > 1 else 0)
    torch.cuda.synchronize()
    assert torch.isfinite(ws).all()
    assert rel(ws.sum(0), ref) < 1e-3


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
def test_add3_mask_rows(cuda, dt, code):
    """fs2_add3_mask_rows: X = (X + Y + Z) * keep[row] in fp32 with one rounding, row pitch > D."""
    from fastspeech2 import ops
    torch.manual_seed(5)
    M, D, ld = 301, 384, 392
    X, Y, Z = (torch.randn(M, ld, device=cuda).to(dt) for _ in range(3))
    keep = (torch.rand(M, device=cuda) > 0.3).float()
    ref = ((X.float() + Y.float()) + Z.float()) * keep[:, None]
    X0 = X.clone()
    ops.add3_mask_rows(X, Y, Z, ld, keep, M, D, dt=code)
    assert torch.equal(X[:, :D], ref[:, :D].to(dt))
    assert torch.equal(X[:, D:], X0[:, D:])


@pytest.mark.parametrize("M,N,K,c32", [(1000, 1536, 2048, 0), (31264, 1536, 3456, 0),
                                        (700, 384, 4096, 1), (300, 200, 2056, 1),
                                        (6400, 1536, 3456, 0), (2000, 384, 8192, 1),
                                        (5000, 700, 3000, 1), (10752, 1536, 2048, 1)])
def test_gemm_persistent_long_k(cuda, M, N, K, c32):
    """Long-K K-major GEMMs take the persistent 256 x 256 / 256 x 192 kernel (gemm_ps_kernel):
    both tile widths, partial row / column tiles, a partial last K-tile (K = 2056), bf16 and
    fp32 outputs, the bias + ReLU + row-scale epilogue; fp32 reference on the same bf16 values.
    The last three: the encoder FFN conv1 shape as a plain GEMM (one round of 200 tiles), 16
    tiles at K = 8192, and a ragged one (partial rows, columns and last K-tile)."""
    from fastspeech2 import ops
    torch.manual_seed(M + N)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda)
    rs = (torch.rand(M, device=cuda) > 0.2).float()
    rs2 = torch.rand(M, device=cuda) + 0.5
    ref = torch.relu(A.float() @ W.float().t() + bias) * rs[:, None] * rs2[:, None]
    C = torch.full((M, N), float("nan"), device=cuda, dtype=torch.float32 if c32 else torch.bfloat16)
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, c_fp32=c32, bias=bias, relu=1, row_scale=rs,
             row_scale_post=rs2)
    assert torch.isfinite(C.float()).all()
    assert rel(C, ref) < 1e-2
    # plain (no epilogue operands), output written with a row pitch > N
    C2 = torch.zeros(M, N + 8, device=cuda, dtype=torch.bfloat16)
    ops.gemm(M, N, K, A, K, W, K, C2, N + 8, dt=1)
    assert rel(C2[:, :N], A.float() @ W.float().t()) < 1e-2
    assert (C2[:, N:] == 0).all()


@pytest.mark.parametrize("M,N,K,c32,crow", [(31264, 1536, 3456, 0, None),
                                             (31000, 1000, 2048, 1, (300, 8)),
                                             (20000, 520, 2048, 1, None),
                                             (6656, 1536, 3456, 0, (200, -8)),
                                             (31520, 384, 4096, 1, None),
                                             (12000, 776, 2304, 0, (200, -4))])
def test_gemm_four_wave(cuda, M, N, K, c32, crow):
    """Plain K-major GEMMs with N >= 384, K % 128 == 0, K >= 2048, M >= 2048 and >= 160 tiles
    take the 4-wave kernel (gemm_w4b_kernel: 128 x 128 or 128 x 96 per wave, 64-deep stages in
    two LDS-DMA slots): the decoder FFN conv1 forward shape (256 x 256 tiles), the encoder's
    over its padded image and the decoder conv1 data gradient's N = 384 (256 x 192 tiles),
    partial row and column tiles on both tile widths (M = 31000 / 20000 / 12000, N = 1000 / 520
    / 776: the zero-filled operand tails), both output types, bias + ReLU, and both c_row
    remaps (gaps inserted every 300 rows; pad rows dropped).  NaN-filled outputs: rows the
    remap skips stay NaN, every other row is written.  fp32 reference on the same bf16 values,
    rel 1e-2."""
    from fastspeech2 import ops
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda)
    ref = torch.relu(A.float() @ W.float().t() + bias)
    odt = torch.float32 if c32 else torch.bfloat16
    m = torch.arange(M, device=cuda)
    if crow is None:
        rows, keep = m, torch.ones(M, dtype=torch.bool, device=cuda)
        nrows = M
    elif crow[1] > 0:
        rows, keep = m + (m // crow[0]) * crow[1], torch.ones(M, dtype=torch.bool, device=cuda)
        nrows = M + (M // crow[0] + 1) * crow[1]
    else:
        L = crow[0] - crow[1]
        rows, keep = (m // L) * crow[0] + m % L, (m % L) < crow[0]
        nrows = (M // L + 1) * crow[0]
    C = torch.full((nrows, N), float("nan"), device=cuda, dtype=odt)
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, c_fp32=c32, bias=bias, relu=1,
             **({"c_row": crow} if crow else {}))
    torch.cuda.synchronize()
    written = torch.zeros(nrows, dtype=torch.bool, device=cuda)
    written[rows[keep]] = True
    assert torch.isfinite(C[written].float()).all()
    assert torch.isnan(C[~written].float()).all()
    assert rel(C[rows[keep]], ref[keep]) < 1e-2


@pytest.mark.parametrize("M,N,K,op", [(31264, 384, 1152, "residual"), (31264, 1536, 384, "gate"),
                                       (26000, 400, 384, "residual"), (26000, 400, 1000, "gate"),
                                       (31264, 384, 1536, None), (26000, 1152, 384, None)])
def test_gemm_persistent_short_k(cuda, M, N, K, op):
    """Short-K GEMMs whose 256-row tiles fill a round of the CUs take the persistent kernel
    (gemm_ps_kernel): the decoder's QKV data gradient (+ residual), FFN conv2 data gradient
    (ReLU gate), conv2 forward and QKV projection shapes, and ragged ones (partial row / column
    tiles, K not a multiple of 64).  The gate / residual instance loads its operand in the
    tile's last K-tile; bias + row scales come from the LDS-staged epilogue operands.  fp32
    reference on the same bf16 values, rel 1e-2."""
    from fastspeech2 import ops
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda)
    rs = (torch.rand(M, device=cuda) > 0.2).float()
    rs2 = torch.rand(M, device=cuda) + 0.5
    E = torch.randn(M, N + 8, device=cuda).to(torch.bfloat16)     # operand with a row pitch > N
    x = A.float() @ W.float().t() + bias
    kw = {}
    if op == "gate":
        x = torch.where(E[:, :N].float() > 0, x, torch.zeros_like(x)) * rs[:, None]
        kw = dict(gate=E, ldg=N + 8)
    elif op == "residual":
        x = x * rs[:, None] + E[:, :N].float()
        kw = dict(residual=E, ldr=N + 8)
    else:
        x = x * rs[:, None]
    ref = x * rs2[:, None]
    C = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, bias=bias, row_scale=rs, row_scale_post=rs2, **kw)
    torch.cuda.synchronize()
    assert torch.isfinite(C.float()).all()
    assert rel(C, ref) < 1e-2


@pytest.mark.parametrize("M,N,K,op,c32", [(6400, 384, 384, None, 0), (6400, 384, 1536, "residual", 0),
                                          (6400, 1152, 1152, None, 1), (6400, 768, 384, "gate", 0),
                                          (6400, 384, 776, None, 0), (31264, 80, 384, None, 0),
                                          (31264, 384, 80, "residual", 0), (5000, 200, 3000, "gate", 1)])
def test_gemm_persistent_small_tiles(cuda, M, N, K, op, c32):
    """The persistent short-K kernel's 128 x 128 / 128 x 64 tile instances (round 4), which the
    dispatcher picks below 160 tiles of 256 x 128 (the encoder / predictor / concat / mel-linear
    shapes, M = 6400 or N = 80): bias + row scales + gate or residual epilogues, partial row /
    column / K tiles, bf16 and fp32 outputs; fp32 reference on the same bf16 values, rel 1e-2."""
    from fastspeech2 import ops
    torch.manual_seed(M + N + K + 7)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda)
    rs = (torch.rand(M, device=cuda) > 0.2).float()
    rs2 = torch.rand(M, device=cuda) + 0.5
    E = torch.randn(M, N + 8, device=cuda).to(torch.bfloat16)
    x = A.float() @ W.float().t() + bias
    kw = {}
    if op == "gate":
        x = torch.where(E[:, :N].float() > 0, x, torch.zeros_like(x)) * rs[:, None]
        kw = dict(gate=E, ldg=N + 8)
    elif op == "residual":
        x = x * rs[:, None] + E[:, :N].float()
        kw = dict(residual=E, ldr=N + 8)
    else:
        x = x * rs[:, None]
    ref = x * rs2[:, None]
    C = torch.full((M, N), float("nan"), device=cuda,
                   dtype=torch.float32 if c32 else torch.bfloat16)
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, c_fp32=c32, bias=bias, row_scale=rs,
             row_scale_post=rs2, **kw)
    torch.cuda.synchronize()
    assert torch.isfinite(C.float()).all()
    assert rel(C, ref) < 1e-2


def test_gemm_grid_budget(cuda):
    """fs2_gemm_desc.max_ctas: persistent GEMMs given a grid budget (the weight-gradient side
    stream's GEMMs run at 208 blocks) walk more tiles per block and give results bit-identical
    to the full-grid launch, for the long-K (gemm_ps_kernel) and short-K (gemm_pk_kernel,
    128-row and 256-row tiles) instances, on any stream; out-of-range budgets mean the full
    grid (8 is the floor).  The budget is per call: the library keeps no per-stream state."""
    from fastspeech2 import ops
    torch.manual_seed(11)
    shapes = [(31264, 1536, 3456), (31264, 1152, 384), (6400, 384, 1152)]
    s_side = torch.cuda.Stream()
    for M, N, K in shapes:
        A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
        W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device=cuda)
        C0 = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        ops.gemm(M, N, K, A, K, W, K, C0, N, dt=1, bias=bias, relu=1)
        outs = []
        s_side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_side):
            for ctas in (64, 208, 3, 300):
                C1 = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
                ops.gemm(M, N, K, A, K, W, K, C1, N, dt=1, bias=bias, relu=1, max_ctas=ctas)
                outs.append(C1)
        # the same stream, no budget: the full grid again (nothing was registered)
        C2 = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.gemm(M, N, K, A, K, W, K, C2, N, dt=1, bias=bias, relu=1)
        torch.cuda.current_stream().wait_stream(s_side)
        torch.cuda.synchronize()
        for C1 in outs + [C2]:
            assert torch.equal(C0, C1), (M, N, K)


@pytest.mark.parametrize("M,N,K,conv", [(31264, 1152, 384, None), (6400, 384, 1536, None),
                                         (31264, 1536, 3456, (1, 977, 9, 384)),
                                         (31264, 384, 13824, (4, 977, 9, 1536)), (200, 80, 384, None)])
def test_gemm_nan_passes_without_activation(cuda, M, N, K, conv):
    """A NaN input row comes out NaN through every bf16 GEMM kernel family when the epilogue
    has no activation (persistent short-K, 256x128, 256x256 implicit conv, persistent long-K
    padded-domain conv, 128x128): the epilogue's 'no activation' is a select, not a max
    against -inf, so NaN-based divergence checks still see the NaN."""
    from fastspeech2 import ops
    torch.manual_seed(K)
    if conv is not None and conv[0] == 4:
        T = conv[1]
        M = (M // T) * (T + 2 * 4)            # padded-domain rows (T + 2P per utterance)
        A = (torch.randn(31264, conv[3], device=cuda) * 0.5).to(torch.bfloat16)
        A[5, :] = float("nan")
        lda = conv[3]
    else:
        A = (torch.randn(M if conv is None else M, K if conv is None else conv[3], device=cuda)
             * 0.5).to(torch.bfloat16)
        A[5, :] = float("nan")
        lda = A.shape[1]
    W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    C = torch.zeros(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm(M, N, K, A, lda, W, K, C, N, dt=1, conv=conv)
    torch.cuda.synchronize()
    nan_rows = torch.isnan(C.float()).any(1).nonzero().flatten().tolist()
    assert nan_rows, "the NaN input did not reach the output"
    if conv is None:
        assert nan_rows == [5]


def test_gemm_short_k_two_streams(cuda):
    """The persistent short-K kernel (gemm_pk_kernel) under concurrency: 40 back-to-back
    launches alternating between two streams (different tile counts, nk = 1 and nk = 6, bias
    + ReLU-gate epilogue) each cover every tile exactly once -- equal to the first launch of
    the shape and to the fp32 reference on the same bf16 values.  (A per-stream dynamic tile
    queue for this kernel measured 1.1 ms/step slower: each claim's device-scope atomic
    stalls the block once per tile.)"""
    from fastspeech2 import ops
    torch.manual_seed(3)
    shapes = [(31264, 1152, 384), (6400, 384, 1536), (3000, 1536, 64)]
    data = []
    for M, N, K in shapes:
        A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
        W = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device=cuda)
        G = torch.randn(M, N, device=cuda).to(torch.bfloat16)
        ref = torch.where(G.float() > 0, A.float() @ W.float().t() + bias, 0.0)
        data.append((M, N, K, A, W, bias, G, ref))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    outs = []
    for i in range(40):
        M, N, K, A, W, bias, G, ref = data[i % len(data)]
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            # the NaN fill on the GEMM's own stream: a fill on the default stream would race
            # the launch (the two streams waited for the default stream only before the loop)
            C = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
            ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, bias=bias, gate=G, ldg=N)
        outs.append((i, C))
    torch.cuda.synchronize()
    first = {}
    for i, C in outs:
        M, N, K, A, W, bias, G, ref = data[i % len(data)]
        assert torch.isfinite(C.float()).all(), (i, M, N, K)
        if i < len(data):
            assert rel(C, ref) < 1e-2
            first[i] = C
        else:
            assert torch.equal(C, first[i % len(data)]), (i, M, N, K)


@pytest.mark.parametrize("dt,code,tol", DT)
@pytest.mark.parametrize("M,N,ldx", [(31264, 1536, 1536), (6400, 1152, 1152 * 3), (777, 90, 96),
                                      (31264, 1152, 1152), (5000, 264, 264), (1000, 520, 528),
                                      (33, 384, 384)])
def test_colsum_bias_gradient(cuda, dt, code, tol, M, N, ldx):
    """fs2_colsum (bias gradients): out (+)= column sums over rows of a row-pitched matrix
    (N / VEC >= 32: the column-slab kernel, partial last slab at N = 264 / 520; else the
    sub-row kernel)."""
    from fastspeech2 import ops
    torch.manual_seed(M)
    X = torch.randn(M, ldx, device=cuda).to(dt)
    out = torch.full((N,), 2.0, device=cuda)
    ws = torch.empty(int(ops.colsum_ws(M, N)), device=cuda)
    ops.colsum(X, ldx, M, N, out, dt=code, ws=ws, accumulate=1)
    ref = X[:, :N].double().sum(0)
    assert ((out.double() - 2.0 - ref).abs().max() / ref.abs().max()).item() < 1e-5


def _keep_np(seed, salt, idx, p):
    """numpy restatement of fs2_keep_fast (fs2_common.h): the LayerNorm dropout masks."""
    M32 = np.uint64(0xffffffff)

    def mix(h):
        h = h & M32
        h ^= h >> np.uint64(16)
        h = (h * np.uint64(0x85ebca6b)) & M32
        h ^= h >> np.uint64(13)
        h = (h * np.uint64(0xc2b2ae35)) & M32
        h ^= h >> np.uint64(16)
        return h

    key = int(mix(np.uint64((seed ^ ((salt * 0x9E3779B9) & 0xffffffff)) & 0xffffffff))) | 1
    idx = idx.astype(np.uint64)
    pair = idx >> np.uint64(1)
    h = ((pair & M32) * np.uint64(0x9E3779B1)) & M32
    h ^= ((pair >> np.uint64(32)) * np.uint64(0x85EBCA77)) & M32
    h ^= np.uint64(key)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x2C1B3C6D)) & M32
    h ^= h >> np.uint64(12)
    h = (h * np.uint64(0x297A2D39)) & M32
    h ^= h >> np.uint64(15)
    bits = (h >> ((idx & np.uint64(1)) * np.uint64(16))) & np.uint64(0xffff)
    return bits >= np.uint64(int(p * 65536 + 0.5))


def _attn_keep_np(seed, salt, rows, keys, p):
    """numpy restatement of fs2_attn_keep (fs2_common.h), the attention-probability dropout:
    a lowbias32 hash per query row (rows = (b*H + h)*T + q), one add of (key >> 1) * KC and one
    xorshift / 24-bit multiply / xorshift round per key pair.  rows (R, 1), keys (1, K)."""
    M32 = np.uint64(0xffffffff)

    def mix(h):
        h = h & M32
        h ^= h >> np.uint64(16)
        h = (h * np.uint64(0x85ebca6b)) & M32
        h ^= h >> np.uint64(13)
        h = (h * np.uint64(0xc2b2ae35)) & M32
        h ^= h >> np.uint64(16)
        return h

    dkey = int(mix(np.uint64((seed ^ ((salt * 0x9E3779B9) & 0xffffffff)) & 0xffffffff))) | 1
    r = rows.astype(np.uint64)
    k = keys.astype(np.uint64)
    h = ((r * np.uint64(0x9E3779B1)) & M32) ^ np.uint64(dkey)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & M32
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & M32
    h ^= h >> np.uint64(16)
    u = (h + (k >> np.uint64(1)) * np.uint64(0x27D4EB2F)) & M32
    u ^= u >> np.uint64(15)
    u = ((u & np.uint64(0xffffff)) * np.uint64(0x5BD1E9)) & M32
    u ^= u >> np.uint64(13)
    bits = (u >> ((k & np.uint64(1)) * np.uint64(16))) & np.uint64(0xffff)
    return bits >= np.uint64(int(p * 65536 + 0.5))


@pytest.mark.parametrize("dh,T,p_drop,B", [(192, 150, 0.0, 3), (192, 150, 0.1, 3), (64, 70, 0.1, 3),
                                            (256, 130, 0.0, 3), (192, 977, 0.0, 32),
                                            (192, 977, 0.1, 32), (256, 977, 0.1, 32),
                                            (192, 200, 0.0, 32), (128, 300, 0.1, 4)])
def test_fused_attention_vs_torch(cuda, dh, T, p_drop, B):
    """fs2_attn_fwd/bwd (bf16) against torch fp32 on the same bf16 Q/K/V: the head-major mask
    tiling rule, ragged lengths, and (p > 0) the counter-hash dropout masks restated in numpy.
    B=32 with T=977 / 200 are the bench's decoder / encoder shapes: 128-row (W8 = 8) blocks for
    the decoder, 64-row blocks for the encoder, descending ragged lengths as the collate sorts,
    with and without dropout; dh=256 (BASELINE config 4) at T=977.
    Tolerance rel 2e-2 (O) / 3e-2 (dQ, dK, dV): bf16 operands and probabilities."""
    from fastspeech2 import ops
    torch.manual_seed(dh + T)
    H = 2
    D = H * dh
    if B <= 4:
        lens = [T, T - 37, T - 90, T - 11][:B]
    else:
        g = torch.Generator().manual_seed(T)
        lens = sorted([T] + torch.randint(T // 2, T + 1, (B - 1,), generator=g).tolist(),
                      reverse=True)
    qkv = (torch.randn(B * T, 3 * D, device=cuda) * 0.5).to(torch.bfloat16)
    kp = torch.zeros(B, T, dtype=torch.uint8, device=cuda)
    for b, L in enumerate(lens):
        kp[b, L:] = 1
    scale = 1.0 / math.sqrt(dh)
    seed, salt = 77, 5
    out = torch.empty(B * T, D, device=cuda, dtype=torch.bfloat16)
    lse = torch.empty(B * H, T, device=cuda)
    ops.attn_fwd(qkv, 3 * D, kp, B, H, T, dh, scale, p_drop, seed, salt, out, D, lse, dt=1)
    # torch reference
    x = qkv.float().view(B, T, 3, H, dh)
    q = x[:, :, 0].permute(0, 2, 1, 3).clone().requires_grad_(True)
    k = x[:, :, 1].permute(0, 2, 1, 3).clone().requires_grad_(True)
    v = x[:, :, 2].permute(0, 2, 1, 3).clone().requires_grad_(True)
    pad = kp.bool()
    b2 = [(b * H + h) % B for b in range(B) for h in range(H)]
    mask = (pad.repeat_interleave(H, 0) | pad[b2]).view(B, H, 1, T)
    s = (q @ k.transpose(-1, -2)) * scale
    P = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
    if p_drop > 0:
        keep = _attn_keep_np(seed, salt, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p_drop)
        keep = torch.from_numpy(keep.reshape(B, H, T, T)).to(cuda)
        P = P * keep / (1 - p_drop)
    o = P @ v
    ref = o.permute(0, 2, 1, 3).reshape(B * T, D)
    assert rel(out, ref) < 2e-2
    dout = torch.randn(B * T, D, device=cuda).to(torch.bfloat16)
    ref.backward(dout.float())
    dqkv = torch.full((B * T, 3 * D), float("nan"), device=cuda, dtype=torch.bfloat16)
    ws = torch.empty(int(ops.attn_ws(B, H, T)), device=cuda)
    ops.attn_bwd(qkv, 3 * D, kp, out, D, dout, D, lse, B, H, T, dh, scale, p_drop, seed, salt,
                 dqkv, 3 * D, dt=1, ws=ws)
    for i, t in enumerate((q, k, v)):
        r = t.grad.permute(0, 2, 1, 3).reshape(B * T, D)
        assert rel(dqkv[:, i * D:(i + 1) * D], r) < 3e-2, i


def test_weight_prep_batched_layouts(cuda):
    """fs2_weight_prep_batched: fp32 masters ([O][KW][C] conv weights, [O][C] linear weights,
    shapes not multiples of the 64x64 tile) -> bf16 Wf[O][ldf] (zero column padding) and
    Wb[C][KW*O], exactly the bf16 rounding of the expected images."""
    from fastspeech2 import ops
    torch.manual_seed(12)
    shapes = [(384, 384, 9), (80, 384, 1), (130, 72, 5), (1152, 384, 1)]
    entries, refs = [], []
    for O, C, KW in shapes:
        W = torch.randn(O, KW, C, device=cuda) if KW > 1 else torch.randn(O, C, device=cuda)
        ldf = ops.round_up(KW * C, 8)
        Wf = torch.full((O, ldf), float("nan"), device=cuda).to(torch.bfloat16)
        Wb = torch.full((C, KW * O), float("nan"), device=cuda).to(torch.bfloat16)
        entries.append((W, O, C, KW, int(KW > 1), Wf, ldf, Wb, KW * O))
        W3 = W.view(O, KW, C)
        ref_f = torch.zeros(O, ldf, device=cuda)
        ref_f[:, :KW * C] = W3.reshape(O, KW * C)
        ref_b = W3.permute(2, 1, 0).reshape(C, KW * O)      # [c][j*O + o]
        refs.append((Wf, Wb, ref_f.to(torch.bfloat16), ref_b.to(torch.bfloat16)))
    table = ops.weight_prep_table(entries)
    ops.weight_prep_batched(*table, dt=1)
    torch.cuda.synchronize()
    for Wf, Wb, rf, rb in refs:
        assert torch.equal(Wf, rf)
        assert torch.equal(Wb, rb)


def test_weight_prep_reversed_taps(cuda):
    """w_okc bit 1: the data-gradient image Wb with its taps reversed, Wb[c][(KW-1-j)*O + o],
    in fs2_weight_prep_batched, fs2_weight_prep and the fused AdamW image pass (zero step:
    decay 1, step size 0), exactly the bf16 rounding of the expected image."""
    from fastspeech2 import ops
    torch.manual_seed(13)
    O, C, KW = 136, 72, 9
    W = torch.randn(O, KW, C, device=cuda)
    ldf = ops.round_up(KW * C, 8)
    ref_b = W.flip(1).permute(2, 1, 0).reshape(C, KW * O).to(torch.bfloat16)
    ref_f = torch.zeros(O, ldf, device=cuda)
    ref_f[:, :KW * C] = W.reshape(O, KW * C)
    ref_f = ref_f.to(torch.bfloat16)
    Wf = torch.full((O, ldf), float("nan"), device=cuda).to(torch.bfloat16)
    Wb = torch.full((C, KW * O), float("nan"), device=cuda).to(torch.bfloat16)
    table = ops.weight_prep_table([(W, O, C, KW, 3, Wf, ldf, Wb, KW * O)])
    ops.weight_prep_batched(*table, dt=1)
    torch.cuda.synchronize()
    assert torch.equal(Wf, ref_f) and torch.equal(Wb, ref_b)
    Wb.fill_(float("nan"))
    ops.weight_prep(W, O, C, KW, Wf, ldf, Wb, KW * O, dt=1, w_okc=3)
    torch.cuda.synchronize()
    assert torch.equal(Wb, ref_b)


@pytest.mark.parametrize("O,C,KW", [(1536, 384, 9), (192, 72, 5), (128, 40, 3), (256, 128, 9)])
def test_weight_prep_tap_inner(cuda, O, C, KW):
    """w_okc bit 2: Wb's columns in tap-inner 64-channel chunks, (o/64)*KW*64 + j*64 + o%64
    (with bit 1: taps reversed); bit 3 (C % 64 == 0): Wf's columns the same way over c -- in
    fs2_weight_prep_batched and fs2_weight_prep, exactly the bf16 rounding of the permuted
    images."""
    from fastspeech2 import ops
    torch.manual_seed(O + KW)
    W = torch.randn(O, KW, C, device=cuda)
    ldf = ops.round_up(KW * C, 8)
    okc = 7 | (8 if C % 64 == 0 else 0)
    nat = W.flip(1).permute(2, 1, 0)                      # [C][j][O], taps reversed
    ref_b = nat.reshape(C, KW, O // 64, 64).permute(0, 2, 1, 3).reshape(C, KW * O)
    ref_b = ref_b.to(torch.bfloat16)
    if okc & 8:
        ref_f = W.view(O, KW, C // 64, 64).permute(0, 2, 1, 3).reshape(O, KW * C)
    else:
        ref_f = torch.zeros(O, ldf, device=cuda)
        ref_f[:, :KW * C] = W.reshape(O, KW * C)
    ref_f = ref_f.to(torch.bfloat16)
    Wf = torch.full((O, ldf), float("nan"), device=cuda).to(torch.bfloat16)
    Wb = torch.full((C, KW * O), float("nan"), device=cuda).to(torch.bfloat16)
    table = ops.weight_prep_table([(W, O, C, KW, okc, Wf, ldf, Wb, KW * O)])
    ops.weight_prep_batched(*table, dt=1)
    torch.cuda.synchronize()
    assert torch.equal(Wb, ref_b) and torch.equal(Wf, ref_f)
    Wb.fill_(float("nan"))
    Wf.fill_(float("nan"))
    ops.weight_prep(W, O, C, KW, Wf, ldf, Wb, KW * O, dt=1, w_okc=okc)
    torch.cuda.synchronize()
    assert torch.equal(Wb, ref_b) and torch.equal(Wf, ref_f)


@pytest.mark.parametrize("B,T,O,C,KW", [(32, 977, 1536, 384, 9), (3, 37, 256, 128, 9),
                                         (2, 50, 192, 256, 5), (4, 120, 128, 384, 3)])
def test_conv_dgrad_padded_image(cuda, B, T, O, C, KW):
    """The FFN conv1 data gradient over a zero-padded token-major dY image: (1) a gated GEMM
    writes its rows into the image's data rows (fs2_gemm c_row = (T, 2P)), leaving the zero
    pad rows untouched; (2) the plain K-major GEMM over the image with overlapping A rows
    (lda = O) against the tap-reversed Wb equals the shift-conv GEMM (conv_mode 4) over
    token-major dY with the natural Wb -- the same products in another K order (fp32 rel
    1e-5); (3) so does the tap-inner K order (a_kw, 64-channel chunks outer, taps inner, Wb
    built with w_okc bit 2) on the 4-wave kernel, where K % 128 == 0.  Decoder shape, a ragged
    small one (one partial row tile), a k = 5 one (K % 128 != 0: natural order only), a k = 3
    one (two chunks of three taps)."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + KW)
    P = (KW - 1) // 2
    M = B * T
    L = T + 2 * P
    Mp = B * L
    bf = torch.bfloat16
    # (1) gated GEMM (the conv2 data gradient: M x O from K = C2) into the padded image
    C2 = 384
    A = (torch.randn(M, C2, device=cuda) * 0.5).to(bf)
    W2 = (torch.randn(O, C2, device=cuda) * 0.05).to(bf)
    G = torch.randn(M, O, device=cuda).to(bf)
    buf = torch.full(((B + 1) * L, O), float("nan"), device=cuda, dtype=bf)
    buf.view(B + 1, L, O)[:, T:] = 0
    img = buf[T:]
    ops.gemm(M, O, C2, A, C2, W2, C2, img[2 * P:], O, dt=1, gate=G, ldg=O, c_row=(T, 2 * P))
    dY = torch.empty(M, O, device=cuda, dtype=bf)
    ops.gemm(M, O, C2, A, C2, W2, C2, dY, O, dt=1, gate=G, ldg=O)
    torch.cuda.synchronize()
    data = img[2 * P:2 * P + Mp].view(B, L, O)
    # (the padded write always runs on the persistent kernel; small unpadded shapes may not)
    assert rel(data[:, :T].reshape(M, O), dY) < (1e-6 if M >= 31264 else 1e-2)
    assert not data[:, T:].float().abs().gt(0).any()          # pad rows still zero
    assert not img[:2 * P].float().abs().gt(0).any()
    # (2) data gradient: plain GEMM over the image vs conv_mode 4
    Wm = torch.randn(O, KW, C, device=cuda) * 0.05
    ldf = ops.round_up(KW * C, 8)
    Wf = torch.empty(O, ldf, device=cuda, dtype=bf)
    Wb = torch.empty(C, KW * O, device=cuda, dtype=bf)
    Wr = torch.empty(C, KW * O, device=cuda, dtype=bf)
    ops.weight_prep(Wm, O, C, KW, Wf, ldf, Wb, KW * O, dt=1, w_okc=1)
    ops.weight_prep(Wm, O, C, KW, Wf, ldf, Wr, KW * O, dt=1, w_okc=3)
    X4 = torch.empty(Mp, C, device=cuda)
    X0 = torch.empty(Mp, C, device=cuda)
    ops.gemm(Mp, C, KW * O, dY, O, Wb, KW * O, X4, C, dt=1, conv=(4, T, KW, O), c_fp32=1)
    ops.gemm(Mp, C, KW * O, img, O, Wr, KW * O, X0, C, dt=1, c_fp32=1)
    torch.cuda.synchronize()
    assert torch.isfinite(X0).all()
    assert rel(X0, X4) < 1e-5
    # (3) the tap-inner K order (fs2_gemm_desc.a_kw, Wb with w_okc bit 2; the 4-wave kernel)
    if O % 64 == 0 and (KW * O) % 128 == 0:
        Wt = torch.empty(C, KW * O, device=cuda, dtype=bf)
        ops.weight_prep(Wm, O, C, KW, Wf, ldf, Wt, KW * O, dt=1, w_okc=7)
        Xt = torch.full((Mp, C), float("nan"), device=cuda)
        ops.gemm(Mp, C, KW * O, img, O, Wt, KW * O, Xt, C, dt=1, c_fp32=1, a_kw=KW)
        torch.cuda.synchronize()
        assert torch.isfinite(Xt).all()
        assert rel(Xt, X4) < 1e-5


@pytest.mark.parametrize("B,T,D,P", [(32, 977, 384, 4), (32, 200, 384, 4), (3, 7, 384, 4),
                                     (2, 50, 1024, 2), (4, 9, 80, 4)])
def test_ln_fwd_padded_image(cuda, B, T, D, P):
    """fs2_ln_fwd's img output: the LayerNorm output y, bit-identical to a call without it, and
    its reflect-padded token-major image, exactly what fs2_pad_rows makes from y (pad rows
    mirrored; T = 7 and 9 with P = 4: every row of a short utterance lands in a pad row too).
    D = 1024 takes the one-row vector kernel and the image from a second pass."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + D)
    bf = torch.bfloat16
    M, L = B * T, T + 2 * P
    x = torch.randn(M, D, device=cuda).to(bf)
    r = torch.randn(M, D, device=cuda).to(bf)
    g = torch.randn(D, device=cuda)
    b = torch.randn(D, device=cuda)
    outs = []
    for with_img in (False, True):
        y = torch.empty(M, D, device=cuda, dtype=bf)
        s = torch.empty(M, D, device=cuda, dtype=bf)
        mean = torch.empty(M, device=cuda)
        rstd = torch.empty(M, device=cuda)
        img = torch.full((B * L, D), float("nan"), device=cuda, dtype=bf) if with_img else None
        ops.ln_fwd(x, D, g, b, 1e-6, y, D, mean, rstd, M, D, dt=1, seed=3, r=r, ldr=D, p_r=0.1,
                   salt_r=5, s_out=s, img=img, img_t=T, img_p=P)
        outs.append((y, s, img))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = torch.full((B * L, D), float("nan"), device=cuda, dtype=bf)
    ops.pad_rows(outs[1][0], D, B, T, D, P, 1, 0, ref, D, dt=1)
    torch.cuda.synchronize()
    assert torch.equal(outs[1][2], ref)


@pytest.mark.parametrize("B,T,C,O,KW", [(32, 977, 384, 1536, 9), (32, 200, 384, 1536, 9),
                                         (3, 37, 128, 256, 9), (2, 50, 192, 320, 5)])
def test_conv_fwd_padded_image(cuda, B, T, C, O, KW):
    """The FFN conv1 forward over the padded token domain: fs2_pad_rows writes the
    reflect-padded token-major image (checked exactly against torch's reflect pad), then a
    plain K-major GEMM with overlapping rows (lda = C) drops each utterance's 2P pad rows in
    its epilogue (c_row = (T, -2P)) -- equal to the implicit reflect conv (conv_mode 1) with
    bias + ReLU (bf16 outputs, rel 1e-2: two kernels, one sum order), and so does the
    tap-inner K order where C % 64 == 0.  Every token row is written (NaN-filled output)."""
    from fastspeech2 import ops
    torch.manual_seed(B + T + KW)
    P = (KW - 1) // 2
    M, L = B * T, T + 2 * P
    bf = torch.bfloat16
    X = (torch.randn(M, C, device=cuda) * 0.5).to(bf)
    img = torch.full((B * L + 2 * P, C), float("nan"), device=cuda, dtype=bf)
    ops.pad_rows(X, C, B, T, C, P, 1, 2 * P, img, C, dt=1)
    ref_img = F.pad(X.float().view(B, T, C).transpose(1, 2), (P, P), mode="reflect")
    torch.cuda.synchronize()
    assert torch.equal(img[:B * L].float().view(B, L, C), ref_img.transpose(1, 2))
    assert not img[B * L:].float().abs().gt(0).any()
    W = (torch.randn(O, KW * C, device=cuda) * 0.05).to(bf)
    bias = torch.randn(O, device=cuda)
    Y1 = torch.full((M, O), float("nan"), device=cuda, dtype=bf)
    Y0 = torch.full((M, O), float("nan"), device=cuda, dtype=bf)
    ops.gemm(M, O, KW * C, X, C, W, KW * C, Y1, O, dt=1, conv=(1, T, KW, C), bias=bias, relu=1)
    ops.gemm(B * L, O, KW * C, img, C, W, KW * C, Y0, O, dt=1, bias=bias, relu=1,
             c_row=(T, -2 * P))
    torch.cuda.synchronize()
    assert torch.isfinite(Y0.float()).all()
    assert rel(Y0, Y1) < 1e-2
    # the tap-inner K order (fs2_gemm_desc.a_kw; W's columns in 64-channel chunks, as
    # fs2_weight_prep w_okc bit 3 builds them) on the 4-wave kernel
    if C % 64 == 0 and (KW * C) % 128 == 0:
        Wt = W.view(O, KW, C // 64, 64).permute(0, 2, 1, 3).reshape(O, KW * C).contiguous()
        Y2 = torch.full((M, O), float("nan"), device=cuda, dtype=bf)
        ops.gemm(B * L, O, KW * C, img, C, Wt, KW * C, Y2, O, dt=1, bias=bias, relu=1,
                 c_row=(T, -2 * P), a_kw=KW)
        torch.cuda.synchronize()
        assert torch.isfinite(Y2.float()).all()
        assert rel(Y2, Y1) < 1e-2


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("B,T,V", [(32, 200, 95), (3, 37, 128), (1, 5, 7), (4, 50, 200),
                                   (2, 40, 300)])
def test_embedding_fwd_bwd(cuda, dt, code, B, T, V):
    """fs2_embed_fwd (table row + positional encoding, pad rows zero) and fs2_embed_bwd (token
    rows scatter-added into the table gradient through per-wave LDS accumulators, fixed-order
    combine) against torch: forward exact up to the output rounding, backward rel 1e-5 (fp32
    sums of the same values in another order).  Bench shape (B*T_p = 6400, V = 95 = n_char),
    a ragged one with V at one grid.z id window (128), a tiny one, and V = 200 / 300 (two and
    three id windows); pad tokens (id 0) are masked."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + V)
    D = 384
    M = B * T
    tok = torch.randint(0, V, (B, T), device=cuda)
    tok[:, T - T // 4:] = 0
    table = torch.randn(V, D, device=cuda)
    pe = torch.randn(T, D, device=cuda)
    X = torch.empty(M, D, device=cuda, dtype=dt)
    keep = torch.empty(M, device=cuda)
    ops.embed_fwd(tok, table, pe, 0, B, T, D, X, keep, dt=code)
    k_ref = (tok.reshape(-1) != 0).float()
    ref = (table[tok.reshape(-1)] + pe.repeat(B, 1)) * k_ref[:, None]
    assert torch.equal(keep, k_ref)
    assert rel(X, ref.to(dt)) < (1e-6 if dt == torch.float32 else 1e-2)
    dX = torch.randn(M, D, device=cuda).to(dt)
    dtab = torch.full((V, D), 0.5, device=cuda)
    ws = torch.empty(ops.embed_bwd_ws(D, V), device=cuda)
    ops.embed_bwd(tok.reshape(-1), dX, keep, M, D, V, dtab, dt=code, ws=ws)
    g = torch.zeros(V, D, device=cuda).index_add_(0, tok.reshape(-1), dX.float() * keep[:, None])
    assert rel(dtab - 0.5, g) < 1e-5


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("M,D,ldu", [(6400, 384, 384), (999, 256, 264), (777, 200, 203),
                                     (130, 1104, 1112)])
def test_rowdot_bwd(cuda, dt, code, M, D, ldu):
    """fs2_rowdot_bwd (the variance predictors' 384 -> 1 head): du = dy * scale * w per row,
    dw / db = fixed-order column partials; against torch fp32 on the same values.  The bench
    shape, a ragged one, an odd pitch (ldu = 203: the one-column-per-lane fallback) and a row
    wider than one 64 x 16 B column slab (grid.y = 3 / 5 slabs)."""
    from fastspeech2 import ops
    torch.manual_seed(M + D)
    u = torch.randn(M, ldu, device=cuda).to(dt)
    dy = torch.randn(M, device=cuda).to(dt)
    w = torch.randn(D, device=cuda)
    scale = 0.7
    du = torch.empty(M, D, device=cuda, dtype=dt)
    dw, db = torch.zeros(D, device=cuda), torch.zeros(1, device=cuda)
    ws = torch.empty(256 * (D + 1), device=cuda)
    ops.rowdot_bwd(dy, u, ldu, w, scale, M, D, du, dw, db, dt=code, ws=ws)
    g = dy.float() * scale
    assert rel(du, (g[:, None] * w[None, :]).to(dt)) < (1e-6 if dt == torch.float32 else 1e-2)
    assert rel(dw, (g[:, None] * u[:, :D].float()).sum(0)) < 1e-5
    assert abs(db.item() - g.sum().item()) <= 1e-4 * max(1.0, abs(g.sum().item()))


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("B,T,D,KW", [(32, 200, 384, 3), (3, 37, 256, 5), (2, 9, 1104, 8),
                                      (5, 17, 201, 1), (1, 4, 64, 7)])
def test_embed1d_bwd(cuda, dt, code, B, T, D, KW):
    """fs2_embed1d_bwd (pitch / energy embedding conv, SB Conv1d(1 -> D, k, reflect) weight and
    bias gradients, model.py:226-240): dW[o][j] += sum dOut[b,t,o] a[b, refl(t+j-P)], dbias
    += sum dOut, against torch autograd of the same conv in fp32 on the same (rounded) dOut.
    Bench shape (M = 6400, D = 384, k = 3), ragged rows, a row of three 16 B slabs, D = 201
    (odd: the one-column-per-lane fallback), k = 1 and k = 7 / 8 with T just above the reflect
    pad."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + D + KW)
    M = B * T
    a = torch.randn(B, T, device=cuda)
    dout = torch.randn(M, D, device=cuda).to(dt)
    dW = torch.full((D, KW), 0.25, device=cuda)
    db = torch.full((D,), -0.5, device=cuda)
    ws = torch.empty(128 * (KW + 1) * D, device=cuda)
    ops.embed1d_bwd(dout, a, B, T, D, KW, dW, db, dt=code, ws=ws)
    P = (KW - 1) // 2
    W = torch.zeros(D, 1, KW, device=cuda, requires_grad=True)
    bias = torch.zeros(D, device=cuda, requires_grad=True)
    x = F.pad(a[:, None, :], (P, KW - 1 - P), mode="reflect") if KW > 1 else a[:, None, :]
    y = F.conv1d(x, W, bias)                                   # [B][D][T]
    y.backward(dout.float().reshape(B, T, D).transpose(1, 2))
    assert rel(dW - 0.25, W.grad[:, 0, :]) < 1e-5
    assert rel(db + 0.5, bias.grad) < 1e-5


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("B,T,D,n_spk", [(32, 200, 384, 4), (3, 37, 256, 2), (4, 11, 1104, 3),
                                         (2, 5, 201, 5)])
def test_concat_bwd_spk(cuda, dt, code, B, T, D, n_spk):
    """fs2_concat_bwd_spk (speaker-embedding gradient of the conditioning concat, model.py:
    352-358): dSpk[spk[b]] += sum_t dcat[b,t,D:2D] in utterance order, against torch index_add
    in fp32.  Bench shape, ragged, three 16 B slabs per row, and D = 201 (odd pitch: the
    one-column-per-lane fallback); speaker 0 of n_spk = 5 gets no utterance in the last case
    (its row must stay as it was)."""
    from fastspeech2 import ops
    torch.manual_seed(B * T + D)
    dcat = torch.randn(B * T, 2 * D, device=cuda).to(dt)
    spk = torch.randint(1 if n_spk > 4 else 0, n_spk, (B,), device=cuda)
    dspk = torch.full((n_spk, D), 0.5, device=cuda)
    ws = torch.empty(B * D, device=cuda)
    ops.concat_bwd_spk(dcat, 2 * D, spk, B, T, D, n_spk, dspk, dt=code, ws=ws)
    U = dcat.float().reshape(B, T, 2 * D)[:, :, D:].sum(1)
    ref = torch.zeros(n_spk, D, device=cuda).index_add_(0, spk, U)
    assert rel(dspk - 0.5, ref) < 1e-5
    if n_spk > 4:
        assert torch.equal(dspk[0], torch.full((D,), 0.5, device=cuda))


def test_attention_dropout_mask_statistics(cuda, parity_log):
    """Quality of the attention-probability dropout draw (fs2_attn_rowhash + one fs2_attn_mix
    round per key pair, fs2_common.h), on the bench decoder grid (B*H*T rows x T keys = 61 M
    draws, p = 0.1) taken from the materialised softmax path, which uses the same bits as the
    fused kernels: keep rate within 6 binomial sigmas of 0.9; lag-1 (inside and across key
    pairs) and lag-2 correlations along keys, and lag-1 / lag-2 along rows, below 0.002 (an
    ideal generator's sigma here is ~1.3e-4); two dropout salts draw unrelated masks."""
    from fastspeech2 import ops
    B, H, T, p = 32, 2, 977, 0.1
    ldt = (T + 7) // 8 * 8
    S = torch.zeros(B * H, T, ldt, device=cuda)
    kp = torch.zeros(B * T, dtype=torch.uint8, device=cuda)
    Pm = torch.empty_like(S)
    stats = {}

    def keep_bits(salt):
        Pd = torch.empty_like(S)
        ops.softmax_fwd(S, kp, B, H, T, T, ldt, 1.0, p, 1234, salt, Pm, Pd, dt=0)
        torch.cuda.synchronize()
        return (Pd[:, :, :T] > 0).reshape(B * H * T, T).float()

    def corr(a, b):
        a = a - a.mean()
        b = b - b.mean()
        return ((a * b).mean() / (a.std() * b.std())).item()

    k = keep_bits(9)
    n = k.numel()
    rate = k.mean().item()
    sigma = (p * (1 - p) / n) ** 0.5
    assert abs(rate - (1 - p)) <= 6 * sigma, rate
    stats["keep_rate"] = rate
    stats["lag1_key_in_pair"] = corr(k[:, 0:T - 1:2], k[:, 1:T:2])
    stats["lag1_key_across_pair"] = corr(k[:, 1:T - 1:2], k[:, 2:T:2])
    stats["lag2_key"] = corr(k[:, :-2], k[:, 2:])
    stats["lag1_row"] = corr(k[:-1], k[1:])
    stats["lag2_row"] = corr(k[:-2], k[2:])
    stats["other_salt"] = corr(k, keep_bits(10))
    for name, c in stats.items():
        if name != "keep_rate":
            assert abs(c) < 2e-3, (name, c)
    parity_log["attn_dropout_mask_stats"] = stats
