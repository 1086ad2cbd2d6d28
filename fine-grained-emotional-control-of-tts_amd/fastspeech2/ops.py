"""Python operator layer over the C ABI (include/fs2_hip.h).

Every function here is a thin, allocation-free wrapper: it turns tensors into device
pointers, passes torch's *current* HIP stream, and raises if the native call reports an
error.  Tensors are owned by torch's caching allocator; the kernels never allocate.
"""

import collections
import ctypes
import os
import sys

import torch

from . import _native as N

EPC = {N.F32: 4, N.BF16: 8}   # elements per 16-byte chunk (GEMM K / pitch granularity)


def _p(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _s():
    return N.stream_ptr()


def _chk(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} returned {rc}")


def round_up(x, m):
    return (x + m - 1) // m * m


# FS2_GEMM_TRACE=1: count fs2_gemm calls by (shape, operand flags, calling engine line); the
# table is printed to stderr at exit (tools/gemm_sites.sh) -- which call sites take which kernel
_TRACE = collections.Counter() if os.environ.get("FS2_GEMM_TRACE") else None


def _trace(d, conv):
    f = sys._getframe(2)
    while f is not None and os.path.basename(f.f_code.co_filename) == "ops.py":
        f = f.f_back
    site = f"{f.f_code.co_name}:{f.f_lineno}" if f is not None else "?"
    flags = "".join(k for k, v in (("a", not d.a_kmajor), ("b", not d.b_kmajor), ("f", d.c_fp32),
                                   ("B", d.bias), ("r", d.relu), ("g", d.gate), ("R", d.residual),
                                   ("s", d.row_scale), ("S", d.row_scale_post),
                                   ("+", d.accumulate), ("c", d.c_row_t)) if v)
    _TRACE[(d.M, d.N, d.K, conv[0] if conv else 0, d.split_k, d.batch, flags, site)] += 1


def _trace_dump():
    for k, n in sorted(_TRACE.items(), key=lambda x: -x[0][0] * x[0][1] * x[0][2] * x[1]):
        M, N_, K, cm, sk, b, fl, site = k
        print(f"gemm {n:4d}x M {M:6d} N {N_:5d} K {K:6d} conv {cm} split {sk} batch {b:4d} "
              f"[{fl}] {site}", file=sys.stderr)


if _TRACE is not None:
    import atexit
    atexit.register(_trace_dump)


def gemm(M, N_, K, A, lda, B, ldb, C, ldc, *, dt, a_kmajor=1, b_kmajor=1, conv=None, c_fp32=0,
         c_conv_kw=0, bias=None, relu=0, gate=None, ldg=0, row_scale=None, residual=None, ldr=0,
         row_scale_post=None, accumulate=0, split_k=1, split_stride=0, kvalid=0, mvalid=0,
         nvalid=0, batch=1, batch_div=1, strides=None, conv_dil=1, c_row=None, max_ctas=0,
         a_kw=0):
    d = N.GemmDesc()
    d.conv_dil = conv_dil
    d.a_kw = a_kw             # tap-inner K order of an overlapping-row A (fs2_gemm_desc.a_kw)
    d.max_ctas = max_ctas     # persistent-kernel grid budget (0: one block per CU)
    if c_row is not None:     # (T, pad): output row m stored at m + (m // T) * pad
        d.c_row_t, d.c_row_pad = c_row
    d.M, d.N, d.K, d.kvalid, d.mvalid, d.nvalid, d.dtype = M, N_, K, kvalid, mvalid, nvalid, dt
    d.A, d.lda, d.a_kmajor = _p(A), lda, a_kmajor
    d.B, d.ldb, d.b_kmajor = _p(B), ldb, b_kmajor
    if conv is not None:
        d.conv_mode, d.conv_t, d.conv_kw, d.conv_c = conv
    d.C, d.ldc, d.c_fp32, d.c_conv_kw = _p(C), ldc, c_fp32, c_conv_kw
    d.bias, d.relu = _p(bias), relu
    d.gate, d.ldg = _p(gate), ldg
    d.row_scale = _p(row_scale)
    d.residual, d.ldr = _p(residual), ldr
    d.row_scale_post = _p(row_scale_post)
    d.accumulate, d.split_k, d.split_stride = accumulate, split_k, split_stride
    d.batch, d.batch_div = batch, batch_div
    if strides is not None:
        (d.sA1, d.sA2, d.sB1, d.sB2, d.sC1, d.sC2, d.sR1, d.sR2) = strides
    if _TRACE is not None:
        _trace(d, conv)
    _chk(N.lib().fs2_gemm(ctypes.byref(d), _s()), "fs2_gemm")


def conv_fold(Xpad, B, T, P, C, out, ldo, *, dt, residual=None, ldr=0, row_scale=None,
              row_scale_post=None, nsplit=1, split_stride=0):
    _chk(N.lib().fs2_conv_fold(_p(Xpad), nsplit, split_stride, B, T, P, C, _p(out), ldo,
                               _p(residual), ldr,
                               _p(row_scale), _p(row_scale_post), dt, _s()), "fs2_conv_fold")


def pad_transpose(X, ldx, B, T, C, P, reflect, out, ldo, ncols, *, dt, colsum=None, ws=None):
    _chk(N.lib().fs2_pad_transpose(_p(X), ldx, B, T, C, P, reflect, _p(out), ldo, ncols,
                                   _p(colsum), _p(ws), dt, _s()), "fs2_pad_transpose")


def pad_rows(X, ldx, B, T, C, P, reflect, tail, out, ldo, *, dt):
    _chk(N.lib().fs2_pad_rows(_p(X), ldx, B, T, C, P, reflect, tail, _p(out), ldo, dt, _s()),
         "fs2_pad_rows")


def pad_transpose_ws(ncols, C):
    return -(-ncols // 64) * C


def sum_slices(ws, nslices, stride, n, out, accumulate=1):
    _chk(N.lib().fs2_sum_slices(_p(ws), nslices, stride, n, _p(out), accumulate, _s()),
         "fs2_sum_slices")


def colsum(X, ldx, M, N_, out, *, dt, ws, accumulate=1):
    _chk(N.lib().fs2_colsum(_p(X), ldx, M, N_, dt, _p(out), accumulate, _p(ws), _s()), "fs2_colsum")


def colsum_ws(M, N_):
    return N.lib().fs2_colsum_workspace_floats(M, N_)


def ln_fwd(x, ldx, gamma, beta, eps, y, ldy, mean, rstd, M, D, *, dt, seed=0, r=None, ldr=0,
           p_r=0.0, salt_r=0, s_out=None, do_tanh=0, p_o=0.0, salt_o=0, row_mask=None,
           post_add=None, ldp=0, img=None, img_t=0, img_p=0):
    """``img``: also y's reflect-padded token-major image (fs2_pad_rows layout, img_t tokens
    per utterance, img_p pad rows each side)"""
    _chk(N.lib().fs2_ln_fwd(_p(x), ldx, _p(r), ldr, p_r, salt_r, _p(s_out), _p(gamma), _p(beta),
                            eps, do_tanh, p_o, salt_o, _p(row_mask), _p(post_add), ldp, _p(y), ldy,
                            _p(mean), _p(rstd), M, D, dt, seed & 0xffffffff, _p(img), img_t, img_p,
                            _s()), "fs2_ln_fwd")


def ln_bwd(dy, lddy, s, lds, mean, rstd, gamma, beta, ds, ldds, M, D, *, dt, ws, seed=0,
           do_tanh=0, p_o=0.0, salt_o=0, row_mask=None, relu_gate_in=0, dr=None, p_r=0.0,
           salt_r=0, dgamma=None, dbeta=None, dcol=None):
    _chk(N.lib().fs2_ln_bwd(_p(dy), lddy, _p(s), lds, _p(mean), _p(rstd), _p(gamma), _p(beta),
                            do_tanh, p_o, salt_o, _p(row_mask), relu_gate_in, _p(ds), ldds, _p(dr),
                            p_r, salt_r, _p(dgamma), _p(dbeta), _p(dcol), M, D, dt,
                            seed & 0xffffffff,
                            _p(ws), _s()), "fs2_ln_bwd")


def ln_ws(M, D):
    return N.lib().fs2_ln_workspace_floats(M, D)


def attn_supported(T, dh, dt):
    return bool(N.lib().fs2_attn_supported(T, dh, dt))


def attn_fwd(qkv, ldq, key_pad, B, H, T, dh, scale, p_drop, seed, salt, out, ldo, lse, *, dt,
             mask_mode=1):
    """mask_mode 1: the FS2 head-major tiling quirk; 0: plain key padding."""
    _chk(N.lib().fs2_attn_fwd(_p(qkv), ldq, _p(key_pad), mask_mode, B, H, T, dh, scale, p_drop,
                              seed & 0xffffffff, salt, _p(out), ldo, _p(lse), dt, _s()),
         "fs2_attn_fwd")


def attn_bwd(qkv, ldq, key_pad, out, ldo, dout, lddo, lse, B, H, T, dh, scale, p_drop, seed, salt,
             dqkv, lddq, *, dt, ws, mask_mode=1):
    _chk(N.lib().fs2_attn_bwd(_p(qkv), ldq, _p(key_pad), mask_mode, _p(out), ldo, _p(dout), lddo,
                              _p(lse), B, H, T, dh, scale, p_drop, seed & 0xffffffff, salt,
                              _p(dqkv), lddq, _p(ws), dt, _s()), "fs2_attn_bwd")


def attn_ws(B, H, T):
    return N.lib().fs2_attn_workspace_floats(B, H, T)


def softmax_fwd(S, key_pad, B, H, Tq, Tk, ldt, scale, p_drop, seed, salt, P, Pd, *, dt,
                mask_mode=1):
    _chk(N.lib().fs2_softmax_fwd(_p(S), _p(key_pad), mask_mode, B, H, Tq, Tk, ldt, scale, p_drop,
                                 seed & 0xffffffff, salt, _p(P), _p(Pd), dt, _s()), "fs2_softmax_fwd")


def softmax_bwd(dPd, P, B, H, Tq, Tk, ldt, scale, p_drop, seed, salt, dS, *, dt):
    _chk(N.lib().fs2_softmax_bwd(_p(dPd), _p(P), B, H, Tq, Tk, ldt, scale, p_drop,
                                 seed & 0xffffffff, salt, _p(dS), dt, _s()), "fs2_softmax_bwd")


def embed_fwd(tokens, table, pe, pad_idx, B, T, D, X, keep, *, dt):
    _chk(N.lib().fs2_embed_fwd(_p(tokens), _p(table), _p(pe), pad_idx, B, T, D, _p(X), _p(keep),
                               dt, _s()), "fs2_embed_fwd")


def embed_bwd(tokens, dX, keep, M, D, V, dtable, *, dt, ws):
    _chk(N.lib().fs2_embed_bwd(_p(tokens), _p(dX), _p(keep), M, D, V, _p(dtable), _p(ws), dt,
                               _s()), "fs2_embed_bwd")


def embed_bwd_ws(D, V):
    return N.lib().fs2_embed_bwd_workspace_floats(D, V)


def keypad_from_tokens(tokens, pad_idx, M, key_pad):
    _chk(N.lib().fs2_keypad_from_tokens(_p(tokens), pad_idx, M, _p(key_pad), _s()),
         "fs2_keypad_from_tokens")


def keypad_from_lengths(lens, B, T, key_pad, keep=None):
    _chk(N.lib().fs2_keypad_from_lengths(_p(lens), B, T, _p(key_pad), _p(keep), _s()),
         "fs2_keypad_from_lengths")


def concat_fwd(feats, spk_table, spk, intensity, B, T, D, E, cat, ldc, *, dt):
    _chk(N.lib().fs2_concat_fwd(_p(feats), _p(spk_table), _p(spk), _p(intensity), B, T, D, E,
                                _p(cat), ldc, dt, _s()), "fs2_concat_fwd")


def concat_bwd_spk(dcat, ldc, spk, B, T, D, n_spk, dspk, *, dt, ws):
    _chk(N.lib().fs2_concat_bwd_spk(_p(dcat), ldc, _p(spk), B, T, D, n_spk, _p(dspk), dt, _p(ws),
                                    _s()),
         "fs2_concat_bwd_spk")


def mask_rows(X, ldx, keep, M, D, *, dt):
    _chk(N.lib().fs2_mask_rows(_p(X), ldx, _p(keep), M, D, dt, _s()), "fs2_mask_rows")


def add3_mask_rows(X, Y, Z, ld, keep, M, D, *, dt):
    """X = (X + Y + Z) * keep[row], fp32 sum, one rounding."""
    _chk(N.lib().fs2_add3_mask_rows(_p(X), _p(Y), _p(Z), ld, _p(keep), M, D, dt, _s()),
         "fs2_add3_mask_rows")


def rowdot_fwd(u, ldu, w, b, scale, M, D, y, *, dt):
    _chk(N.lib().fs2_rowdot_fwd(_p(u), ldu, _p(w), _p(b), scale, M, D, _p(y), dt, _s()),
         "fs2_rowdot_fwd")


def rowdot_bwd(dy, u, ldu, w, scale, M, D, du, dw, db, *, dt, ws):
    _chk(N.lib().fs2_rowdot_bwd(_p(dy), _p(u), ldu, _p(w), scale, M, D, _p(du), _p(dw), _p(db),
                                dt, _p(ws), _s()), "fs2_rowdot_bwd")


def avg_over_durations(values, Tm_in, durs, B, Tp, avg, ws):
    _chk(N.lib().fs2_avg_over_durations(_p(values), Tm_in, _p(durs), B, Tp, _p(avg), _p(ws), _s()),
         "fs2_avg_over_durations")


def avg_ws(B, Tm_in):
    return N.lib().fs2_avg_workspace_floats(B, Tm_in)


def embed1d_fwd(base, a, W, bias, B, T, D, KW, out, *, dt):
    _chk(N.lib().fs2_embed1d_fwd(_p(base), _p(a), _p(W), _p(bias), B, T, D, KW, _p(out), dt, _s()),
         "fs2_embed1d_fwd")


def embed1d_bwd(dout, a, B, T, D, KW, dW, dbias, *, dt, ws):
    _chk(N.lib().fs2_embed1d_bwd(_p(dout), _p(a), B, T, D, KW, _p(dW), _p(dbias), dt, _p(ws), _s()),
         "fs2_embed1d_bwd")


def lr_index(durs, d_is_float, pace, B, Tp, Tm, mel_len, cum, frame_src):
    _chk(N.lib().fs2_lr_index(_p(durs), d_is_float, pace, B, Tp, Tm, _p(mel_len), _p(cum),
                              _p(frame_src), _s()), "fs2_lr_index")


def lr_gather(X, frame_src, pe, B, Tp, Tm, D, Y, keep, *, dt):
    _chk(N.lib().fs2_lr_gather(_p(X), _p(frame_src), _p(pe), B, Tp, Tm, D, _p(Y), _p(keep), dt,
                               _s()), "fs2_lr_gather")


def lr_scatter(dY, cum, keep, B, Tp, Tm, D, dX, *, dt):
    _chk(N.lib().fs2_lr_scatter(_p(dY), _p(cum), _p(keep), B, Tp, Tm, D, _p(dX), dt, _s()),
         "fs2_lr_scatter")


def loss_fwd_bwd(desc):
    _chk(N.lib().fs2_loss_fwd_bwd(ctypes.byref(desc), _s()), "fs2_loss_fwd_bwd")


def loss_ws(B, Tm, NM):
    return N.lib().fs2_loss_workspace_floats(B, Tm, NM)


def adamw(param, grad, m, v, n, decay_mul, omb1, beta2, omb2, step_size, bc2_sqrt, eps, gscale):
    _chk(N.lib().fs2_adamw(_p(param), _p(grad), _p(m), _p(v), n, decay_mul, omb1, beta2, omb2,
                           step_size, bc2_sqrt, eps, gscale, _s()), "fs2_adamw")


def weight_prep(W, O, C, KW, Wf, ldf, Wb, ldb, *, dt, w_okc=0):
    _chk(N.lib().fs2_weight_prep(_p(W), O, C, KW, w_okc, _p(Wf), ldf, _p(Wb), ldb, dt, _s()),
         "fs2_weight_prep")


def intensity_input(x, layout_bct, B, T, C, X, ldx, *, dt):
    _chk(N.lib().fs2_intensity_input(_p(x), layout_bct, B, T, C, _p(X), ldx, dt, _s()),
         "fs2_intensity_input")


def intensity_head(H, ldh, emo_table, emotions, lengths, Wc, bc, B, T, D, E, I, *, dt):
    _chk(N.lib().fs2_intensity_head(_p(H), ldh, _p(emo_table), _p(emotions), _p(lengths), _p(Wc),
                                    _p(bc), B, T, D, E, _p(I), dt, _s()), "fs2_intensity_head")


def phoneme_average(I, T, E, durations, phon_len, B, Tp, out):
    _chk(N.lib().fs2_phoneme_average(_p(I), T, E, _p(durations), _p(phon_len), B, Tp, _p(out),
                                     _s()), "fs2_phoneme_average")


def collate_phonemes(order, offsets, phonemes, durations, B, Tp, phon_out, dur_out, in_len):
    _chk(N.lib().fs2_collate_phonemes(_p(order), _p(offsets), _p(phonemes), _p(durations), B, Tp,
                                      _p(phon_out), _p(dur_out), _p(in_len), _s()),
         "fs2_collate_phonemes")


def collate_frames(order, frame_offsets, mel, pitch, energy, B, Tm, n_mels, mel_out, pitch_out,
                   energy_out, rank_x, out_len):
    _chk(N.lib().fs2_collate_frames(_p(order), _p(frame_offsets), _p(mel), _p(pitch), _p(energy),
                                    B, Tm, n_mels, _p(mel_out), _p(pitch_out), _p(energy_out),
                                    _p(rank_x), _p(out_len), _s()), "fs2_collate_frames")


def weight_prep_table(entries):
    """Device table of fs2_wprep_desc for fs2_weight_prep_batched.  entries: list of
    (W, O, C, KW, w_okc, Wf, ldf, Wb, ldb); returns (table tensor, n, total_tiles).  The tensors
    must stay alive (and in place) as long as the table is used."""
    arr = (N.WPrepDesc * len(entries))()
    t0 = 0
    for i, (W, O, C, KW, okc, Wf, ldf, Wb, ldb) in enumerate(entries):
        tk = (ldf + 63) // 64
        arr[i] = N.WPrepDesc(_p(W), _p(Wf), _p(Wb), O, C, KW, okc, ldf, ldb, t0, tk)
        t0 += ((O + 63) // 64) * tk
    raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    dev = entries[0][0].device
    return raw.to(dev), len(entries), t0


def adamw_ranges_table(ranges, device):
    """int64 (start, length, first block) triples for fs2_adamw_prep's element-wise part."""
    rows, b0 = [], 0
    for st, ln in ranges:
        rows.append((st, ln, b0))
        b0 += (ln + 1023) // 1024
    t = torch.tensor(rows if rows else [(0, 0, 0)], dtype=torch.int64).reshape(-1)
    return t.to(device), len(rows), b0


def adamw_prep(wtable, rtable, param, grad, m, v, decay_mul, omb1, beta2, omb2, step_size,
               bc2_sqrt, eps, gscale, *, dt):
    (wt, n, tiles), (rt, nr, rb) = wtable, rtable
    _chk(N.lib().fs2_adamw_prep(_p(wt), n, tiles, _p(rt), nr, rb, _p(param), _p(grad), _p(m),
                                _p(v), decay_mul, omb1, beta2, omb2, step_size, bc2_sqrt, eps,
                                gscale, dt, _s()), "fs2_adamw_prep")


def weight_prep_batched(table, n, total_tiles, *, dt):
    _chk(N.lib().fs2_weight_prep_batched(_p(table), n, total_tiles, dt, _s()),
         "fs2_weight_prep_batched")


def vocoder_input(mel, B, n_mels, T, pad, X, ldx, *, dt):
    _chk(N.lib().fs2_vocoder_input(_p(mel), B, n_mels, T, pad, _p(X), ldx, dt, _s()),
         "fs2_vocoder_input")


def leaky_relu(x, y, n, slope, *, dt):
    _chk(N.lib().fs2_leaky_relu(_p(x), _p(y), n, slope, dt, _s()), "fs2_leaky_relu")


def mean3_leaky_relu(a, b, c, y, n, slope, *, dt):
    _chk(N.lib().fs2_mean3_leaky_relu(_p(a), _p(b), _p(c), _p(y), n, slope, dt, _s()),
         "fs2_mean3_leaky_relu")


def fill(X, n, value, *, dt):
    _chk(N.lib().fs2_fill(_p(X), n, value, dt, _s()), "fs2_fill")


def add(X, Y, n, alpha=1.0, *, dt):
    _chk(N.lib().fs2_add(_p(X), _p(Y), n, alpha, dt, _s()), "fs2_add")


def cast(src, src_dt, dst, dst_dt, n):
    _chk(N.lib().fs2_cast(_p(src), src_dt, _p(dst), dst_dt, n, _s()), "fs2_cast")


def set_dropout_seed(seed_base):
    """Device-resident dropout seed base added to every launch's seed (graph replays)."""
    _chk(N.lib().fs2_set_dropout_seed(int(seed_base) & 0xffffffff, _s()), "fs2_set_dropout_seed")
