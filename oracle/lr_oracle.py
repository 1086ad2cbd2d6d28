"""numpy + C oracle for the LengthRegulator index expansion and average_over_durations.

TEST INFRASTRUCTURE ONLY (see oracle/fs2_oracle.py header).  Restates SB ``upsample``
(model.py:406-410) and ``average_over_durations`` (App. A.10,
model.py:383,397); the C restatement (lr_oracle.c, built by ``make -C oracle``) is the
same algorithm and both must agree bit-exactly with each other and with the HIP kernels.
"""

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "liblr_oracle.so")


def lr_index_np(durs, pace=1.0, Tm=None):
    """durs (B,Tp) int64 or float32 -> (mel_len (B,), frame_src (B,Tm) int32, -1 padded)."""
    durs = np.asarray(durs)
    n = (np.float32(pace) * durs.astype(np.float32)).astype(np.float32).astype(np.int64)
    mel_len = n.sum(1)
    Tm = int(mel_len.max()) if Tm is None else Tm
    B, Tp = durs.shape
    fs = np.full((B, Tm), -1, dtype=np.int32)
    for b in range(B):
        idx = np.repeat(np.arange(Tp, dtype=np.int32), n[b])[:Tm]
        fs[b, :len(idx)] = idx
    return mel_len, fs


def avg_over_durations_np(values, durs):
    """values (B,Tm) float32, durs (B,Tp) int -> (B,Tp) float32 (torch-CPU cumsum semantics)."""
    values = np.asarray(values, dtype=np.float32)
    durs = np.asarray(durs, dtype=np.int64)
    B, Tm = values.shape
    vc = np.zeros((B, Tm + 1), dtype=np.float32)
    vc[:, 1:] = np.cumsum(values.astype(np.float64), axis=1).astype(np.float32)
    nc = np.zeros((B, Tm + 1), dtype=np.int64)
    nc[:, 1:] = np.cumsum(values != 0.0, axis=1)
    ends = np.clip(np.cumsum(durs, axis=1), 0, Tm)
    starts = np.concatenate([np.zeros((B, 1), np.int64), ends[:, :-1]], axis=1)
    sums = (np.take_along_axis(vc, ends, 1) - np.take_along_axis(vc, starts, 1)).astype(np.float32)
    nel = (np.take_along_axis(nc, ends, 1) - np.take_along_axis(nc, starts, 1)).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        out = np.where(nel == 0.0, nel, sums / nel)
    return out.astype(np.float32)


def _c():
    if not os.path.exists(_LIB):
        raise FileNotFoundError(f"{_LIB} missing: run `make -C oracle`")
    lib = ctypes.CDLL(_LIB)
    lib.fs2o_lr_index.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.fs2o_avg_over_durations.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


def lr_index_c(durs, pace=1.0, Tm=None):
    durs = np.ascontiguousarray(durs)
    B, Tp = durs.shape
    if Tm is None:
        Tm = int(lr_index_np(durs, pace)[0].max())
    mel_len = np.zeros(B, np.int64)
    fs = np.zeros((B, Tm), np.int32)
    if durs.dtype == np.int64:
        _c().fs2o_lr_index(durs.ctypes.data, None, pace, B, Tp, Tm, mel_len.ctypes.data, fs.ctypes.data)
    else:
        d = np.ascontiguousarray(durs, dtype=np.float32)
        _c().fs2o_lr_index(None, d.ctypes.data, pace, B, Tp, Tm, mel_len.ctypes.data, fs.ctypes.data)
    return mel_len, fs


def avg_over_durations_c(values, durs):
    values = np.ascontiguousarray(values, dtype=np.float32)
    durs = np.ascontiguousarray(durs, dtype=np.int64)
    B, Tm = values.shape
    Tp = durs.shape[1]
    out = np.zeros((B, Tp), np.float32)
    _c().fs2o_avg_over_durations(values.ctypes.data, Tm, durs.ctypes.data, B, Tp, out.ctypes.data)
    return out
