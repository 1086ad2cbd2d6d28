"""ctypes binding of the C ABI in ``include/fs2_hip.h`` (libfs2_hip.so, gfx950).

This is the ONLY way the product path reaches compute: there is no CPU fallback and
no torch-op fallback.  If the shared library is missing or a symbol is absent the import
fails loudly (``NativeLibraryError``) -- on a GPU box that means "run build()", never
"silently use something else".
"""

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FS2_HIP_LIB", os.path.join(_HERE, "libfs2_hip.so"))
# The measurement build (``make experiments`` -> libfs2_hip_exp.so, -DFS2_EXPERIMENTS) is the
# only one whose FS2_* A/B switches do anything; the host side honours them under the same
# condition, so the product path has one configuration.
EXPERIMENTS = os.path.basename(LIB_PATH).startswith("libfs2_hip_exp")


def exp_flag(name, default=False):
    """FS2_* boolean A/B switch: read only with the experiments library, else ``default``."""
    if not EXPERIMENTS:
        return default
    v = os.environ.get(name)
    return default if v is None else v not in ("", "0")


def exp_int(name, default):
    """FS2_* integer A/B switch: read only with the experiments library, else ``default``."""
    if not EXPERIMENTS:
        return default
    v = os.environ.get(name)
    return default if v is None else int(v)

F32 = 0
BF16 = 1


class NativeLibraryError(RuntimeError):
    pass


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("kvalid", ctypes.c_int),
        ("mvalid", ctypes.c_int), ("nvalid", ctypes.c_int), ("dtype", ctypes.c_int),
        ("A", ctypes.c_void_p), ("lda", ctypes.c_int64), ("a_kmajor", ctypes.c_int),
        ("B", ctypes.c_void_p), ("ldb", ctypes.c_int64), ("b_kmajor", ctypes.c_int),
        ("conv_mode", ctypes.c_int), ("conv_t", ctypes.c_int), ("conv_kw", ctypes.c_int),
        ("conv_c", ctypes.c_int),
        ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64), ("c_fp32", ctypes.c_int),
        ("c_conv_kw", ctypes.c_int),
        ("bias", ctypes.c_void_p), ("relu", ctypes.c_int),
        ("gate", ctypes.c_void_p), ("ldg", ctypes.c_int64),
        ("row_scale", ctypes.c_void_p),
        ("residual", ctypes.c_void_p), ("ldr", ctypes.c_int64),
        ("row_scale_post", ctypes.c_void_p),
        ("accumulate", ctypes.c_int), ("split_k", ctypes.c_int),
        ("split_stride", ctypes.c_int64),
        ("batch", ctypes.c_int), ("batch_div", ctypes.c_int),
        ("sA1", ctypes.c_int64), ("sA2", ctypes.c_int64), ("sB1", ctypes.c_int64),
        ("sB2", ctypes.c_int64), ("sC1", ctypes.c_int64), ("sC2", ctypes.c_int64),
        ("sR1", ctypes.c_int64), ("sR2", ctypes.c_int64), ("conv_dil", ctypes.c_int),
        ("c_row_t", ctypes.c_int), ("c_row_pad", ctypes.c_int), ("max_ctas", ctypes.c_int),
        ("a_kw", ctypes.c_int),
    ]


class LossDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("Tm", ctypes.c_int), ("Tp", ctypes.c_int), ("NM", ctypes.c_int),
        ("dtype", ctypes.c_int),
        ("mel_out", ctypes.c_void_p), ("postnet_out", ctypes.c_void_p),
        ("log_dur", ctypes.c_void_p), ("pitch_pred", ctypes.c_void_p),
        ("energy_pred", ctypes.c_void_p),
        ("mel_tgt", ctypes.c_void_p), ("dur_tgt", ctypes.c_void_p),
        ("pitch_avg", ctypes.c_void_p), ("energy_avg", ctypes.c_void_p),
        ("mel_len", ctypes.c_void_p), ("phon_len", ctypes.c_void_p),
        ("w_ssim", ctypes.c_float), ("w_mel", ctypes.c_float), ("w_post", ctypes.c_float),
        ("w_dur", ctypes.c_float), ("w_pitch", ctypes.c_float), ("w_energy", ctypes.c_float),
        ("loss_out", ctypes.c_void_p),
        ("d_mel_out", ctypes.c_void_p), ("d_postnet_out", ctypes.c_void_p),
        ("d_log_dur", ctypes.c_void_p), ("d_pitch", ctypes.c_void_p), ("d_energy", ctypes.c_void_p),
        ("workspace", ctypes.c_void_p),
    ]


class WPrepDesc(ctypes.Structure):
    _fields_ = [
        ("W", ctypes.c_void_p), ("Wf", ctypes.c_void_p), ("Wb", ctypes.c_void_p),
        ("O", ctypes.c_int), ("C", ctypes.c_int), ("KW", ctypes.c_int), ("w_okc", ctypes.c_int),
        ("ldf", ctypes.c_int), ("ldb", ctypes.c_int), ("tile0", ctypes.c_int),
        ("tiles_k", ctypes.c_int),
    ]


P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
U32 = ctypes.c_uint32
Fl = ctypes.c_float

# name -> (restype, argtypes); must match include/fs2_hip.h exactly
SIGNATURES = {
    "fs2_gemm": (I, [ctypes.POINTER(GemmDesc), P]),
    "fs2_colsum": (I, [P, I64, I, I, I, P, I, P, P]),
    "fs2_conv_fold": (I, [P, I, I64, I, I, I, I, P, I64, P, I64, P, P, I, P]),
    "fs2_colsum_workspace_floats": (I64, [I, I]),
    "fs2_sum_slices": (I, [P, I, I64, I64, P, I, P]),
    "fs2_pad_transpose": (I, [P, I64, I, I, I, I, I, P, I64, I, P, P, I, P]),
    "fs2_pad_rows": (I, [P, I64, I, I, I, I, I, I, P, I64, I, P]),
    "fs2_ln_fwd": (I, [P, I64, P, I64, Fl, U32, P, P, P, Fl, I, Fl, U32, P, P, I64, P, I64, P, P,
                       I, I, I, U32, P, I, I, P]),
    "fs2_ln_bwd": (I, [P, I64, P, I64, P, P, P, P, I, Fl, U32, P, I, P, I64, P, Fl, U32, P, P, P,
                       I, I, I, U32, P, P]),
    "fs2_ln_workspace_floats": (I64, [I, I]),
    "fs2_attn_supported": (I, [I, I, I]),
    "fs2_attn_fwd": (I, [P, I64, P, I, I, I, I, I, Fl, Fl, U32, U32, P, I64, P, I, P]),
    "fs2_attn_bwd": (I, [P, I64, P, I, P, I64, P, I64, P, I, I, I, I, Fl, Fl, U32, U32, P, I64,
                         P, I, P]),
    "fs2_attn_workspace_floats": (I64, [I, I, I]),
    "fs2_softmax_fwd": (I, [P, P, I, I, I, I, I, I, Fl, Fl, U32, U32, P, P, I, P]),
    "fs2_softmax_bwd": (I, [P, P, I, I, I, I, I, Fl, Fl, U32, U32, P, I, P]),
    "fs2_embed_fwd": (I, [P, P, P, I, I, I, I, P, P, I, P]),
    "fs2_embed_bwd": (I, [P, P, P, I, I, I, P, P, I, P]),
    "fs2_embed_bwd_workspace_floats": (I64, [I, I]),
    "fs2_keypad_from_tokens": (I, [P, I, I, P, P]),
    "fs2_keypad_from_lengths": (I, [P, I, I, P, P, P]),
    "fs2_concat_fwd": (I, [P, P, P, P, I, I, I, I, P, I, I, P]),
    "fs2_concat_bwd_spk": (I, [P, I, P, I, I, I, I, P, I, P, P]),
    "fs2_mask_rows": (I, [P, I64, P, I, I, I, P]),
    "fs2_add3_mask_rows": (I, [P, P, P, I64, P, I, I, I, P]),
    "fs2_rowdot_fwd": (I, [P, I64, P, P, Fl, I, I, P, I, P]),
    "fs2_rowdot_bwd": (I, [P, P, I64, P, Fl, I, I, P, P, P, I, P, P]),
    "fs2_avg_over_durations": (I, [P, I, P, I, I, P, P, P]),
    "fs2_avg_workspace_floats": (I64, [I, I]),
    "fs2_embed1d_fwd": (I, [P, P, P, P, I, I, I, I, P, I, P]),
    "fs2_embed1d_bwd": (I, [P, P, I, I, I, I, P, P, I, P, P]),
    "fs2_lr_index": (I, [P, I, Fl, I, I, I, P, P, P, P]),
    "fs2_lr_gather": (I, [P, P, P, I, I, I, I, P, P, I, P]),
    "fs2_lr_scatter": (I, [P, P, P, I, I, I, I, P, I, P]),
    "fs2_loss_fwd_bwd": (I, [ctypes.POINTER(LossDesc), P]),
    "fs2_loss_workspace_floats": (I64, [I, I, I]),
    "fs2_adamw": (I, [P, P, P, P, I64, Fl, Fl, Fl, Fl, Fl, Fl, Fl, Fl, P]),
    "fs2_weight_prep": (I, [P, I, I, I, I, P, I, P, I, I, P]),
    "fs2_weight_prep_batched": (I, [P, I, I, I, P]),
    "fs2_adamw_prep": (I, [P, I, I, P, I, I, P, P, P, P, Fl, Fl, Fl, Fl, Fl, Fl, Fl, Fl, I, P]),
    "fs2_intensity_input": (I, [P, I, I, I, I, P, I, I, P]),
    "fs2_intensity_head": (I, [P, I64, P, P, P, P, P, I, I, I, I, P, I, P]),
    "fs2_phoneme_average": (I, [P, I, I, P, P, I, I, P, P]),
    "fs2_collate_phonemes": (I, [P, P, P, P, I, I, P, P, P, P]),
    "fs2_collate_frames": (I, [P, P, P, P, P, I, I, I, P, P, P, P, P, P]),
    "fs2_vocoder_input": (I, [P, I, I, I, I, P, I, I, P]),
    "fs2_leaky_relu": (I, [P, P, I64, Fl, I, P]),
    "fs2_mean3_leaky_relu": (I, [P, P, P, P, I64, Fl, I, P]),
    "fs2_fill": (I, [P, I64, Fl, I, P]),
    "fs2_add": (I, [P, P, I64, Fl, I, P]),
    "fs2_cast": (I, [P, I, P, I, I64, P]),
    "fs2_set_dropout_seed": (I, [U32, P]),
    "fs2_version": (ctypes.c_char_p, []),
    "fs2_source_hash": (ctypes.c_char_p, []),
}

_lib = None


_CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
_HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "fs2_hip.h")


def source_hash():
    """SHA-256 (first 16 hex digits) of the library's sources in this tree, in the Makefile's
    HASH_SRCS order (csrc/*.hip by name, csrc/fs2_common.h, include/fs2_hip.h); None when the
    sources are not present."""
    import hashlib
    names = sorted(f for f in os.listdir(_CSRC) if f.endswith(".hip")) if os.path.isdir(_CSRC) else []
    files = [os.path.join(_CSRC, f) for f in names] + [os.path.join(_CSRC, "fs2_common.h"), _HEADER]
    if not names or not all(os.path.exists(f) for f in files):
        return None
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load(path=None):
    """Load libfs2_hip.so and bind every symbol of include/fs2_hip.h (fail loudly)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NativeLibraryError(
            f"libfs2_hip.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950). There is no fallback path.")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    missing = []
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing:
        raise NativeLibraryError(f"libfs2_hip.so is missing symbols: {missing}")
    built, tree = lib.fs2_source_hash().decode(), source_hash()
    # FS2_LIB_OTHER_SOURCES=1: a deliberately older build (tools/ab_lib.sh's A arm)
    if tree is not None and built != tree and os.environ.get("FS2_LIB_OTHER_SOURCES") != "1":
        raise NativeLibraryError(
            f"{p} was built from other sources (hash {built}, this tree's csrc {tree}): rebuild "
            f"it with `python -c 'import __graft_entry__ as g; g.build()'`")
    if path is None:
        _lib = lib
    return lib


def lib():
    return load()


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_dev = torch._C._cuda_getDevice


def stream_ptr():
    """torch's current HIP stream on the current device, as a raw pointer.  (The C accessors:
    torch.cuda.current_stream() builds a Stream object and re-checks lazy init and the device
    index on every call -- ~5 us, 700+ times a step, which was a quarter of the host's
    enqueue time.)"""
    return _raw_stream(_cur_dev())


def check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise ValueError(f"unsupported activation dtype {dt}")
