"""Explicit forward / backward of the FastSpeech2-with-emotion-intensity train step on the
MI355X kernels of libfs2_hip.so.

The reference runs ``FastSpeech2.forward`` (emo_rank_tts/fastspeech2/model.py:279-441) through
speechbrain lobes and lets autograd derive the backward.  Here the whole step is written out
by hand so that every byte of activation traffic is known: each GEMM-shaped op goes through
``fs2_gemm`` (implicit reflect-padded convolution, fused bias/ReLU/mask/residual epilogues),
LayerNorms fuse their residual add + dropout, attention masks reproduce the head-major
tiling quirk, and parameter gradients are written straight into one flat fp32 buffer
(``model._gflat``) laid out in backward-completion order, ready for a bucketed all-reduce.

Activation storage dtype is fp32 (parity mode) or bf16 (throughput mode); parameters,
gradients, LayerNorm statistics and losses are fp32 in both.
"""

import math
import re

import torch

from . import _native as N
from . import ops
from .ops import round_up

_BK = {N.F32: 32, N.BF16: 64}


class _Salt:
    def __init__(self):
        self.n = 0

    def __call__(self):
        self.n += 1
        return self.n


_NO_FLASH = N.exp_flag("FS2_NO_FLASH")


def dgrad_split(Mp, C, K, dt, n_cu=256, max_split=8):
    """K split for the shift-conv data gradient, chosen for wave quantisation over the 256 CUs
    (one 256x128 tile per CU at a time): the decoder's 372 tiles fill 1.45 rounds (73 %), two
    slices fill 2.9 (97 %); the encoder's 78 tiles fill 30 %, three slices 91 %.  Slices are
    fp32 planes summed by fs2_conv_fold, so a split must gain > 5 % occupancy to pay for its
    extra plane."""
    if dt != 1:
        return 1
    if not _NO_PS and _PS_MODES & 4 and K >= 2048 and C >= 128 and C % 4 == 0:
        # the persistent 256 x 192 / 256 x 256 kernel (gemm_ps_kernel) takes an unsplit data
        # gradient when its tiles fill most of one round (the decoder: 124 x 2 = 248 tiles)
        w = 192 if C % 256 and -(-C // 192) * 192 < -(-C // 256) * 256 else 256
        if -(-Mp // 256) * -(-C // w) >= 200:
            return 1
    tiles = -(-Mp // 256) * -(-C // 128)

    def eff(s):
        return tiles * s / (n_cu * -(-(tiles * s) // n_cu))

    best, best_eff = 1, eff(1)
    for s in range(2, max(1, min(max_split, (K // 64) // 8)) + 1):
        if eff(s) > best_eff + 0.05:
            best, best_eff = s, eff(s)
    return best


_NO_SLICES = N.exp_flag("FS2_NO_WGRAD_SLICES")
_NO_PS = N.exp_flag("FS2_GEMM_NO_PS")
_PS_MODES = N.exp_int("FS2_PS_MODES", 5)
# large weight gradients (the FFN conv1 weights, 5.3 M floats) as split-K planes + fixed-order
# sum instead of split-K fp32 atomics: decoder 428 -> 420 us, encoder 128 -> 119 us, and the
# result no longer depends on atomic ordering.  FS2_NO_WGRAD_BIG_SLICES=1 restores the atomics.
_BIG_SLICES = not N.exp_flag("FS2_NO_WGRAD_BIG_SLICES")
_SLICE_TARGET = N.exp_int("FS2_WGRAD_SLICE_TARGET", 240)
# CU budget of the small weight gradients' split-K on the side stream: sliced ones fill
# _WG_SLICE_CU CUs, the atomic ones _WG_ATOMIC_UNITS (tile, split) units (experiments build)
_WG_SLICE_CU = N.exp_int("FS2_WG_SLICE_CU", 256)
_WG_ATOMIC_UNITS = N.exp_int("FS2_WG_ATOMIC_UNITS", 512)
# conv weight gradients with both operands K-major (channel-major padded images, conv_mode 6):
# FS2_KM_WGRAD=0 restores the MN-major implicit-conv GEMM for A/B runs
_KM_WGRAD = N.exp_int("FS2_KM_WGRAD", 1)
# decoder FFN conv1 data gradient over the zero-padded dY image (engine._pad_dgrad)
_PAD_DGRAD = N.exp_int("FS2_PAD_DGRAD", 1)
# FFN conv1 forward over a reflect-padded X image (engine._pad_fwd)
_PAD_FWD = N.exp_int("FS2_PAD_FWD", 2)
# decoder FFN conv1 data gradient in the tap-inner K order (engine._tap_inner): off -- 11 %
# faster standalone and 190 instead of 995 MB read, but the step measured 0.03-0.08 ms slower
# with it in three same-box A/Bs (17.18 vs 17.13 ms on the final tree); the FFN conv1 forward in
# that order (engine._tap_inner_fwd): off -- 316-318 vs 314 us for the decoder's in the step,
# step 17.42 vs 17.37 ms (experiments library, 2 x 2 interleaved)
_TAP_INNER = N.exp_int("FS2_TAP_INNER", 0)
# the FFN conv1 forward's padded image written by the LayerNorm before it (FS2_LN_IMG=0,
# experiments build: a separate fs2_pad_rows pass)
_LN_IMG = N.exp_int("FS2_LN_IMG", 1)
_TAP_INNER_FWD = N.exp_int("FS2_TAP_INNER_FWD", 0)
# serial mode for per-call-site timing (bench.py --detail runs with the experiments library)
_NO_SIDE = N.exp_flag("FS2_NO_SIDE_STREAM")
_NO_AUX = N.exp_flag("FS2_NO_AUX_STREAM")
# persistent-GEMM grid budget of the weight-gradient side stream (fs2_gemm_desc.max_ctas, passed
# with every weight-gradient GEMM enqueued there): the CUs it leaves free take the main stream's LayerNorm / reduction / short GEMM launches, which
# otherwise queue behind side-stream blocks that hold a whole CU's registers.  Same-box sweep
# (tools/r04_side.sh, 2 x 7 interleaved bench runs): 256 -> 18.23-18.29 ms, 176-240 ->
# 18.01-18.13, 160 -> 18.87; 208 kept.  FS2_SIDE_CTAS overrides in the experiments build.
_SIDE_CTAS = N.exp_int("FS2_SIDE_CTAS", 208)
# AdamW of the decoder / mel-linear / PostNet parameters on the aux stream during the encoder
# backward (FusedTrainer.step, one process); FS2_ADAM_OVERLAP=0 (experiments build): one launch
_ADAM_OVERLAP = N.exp_int("FS2_ADAM_OVERLAP", 1)
# the energy predictor's forward and backward on the aux stream (FS2_AUX_ENERGY=0: on the main
# stream, its backward fused into the residual epilogue, for A/B runs)
_AUX_ENERGY = N.exp_int("FS2_AUX_ENERGY", 1)
# the pitch / energy embedding and speaker-embedding weight gradients on the side stream
# (FS2_SIDE_SMALL=0: on the main stream, for A/B runs)
_SIDE_SMALL = N.exp_int("FS2_SIDE_SMALL", 1)


def ps_plain_ok(M, lda, N, ldb, out_rows, ldc, out_bytes):
    """fs2_gemm can take a padded-domain GEMM (c_row output remap) only on its persistent
    kernel: plain operands enabled (FS2_GEMM_NO_PS / FS2_PS_MODES bit 0 in the experiments
    build) and every operand within the kernel's 32-bit buffer offsets -- otherwise the engine
    keeps the implicit-conv path instead of handing fs2_gemm a call it refuses."""
    lim = 0x7fffffff
    return (not _NO_PS and bool(_PS_MODES & 1) and M * lda * 2 < lim and N * ldb * 2 < lim and
            out_rows * ldc * out_bytes < lim)


def eff_split(K, ns, bk):
    """the split-K slice count fs2_gemm actually uses for ``ns`` requested slices of K (it
    rounds the K-tiles per slice up, which can leave trailing slices empty -- those it zeroes
    with a memset so a consumer summing all ``ns`` stays right).  Requesting this count instead
    skips the memset launch."""
    if ns <= 1:
        return 1
    nkt = -(-K // bk)
    return -(-nkt // -(-nkt // ns))


def wgrad_slices(O, Ncols, ldc, K, dt, n_cu=256):
    """Split-K slice count for a weight gradient with a small output: enough 256x128 tiles x
    slices to fill the 256 CUs once, each slice >= 8 K-tiles; slices are fp32 planes summed in
    a fixed order instead of tens of fp32 atomics landing on every output element.  Applied
    where it measured faster (bench.py --detail, FS2_NO_WGRAD_SLICES=1 for the A/B): outputs of
    >= 256 rows and <= 256 K elements (out-projection 62 -> 55 us, PostNet conv_pre 73 -> 57 us),
    or <= 600 K elements over encoder-length K (conv2 58 -> 42 us, out-projection 47 -> 31 us).
    1 = the atomic split-K path (decoder conv2 91 vs 144 us, PostNet 150 vs 231 us)."""
    if dt != 1 or ldc % 8 or Ncols != ldc or O < 256:
        return 1
    n = O * ldc
    if not (n <= (1 << 18) or (n <= 600_000 and K <= 8192)):
        return 1
    tiles = -(-O // 256) * -(-Ncols // 128)
    ns = min(-(-n_cu // tiles), max(1, (K // 64) // 8))
    return ns if ns >= 2 else 1


class FS2Engine:
    def __init__(self, model, act_dtype=torch.float32):
        self.m = model
        self.cfg = model.cfg
        self.adt = act_dtype
        self.dt = N.dtype_code(act_dtype)
        self.epc = ops.EPC[self.dt]
        N.load()
        model._ensure_packed()
        self.dev = model._flat.device
        self.params = dict(model.named_parameters())
        self.grads = dict(model._grad_views)
        self.pe_enc = model.sinusoidal_positional_embed_encoder.pe[0].float().contiguous()
        self.pe_dec = model.sinusoidal_positional_embed_decoder.pe[0].float().contiguous()
        self._ws = torch.empty(1 << 20, dtype=torch.float32, device=self.dev)
        self._ws_key = torch.cuda.current_stream(self.dev).cuda_stream
        self._ws_other = {}
        self._side = torch.cuda.Stream(self.dev) if (self.dt == N.BF16 and not _NO_SIDE) else None
        # grid budget of the persistent GEMMs this engine enqueues on its side stream (per call,
        # in the GEMM descriptor: no library state, whichever stream handle torch recycles)
        self._side_ctas = min(256, max(8, _SIDE_CTAS // 8 * 8)) if self._side is not None else 256
        # duration / pitch predictor chains (independent of the rest of the step when the
        # pitch target is given) run on a third stream; their weight gradients stay on it
        self._aux = torch.cuda.Stream(self.dev) if (self._side is not None and not _NO_AUX) else None
        self.w = {}
        self._wspecs = self._weight_specs()
        self._fuse_pred_conv1()
        self._prepared_version = None
        self._wtable = None          # device descriptor table of every GEMM weight image
        self.on_grads_ready = None   # optional callback(tag) for DP overlap
        self.timer = None            # optional KernelTimer: HIP events around tagged launches
        self._km = {}                # conv_mode-6 images, reused layer after layer (side stream)
        self._img = {}               # per-layer zero-padded dY images (_dy_image)
        self._fimg = {}              # padded FFN conv1 forward images (_fwd_image)
        # FusedTrainer.step sets adam_split = (optimizer, AdamW scalars): the backward then updates
        # the parameters whose gradients are final after the decoder (_adam_late) on the aux
        # stream while the main stream runs the encoder backward; adamw_step_split does the rest
        self.adam_split = None
        self._adam_late_done = False
        # DP (FusedTrainer): (ready(), wait(stream)) of the gradient buckets holding the late
        # parameters -- the late AdamW is launched from the notify hook once they are all queued,
        # its aux stream waiting for their all-reduce
        self.dp_late = None
        self.n_adam_late = 0         # late AdamW launches from inside the backward (tests)
        self._adam_tabs = None

    def _fwd_image(self, rows, tail, C):
        """the FFN conv1 forward's padded image [rows + tail][C], one per shape: every layer's
        forward rewrites its first ``rows`` rows before the GEMM reads them (main stream), and
        the ``tail`` rows past them stay zero"""
        key = (rows, tail, C, self.adt)
        img = self._fimg.get(key)
        if img is None:
            img = self.empty(rows + tail, C)
            img[rows:].zero_()
            self._fimg[key] = img
        return img

    def _tic(self, tag):
        if self.timer is not None:
            self.timer.start(tag)

    def _toc(self, tag):
        if self.timer is not None:
            self.timer.stop(tag)

    # ------------------------------------------------------------------ helpers
    def use_flash(self, T, dh):
        """fused attention kernels on the bf16 path (fp32 parity mode keeps the materialised
        softmax); FS2_NO_FLASH=1 forces the materialised path for A/B runs."""
        return self.dt == 1 and not _NO_FLASH and ops.attn_supported(T, dh, self.dt)

    def ws(self, n):
        """scratch buffer of the CURRENT stream (the weight-gradient side stream has its own)"""
        n = int(n)
        key = N.stream_ptr()
        buf = self._ws if key == self._ws_key else self._ws_other.get(key)
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(int(n * 1.25) + 1024, 1 << 20), dtype=torch.float32,
                              device=self.dev)
            if key == self._ws_key:
                self._ws = buf
            else:
                self._ws_other[key] = buf
        return buf

    # ------------------------------------------------------------------ side stream
    # Weight and bias gradients depend only on tensors the data-gradient chain has already
    # produced, so they run on a second stream: the encoder's GEMMs (M = 6400) and the tail
    # rounds of the decoder's leave CUs idle that the other chain fills.
    def _side_enter(self, *tensors):
        if self._side is None:
            return None
        main = torch.cuda.current_stream(self.dev)
        if self._aux is not None and main.cuda_stream == self._aux.cuda_stream:
            return None          # the aux chain is already off the critical path
        self._side.wait_stream(main)
        ctx = torch.cuda.stream(self._side)
        ctx.__enter__()
        return ctx, tensors

    def _side_exit(self, h):
        if h is None:
            return
        ctx, tensors = h
        ctx.__exit__(None, None, None)
        for t in tensors:
            if t is not None:
                t.record_stream(self._side)

    def _aux_fork(self, *tensors):
        """enter the aux stream after everything queued so far on the current stream"""
        main = torch.cuda.current_stream(self.dev)
        self._aux.wait_stream(main)
        for t in tensors:
            if t is not None:
                t.record_stream(self._aux)
        ctx = torch.cuda.stream(self._aux)
        ctx.__enter__()
        return ctx, main

    def _aux_exit(self, h):
        h[0].__exit__(None, None, None)

    def _aux_join(self, main, *tensors):
        """the main stream waits for the aux chain; its outputs are now used on main"""
        main.wait_stream(self._aux)
        for t in tensors:
            if t is not None:
                t.record_stream(main)

    def _flat_is(self, flat):
        """the engine's weight-image table was built over this flat parameter buffer"""
        return self.m._flat is flat and self.dev == flat.device

    def grad_streams(self):
        """streams that may hold queued parameter-gradient writes (the aux stream's are joined
        into the main stream before the variance group completes)"""
        main = torch.cuda.current_stream(self.dev)
        return [main] if self._side is None else [main, self._side]

    def side_join(self):
        if self._side is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self._side)

    def empty(self, *shape, dtype=None):
        return torch.empty(*shape, dtype=dtype or self.adt, device=self.dev)

    # the duration and pitch predictors' conv1 (same input Z, model.py:366,379) as one conv with
    # 2 x 384 output channels: forward and weight gradient are single N = 768 GEMMs, and the data
    # gradient one K = 3 x 768 GEMM that also sums the two predictors' input gradients
    PRED1 = "varPred.conv1"

    def _fuse_pred_conv1(self):
        """register the fused duration / pitch conv1 weight, bias and gradients (flat-buffer
        views over the two adjacent parameters, model._group_key) in place of the two specs"""
        wd, wp = "durPred.conv1.conv.weight", "pitchPred.conv1.conv.weight"
        bd, bp = "durPred.conv1.conv.bias", "pitchPred.conv1.conv.bias"
        self._gemm_params = set(self._wspecs)
        if wd not in self._wspecs or self._wspecs[wd] != self._wspecs[wp]:
            return
        lay = {n: (o, k) for n, o, k, _, _ in self.m._layout}
        O, C, KW = self._wspecs[wd]
        if not (lay[wp][0] == lay[wd][0] + lay[wd][1] and lay[bp][0] == lay[bd][0] + lay[bd][1]):
            return
        f, gf = self.m._flat, self.m._gflat
        ow, nw = lay[wd][0], 2 * lay[wd][1]
        ob = lay[bd][0]
        del self._wspecs[wd], self._wspecs[wp]
        self._wspecs[self.PRED1] = (2 * O, C, KW)
        self.params[self.PRED1 + ".weight"] = f[ow:ow + nw].view(2 * O, KW, C).permute(0, 2, 1)
        self.grads[self.PRED1] = gf[ow:ow + nw].view(2 * O, KW, C).permute(0, 2, 1)
        self.params[self.PRED1 + ".bias"] = f[ob:ob + 2 * O]
        # the fused gradient view covers the same flat range as the two per-predictor conv1
        # weight-gradient views: drop those, so nothing that walks self.grads counts it twice
        del self.grads[wd], self.grads[wp]

    def _weight_specs(self):
        """name -> (O, C, KW, ldf, ldb_rows) for every GEMM weight."""
        c = self.cfg
        D = c.enc_d_model
        specs = {}
        for stack, L, F in (("encoder", c.enc_num_layers, c.enc_ffn_dim),
                            ("decoder", c.dec_num_layers, c.dec_ffn_dim)):
            k0, k1 = c.ffn_cnn_kernel_size_list
            for i in range(L):
                p = f"{stack}.layers.{i}."
                specs[p + "self_att.att.in_proj_weight"] = (3 * D, D, 1)
                specs[p + "self_att.att.out_proj.weight"] = (D, D, 1)
                specs[p + "pos_ffn.0.conv.weight"] = (F, D, k0)
                specs[p + "pos_ffn.2.conv.weight"] = (D, F, k1)
        specs["concat_proj.w.weight"] = (D, 2 * D + 5, 1)
        for pred in ("durPred", "pitchPred", "energyPred"):
            k = c.dur_pred_kernel_size
            specs[f"{pred}.conv1.conv.weight"] = (D, D, k)
            specs[f"{pred}.conv2.conv.weight"] = (D, D, k)
        specs["linear.w.weight"] = (c.n_mels, D, 1)
        E, KP = c.postnet_embedding_dim, c.postnet_kernel_size
        specs["postnet.conv_pre.conv.weight"] = (E, c.n_mels, KP)
        for i in range(c.postnet_n_convolutions - 2):
            specs[f"postnet.convs_intermedite.{i}.conv.weight"] = (E, E, KP)
        specs["postnet.conv_post.conv.weight"] = (c.n_mels, E, KP)
        return specs

    def prepare_weights(self, force=False):
        """fp32 master weights -> K-major GEMM images in the activation dtype (fwd + dgrad), all
        weights in one fs2_weight_prep_batched launch per parameter update."""
        ver = (self.m._param_version, self.m._flat._version)
        if torch.cuda.is_current_stream_capturing():
            force = True     # a captured step must re-prepare on every replay
        if not force and self._prepared_version == ver:
            return
        if self._wtable is None:
            entries = []
            self._wentries = {}
            for name, (O, C, KW) in self._wspecs.items():
                ldf = round_up(KW * C, self.epc)
                ldb = KW * O
                if name not in self.w:
                    self.w[name] = (self.empty(O, ldf), self.empty(C, ldb))
                Wf, Wb = self.w[name]
                W = self.params[name + ".weight" if name == self.PRED1 else name]
                # conv weights are [O][KW][C] in the flat buffer (model._kw_major); the FFN
                # conv1 data-gradient image has its taps reversed on the padded-dY path, and
                # its columns in tap-inner 64-channel chunks where that GEMM reads the image
                # in that order (_tap_inner)
                okc = int(KW > 1) | (2 if self._pad_dgrad(name) else 0) | \
                    (4 if self._tap_inner(name) else 0) | \
                    (8 if self._tap_inner_fwd(name) else 0)
                entries.append((W, O, C, KW, okc, Wf, ldf, Wb, ldb))
                self._wentries[name] = entries[-1]
            self._wtable = ops.weight_prep_table(entries)
        ops.weight_prep_batched(*self._wtable, dt=self.dt)
        self._prepared_version = ver

    def _adam_ranges(self):
        """flat (start, length) ranges of every parameter that is not a GEMM weight (the
        element-wise part of fs2_adamw_prep); neighbours separated only by the 16-float
        alignment padding (zeros in every flat buffer) are merged"""
        rng = []
        for name, off, k, _, _ in self.m._layout:
            if name in self._gemm_params:
                continue
            if rng and off - (rng[-1][0] + rng[-1][1]) < 16:
                rng[-1] = (rng[-1][0], off + k - rng[-1][0])
            else:
                rng.append((off, k))
        return rng

    def adamw_step(self, opt, decay_mul, omb1, beta2, omb2, step_size, bc2_sqrt, eps, gscale):
        """AdamW over the flat buffers fused with the GEMM weight images (fs2_adamw_prep): the
        next forward's prepare_weights finds them current and skips its own pass."""
        m = self.m
        if self._wtable is None:
            self.prepare_weights(force=True)      # builds the descriptor table
        if getattr(self, "_rtable", None) is None:
            self._rtable = ops.adamw_ranges_table(self._adam_ranges(), self.dev)
        ops.adamw_prep(self._wtable, self._rtable, m._flat, m._gflat, opt.exp_avg, opt.exp_avg_sq,
                       decay_mul, omb1, beta2, omb2, step_size, bc2_sqrt, eps, gscale, dt=self.dt)
        m.mark_params_updated()
        self._prepared_version = (m._param_version, m._flat._version)

    @staticmethod
    def _adam_late(name):
        """parameters whose gradients are complete once the backward has passed the decoder and
        the variance adaptor (model.py:430-441 run first in the backward)"""
        return name.startswith(("decoder.", "linear.", "postnet."))

    def _adam_range_list(self, late):
        """flat (start, length) ranges of the late / early non-GEMM parameters (_adam_ranges
        split by _adam_late; neighbours within the 16-float alignment padding merged)"""
        rng = []
        for name, off, k, _, _ in self.m._layout:
            if name in self._gemm_params or self._adam_late(name) != late:
                continue
            if rng and off - (rng[-1][0] + rng[-1][1]) < 16:
                rng[-1] = (rng[-1][0], off + k - rng[-1][0])
            else:
                rng.append((off, k))
        return rng

    def _adam_tables(self, late):
        """(weight table, range table) of fs2_adamw_prep over the late / early parameters"""
        ents = [e for n, e in self._wentries.items() if self._adam_late(n) == late]
        wt = ops.weight_prep_table(ents) if ents else (None, 0, 0)
        return wt, ops.adamw_ranges_table(self._adam_range_list(late), self.dev)

    def late_param_end(self):
        """end of the late parameters in the flat buffer (they lead it: backward order)"""
        return max(off + k for name, off, k, _, _ in self.m._layout if self._adam_late(name))

    def _adam_launch_late(self, wait=None):
        """the late parameters' AdamW on the aux stream, after everything queued on the main and
        the weight-gradient streams (their gradients) and, under DP, after ``wait(aux)`` (the
        all-reduce of their buckets); the main stream does not wait here"""
        opt, scal = self.adam_split
        m = self.m
        if self._wtable is None:
            self.prepare_weights(force=True)
        if self._adam_tabs is None:
            self._adam_tabs = [self._adam_tables(late) for late in (False, True)]
        wl, rl = self._adam_tabs[1]
        h = self._aux_fork()
        self._aux.wait_stream(self._side)
        if wait is not None:
            wait(self._aux)
        ops.adamw_prep(wl, rl, m._flat, m._gflat, opt.exp_avg, opt.exp_avg_sq, *scal, dt=self.dt)
        self._aux_exit(h)
        self._adam_late_done = True
        self.n_adam_late += 1

    def adamw_step_split(self, opt, scal):
        """the rest of a step's AdamW (FusedTrainer.step): the early parameters on the main
        stream after it has joined the aux stream's late update; the whole update if the
        backward did not launch the late part"""
        m = self.m
        if not self._adam_late_done:
            self.adamw_step(opt, *scal)
            return
        self._adam_late_done = False
        we, re_ = self._adam_tabs[0]
        torch.cuda.current_stream(self.dev).wait_stream(self._aux)
        ops.adamw_prep(we, re_, m._flat, m._gflat, opt.exp_avg, opt.exp_avg_sq, *scal, dt=self.dt)
        m.mark_params_updated()
        self._prepared_version = (m._param_version, m._flat._version)

    def _dtag(self, kind, wname, T):
        """per-call-site tag for the detailed timer (FS2 layer indices folded)"""
        if self.timer is None or not getattr(self.timer, "detail", False):
            return None
        return f"{kind}:{re.sub(r'layers[.][0-9]+', 'layers.*', wname)}:T{T}"

    def _fwd(self, X, ldx, M, T, wname, out, ldo, **epi):
        O, C, KW = self._wspecs[wname]
        Wf, _ = self.w[wname]
        K = Wf.shape[1]
        conv = (1, T, KW, C) if KW > 1 else None
        tag = self._dtag("fwd", wname, T)
        if tag:
            self._tic(tag)
        ti = self._tap_inner_fwd(wname)
        if isinstance(X, tuple):
            # reflect-padded X image (_pad_fwd): the conv over the padded domain is a plain
            # K-major GEMM with overlapping rows, A(m, k=(j,c)) = image[m*C + k] (in the
            # tap-inner order with a Wf built that way, fs2_gemm_desc.a_kw); the pad rows'
            # results are dropped by the epilogue (c_row = (T, -2P))
            P = (KW - 1) // 2
            Mp = (M // T) * (T + 2 * P)
            ops.gemm(Mp, O, K, X[0], C, Wf, K, out, ldo, dt=self.dt, c_row=(T, -2 * P),
                     a_kw=KW if ti else 0, **epi)
        else:
            if ti:
                raise ValueError(f"{wname}: its forward image is in the tap-inner order of the "
                                 "padded-image path, which this batch cannot take")
            ops.gemm(M, O, K, X, ldx, Wf, K, out, ldo, dt=self.dt, conv=conv, **epi)
        if tag:
            self._toc(tag)

    def _pad_fwd(self, wname, M, T):
        """FFN conv1 forward over a reflect-padded token-major X image (fs2_pad_rows + a plain
        GEMM whose A rows overlap, 2P dropped rows per utterance): tools/fwd_probe.py, B = 32:
        decoder 374 -> 305 us, encoder 100 -> 89 standalone (the implicit conv's per-K-tile
        reflect rows and tap offsets are gone from the loader)"""
        O, C, KW = self._wspecs[wname]
        # both stacks: over the image the decoder's conv1 is a plain GEMM for the 4-wave kernel
        # (gemm_w4b_kernel), step 17.54 -> 17.35 ms on one box (tools/step_ab.sh, 3 rounds);
        # on the 8-wave implicit conv it had measured no faster.  FS2_PAD_FWD=1 (experiments
        # build): encoder only.
        if _PAD_FWD == 1 and not wname.startswith("encoder."):
            return False
        P = (KW - 1) // 2
        if self._tap_inner_fwd(wname):   # the 4-wave kernel: 32-bit offsets to 2.8 M rows
            return P < T
        return (self.dt == 1 and _PAD_FWD and KW > 1 and C % 64 == 0 and P < T and
                self.w[wname][0].shape[1] == KW * C and
                ps_plain_ok((M // T) * (T + 2 * P), C, O, KW * C, M, O, 2))

    def _dgrad(self, dY, lddy, M, T, wname, out, ldo, n_out=None, **epi):
        tag = self._dtag("dgrad", wname, T)
        if tag:
            self._tic(tag)
        self._dgrad_impl(dY, lddy, M, T, wname, out, ldo, n_out, **epi)
        if tag:
            self._toc(tag)

    def _pad_dgrad(self, wname):
        """FFN conv1 data gradients over a zero-padded token-major dY image (bf16): the
        producing conv2 data gradient writes dY into the image (fs2_gemm c_row_t), and with the
        weight image's taps reversed the shift conv is a plain K-major GEMM whose A rows
        overlap, A(m, k) = image[m * O + k] (tools/dgrad_probe.py, B = 32: decoder 417 -> 339
        us, encoder 83 -> 76) -- no per-K-tile tap offsets or row bounds in the loader."""
        if self.dt != 1 or not _PAD_DGRAD or ".pos_ffn.0." not in wname:
            return False
        if _PAD_DGRAD == 2 and not wname.startswith("decoder."):
            return False     # A/B: decoder only
        O, C, KW = self._wspecs[wname]
        return KW > 1 and self._km_ok(O, C, KW, KW, None)

    def _tap_inner(self, wname):
        """the decoder FFN conv1 data gradient over the padded dY image in the tap-inner K order
        (fs2_gemm_desc.a_kw, Wb built with w_okc bit 2): consecutive 64-deep K-stages read image
        rows one tap apart, so the 96 MB image is fetched from HBM about once instead of once
        per tap (995 MB per launch in the natural order, profiles/r05e_dgrad_traffic.json).
        Always the 4-wave kernel, unsplit; the encoder's (M = 6656) keeps its split-K path."""
        if not (_TAP_INNER and self._pad_dgrad(wname) and wname.startswith("decoder.")):
            return False
        O, C, KW = self._wspecs[wname]
        return O % 64 == 0 and (KW * O) % 128 == 0

    def _tap_inner_fwd(self, wname):
        """the FFN conv1 forward over the reflect-padded X image in the tap-inner K order (Wf
        built with w_okc bit 3), both stacks: the image's rows are fetched about once instead of
        once per tap.  Needs the padded path on every batch (_pad_fwd's conditions other than
        P < T, which the reference's reflect padding requires anyway)."""
        if not (_TAP_INNER_FWD and self.dt == 1 and _PAD_FWD and ".pos_ffn.0." in wname):
            return False
        if _PAD_FWD == 1 and not wname.startswith("encoder."):
            return False
        O, C, KW = self._wspecs[wname]
        return KW > 1 and C % 64 == 0 and (KW * C) % 128 == 0 and \
            self.w[wname][0].shape[1] == KW * C

    def _pad_dgrad_fits(self, wname, B, T):
        """the padded data gradient's GEMM within the persistent kernel's 32-bit offsets"""
        O, C, KW = self._wspecs[wname]
        P = (KW - 1) // 2
        Mp = B * (T + 2 * P)
        # the image (Mp + 2P rows of O), the weight image, the fp32 padded-domain output, and
        # conv2's data gradient written into the image (c_row = (T, 2P))
        return (ps_plain_ok(Mp + 2 * P, O, C, KW * O, Mp, C, 4) and
                ps_plain_ok(B * T, O, O, O, Mp + 2 * P, O, 2))

    def _dy_image(self, key, B, T, P, F):
        """zero-padded token-major image for a k = 2P+1 conv data gradient: 2P zero rows, then
        per utterance T data rows and 2P zero rows (the last P are the end guard); returns
        (image from its first row, data view from the first utterance's row 0).  Token (b, t)
        sits at data row b*T + t remapped to b*(T+2P) + t (fs2_gemm c_row = (T, 2P)).

        Eager steps keep one buffer per layer (``key``) across steps: only its data rows are
        ever written, so its pad rows -- zeroed through a view starting T rows before the image
        -- need zeroing only when the batch shape changes (stream order keeps the reuse safe:
        the next step's main-stream work follows this step's side-stream join).  A step being
        captured into a HIP graph gets its own image from the graph's memory pool with the
        pad-row zeroing captured too, so replays of graphs of other shapes (FusedTrainer keeps
        several) never share or re-lay-out a buffer another graph writes."""
        L = T + 2 * P
        n = (B + 1) * L * F
        shape = (B, T, P, F)
        if torch.cuda.is_current_stream_capturing():
            buf = torch.empty(n, dtype=self.adt, device=self.dev)
            buf.view(B + 1, L, F)[:, T:].zero_()
        else:
            ent = self._img.get(key)
            if ent is None or ent[0] != shape:
                buf = ent[1] if ent is not None and ent[1].numel() >= n else \
                    torch.empty(n, dtype=self.adt, device=self.dev)
                buf[:n].view(B + 1, L, F)[:, T:].zero_()
                ent = self._img[key] = (shape, buf)
            buf = ent[1]
        img = buf[:n].view((B + 1) * L, F)[T:]
        return img, img[2 * P:]

    def _dgrad_impl(self, dY, lddy, M, T, wname, out, ldo, n_out=None, **epi):
        O, C, KW = self._wspecs[wname]
        _, Wb = self.w[wname]
        if KW == 1:
            ops.gemm(M, n_out or C, O, dY, lddy, Wb, O, out, ldo, dt=self.dt, **epi)
            return
        # reflect "same" conv data gradient = zero-padded shift conv over the padded domain
        # (T+2P rows per utterance, fp32) + the reflect fold, which also applies the epilogue
        P = (KW - 1) // 2
        B = M // T
        Mp = B * (T + 2 * P)
        ti = isinstance(dY, tuple) and self._tap_inner(wname)
        split = 1 if ti else dgrad_split(Mp, C, KW * O, self.dt)
        Xpad = torch.empty(split, Mp, C, dtype=torch.float32, device=self.dev)
        if isinstance(dY, tuple):
            # padded dY image (_dy_image): row m of the padded domain reads image rows
            # m .. m + 2P, i.e. A(m, k) = image[m * O + k] against the tap-reversed Wb (in the
            # tap-inner order: k = (64-channel chunk, tap, channel), fs2_gemm_desc.a_kw)
            img = dY[0]
            ops.gemm(Mp, C, KW * O, img, O, Wb, KW * O, Xpad, C, dt=self.dt, c_fp32=1,
                     split_k=split, split_stride=Mp * C if split > 1 else 0,
                     a_kw=KW if ti else 0)
        else:
            ops.gemm(Mp, C, KW * O, dY, lddy, Wb, KW * O, Xpad, C, dt=self.dt, conv=(4, T, KW, O),
                     c_fp32=1, split_k=split, split_stride=Mp * C if split > 1 else 0)
        assert set(epi) <= {"residual", "ldr", "row_scale", "row_scale_post"}, epi
        ops.conv_fold(Xpad, B, T, P, C, out, ldo, dt=self.dt, residual=epi.get("residual"),
                      ldr=epi.get("ldr", 0), row_scale=epi.get("row_scale"),
                      row_scale_post=epi.get("row_scale_post"), nsplit=split,
                      split_stride=Mp * C)

    def _wgrad(self, dY, lddy, X, ldx, M, T, wname, n_cols=None, gemm_tag=None, bias=None,
               dy_img=None):
        """weight gradient on the side stream; ``bias``: also the bias gradient (column sums of
        dY) -- fused into the K-major path's dY transpose, else an fs2_colsum pass; ``dy_img``:
        dY lives in a zero-padded image (_dy_image), read from there"""
        h = self._side_enter(dY, X, dy_img)
        tag = self._dtag("wgrad", wname, T)
        if tag:
            self._tic(tag)
        ctas = self._side_ctas if h is not None else 0
        done = self._wgrad_impl(dY, lddy, X, ldx, M, T, wname, n_cols, gemm_tag, bias, dy_img,
                                ctas)
        if tag:
            self._toc(tag)
        if bias is not None and not done:
            O = self._wspecs[wname][0]
            ops.colsum(dY, lddy, M, O, self.grads[bias], dt=self.dt, ws=self.ws(ops.colsum_ws(M, O)))
        self._side_exit(h)

    def _km_ok(self, O, C, KW, T, n_cols):
        """conv weight gradients that take the K-major path (conv_mode 6): the FFN conv1
        (k = 9) and PostNet (k = 5) weights.  tools/km_wgrad_bench.py, B = 32, GEMM + slice sum
        + both transposes vs the MN-major implicit-conv GEMM: decoder conv1 464 -> 372 us,
        encoder conv1 115 -> 110, PostNet 218 / 237 / 221 -> 125 / 98 / 75; the k = 3
        predictor convs lose (58 -> 67: the transposes cost more than the GEMM saves)."""
        return (self.dt == 1 and _KM_WGRAD and KW >= 5 and n_cols is None and
                C % 8 == 0 and O % 8 == 0 and (KW - 1) // 2 < T)

    def _km_image(self, key, C, ld):
        """bf16 [C][ld] image with a zeroed guard of 64 elements before row 0 and after the
        last row (the tap-shifted reads of conv_mode 6 reach P elements past either end).
        One buffer per (key, C), grown to the largest C*ld seen and re-guarded when ld changes
        (ld follows the batch's T, so a per-ld cache would grow without bound over an epoch);
        it lives on the side stream, whose layers use it one after another.  A captured step
        gets its own zeroed image from the graph's pool (see _dy_image)."""
        n = C * ld
        if torch.cuda.is_current_stream_capturing():
            return torch.zeros(n + 128, dtype=torch.bfloat16, device=self.dev)[64:64 + n]
        k = (key, C)
        ent = self._km.get(k)
        if ent is None or ent[1].numel() < n + 128:
            buf = torch.zeros(n + 128, dtype=torch.bfloat16, device=self.dev)
            self._km[k] = (ld, buf)
        elif ent[0] != ld:
            buf = ent[1]
            buf[64 + n:64 + n + 64].zero_()   # the end guard of the new layout
            self._km[k] = (ld, buf)
        else:
            buf = ent[1]
        return buf[64:64 + n]

    def _wgrad_km(self, dY, lddy, X, ldx, M, T, wname, gemm_tag=None, bias=None, dy_img=None,
                  ctas=0):
        """grad[O][KW][C] += sum_{b,t} dY[b,t,o] X[b, reflect(t+j-P), c] with both GEMM operands
        K-major: dY and X are first written channel-major over the padded token domain (T+2P
        columns per utterance; dY's pad columns zero, X's reflected), where tap j is a constant
        column shift j - P of X's image (fs2_pad_transpose + conv_mode 6).  Same sum as
        _wgrad_impl's implicit-conv GEMM (SB Conv1d weight gradient, model.py:241-267)."""
        O, C, KW = self._wspecs[wname]
        P = (KW - 1) // 2
        B = M // T
        Bt = B * (T + 2 * P)
        ncol = KW * C
        tiles = -(-O // 256) * -(-ncol // 256)
        # one (split, tile) unit per CU; >= 16 K-tiles per unit, <= 25 fp32 slices to sum
        cus = ctas if 0 < ctas < 256 else 256
        S = max(1, min(cus // tiles, -(-Bt // 64) // 16, 25))
        Kp = round_up(Bt, 64 * S)
        dYT = self._km_image("dy", O, Kp)
        XT = self._km_image("x", C, Kp)
        ws = self.ws(max(ops.pad_transpose_ws(Kp, O), 1))
        colsum = self.grads[bias] if bias is not None else None
        if dy_img is not None:
            # the padded dY image already holds the zero pad rows: a plain transpose of its
            # utterance rows (from image row P: T + 2P rows per utterance)
            ops.pad_transpose(dy_img[P:], lddy, B, T + 2 * P, O, 0, 0, dYT, Kp, Kp,
                              dt=self.dt, colsum=colsum, ws=ws)
        else:
            ops.pad_transpose(dY, lddy, B, T, O, P, 0, dYT, Kp, Kp, dt=self.dt, colsum=colsum,
                              ws=ws)
        ops.pad_transpose(X, ldx, B, T, C, P, 1, XT, Kp, Kp, dt=self.dt)
        stride = O * ncol
        ws = self.ws(S * stride)
        if gemm_tag:
            self._tic(gemm_tag)
        ops.gemm(O, ncol, Kp, dYT, Kp, XT, Kp, ws, ncol, dt=self.dt, conv=(6, T, KW, C),
                 c_fp32=1, split_k=S, split_stride=stride if S > 1 else 0, max_ctas=ctas)
        if gemm_tag:
            self._toc(gemm_tag)
        ops.sum_slices(ws, S, stride, stride, self.grads[wname], accumulate=1)
        return True

    def _wgrad_impl(self, dY, lddy, X, ldx, M, T, wname, n_cols=None, gemm_tag=None, bias=None,
                    dy_img=None, ctas=0):
        """grad[O][KW][C] += sum_m dY[m][o] * X[reflect(t+j-P)][c]   (fp32, accumulate).
        ``gemm_tag``: HIP events around the GEMM launch alone (bench.py's roofline entry for
        the FFN conv1 weight gradient), on the stream it runs on (the side stream)."""
        O, C, KW = self._wspecs[wname]
        if self._km_ok(O, C, KW, T, n_cols) and lddy % 8 == 0 and ldx % 8 == 0:
            return self._wgrad_km(dY, lddy, X, ldx, M, T, wname, gemm_tag, bias, dy_img, ctas)
        if dy_img is not None:
            raise RuntimeError(f"{wname}: a padded dY image needs the K-major weight gradient")
        if n_cols is not None and n_cols != KW * C and KW == 1 and n_cols % 8 == 0 and self.dt == 1:
            # padded X columns (concat_proj: 2D + 5 -> 776): split-K slices over the padded width,
            # then the valid columns added into the gradient -- the unpadded GEMM's odd row
            # pitch forced the scalar atomic epilogue (92 -> ~35 us, tools/wgrad1x1_bench.py)
            K = round_up(M, self.epc)
            ns = eff_split(K, wgrad_slices(O, n_cols, n_cols, K, self.dt), _BK[self.dt])
            ns = max(ns, 2)
            stride = O * n_cols
            ws = self.ws((ns + 1) * stride)
            ops.gemm(O, n_cols, K, dY, lddy, X, ldx, ws, n_cols, dt=self.dt, a_kmajor=0,
                     b_kmajor=0, c_fp32=1, kvalid=M, nvalid=n_cols, split_k=ns,
                     split_stride=stride, max_ctas=ctas)
            tot = ws[ns * stride:(ns + 1) * stride]
            ops.sum_slices(ws, ns, stride, stride, tot, accumulate=0)
            self.grads[wname].view(O, C).add_(tot.view(O, n_cols)[:, :C])
            return
        Ncols = n_cols or KW * C
        K = round_up(M, self.epc)
        tiles = -(-O // 128) * -(-Ncols // 128)
        split = 1
        if tiles < 256:
            split = max(1, min(-(-_WG_ATOMIC_UNITS // tiles), K // (_BK[self.dt] * 4)))
        conv = (3, T, KW, C) if KW > 1 else None
        ldc = C * KW
        ns = wgrad_slices(O, Ncols, ldc, K, self.dt, _WG_SLICE_CU) if not _NO_SLICES else 1
        if ns == 1 and _BIG_SLICES and self.dt == 1 and Ncols == ldc and O * ldc > 600_000:
            tiles = -(-O // 256) * -(-Ncols // 256)
            ns = max(1, min(-(-_SLICE_TARGET // tiles), (K // 64) // 8))
        ns = eff_split(K, ns, _BK[self.dt])
        if ns > 1:
            # small outputs: split-K slices into fp32 planes, summed in a fixed order -- instead
            # of tens of fp32 atomics landing on every output element
            stride = O * ldc
            ws = self.ws(ns * stride)
            if gemm_tag:
                self._tic(gemm_tag)
            ops.gemm(O, Ncols, K, dY, lddy, X, ldx, ws, ldc, dt=self.dt, a_kmajor=0, b_kmajor=0,
                     conv=conv, c_fp32=1, kvalid=M, nvalid=ldc, split_k=ns, split_stride=stride,
                     max_ctas=ctas)
            if gemm_tag:
                self._toc(gemm_tag)
            ops.sum_slices(ws, ns, stride, stride, self.grads[wname], accumulate=1)
            return
        # conv weight gradients land contiguous in the [O][KW][C] flat layout (model._kw_major)
        ops.gemm(O, Ncols, K, dY, lddy, X, ldx, self.grads[wname], ldc, dt=self.dt, a_kmajor=0,
                 b_kmajor=0, conv=conv, c_fp32=1, kvalid=M, nvalid=KW * C, accumulate=1,
                 split_k=split, max_ctas=ctas)

    def _bias_grad(self, dY, lddy, M, n, gname):
        h = self._side_enter(dY)
        ops.colsum(dY, lddy, M, n, self.grads[gname], dt=self.dt, ws=self.ws(ops.colsum_ws(M, n)))
        self._side_exit(h)

    # ------------------------------------------------------------------ FFT block
    def _fft_fwd(self, X, B, T, key_pad, prefix, H, p_drop, seed, salt):
        D = self.cfg.enc_d_model
        dh = D // H
        M = B * T
        P = self.params
        ctx = {"X": X}
        QKV = self.empty(M, 3 * D)
        self._fwd(X, D, M, T, prefix + "self_att.att.in_proj_weight", QKV, 3 * D,
                  bias=P[prefix + "self_att.att.in_proj_bias"])
        ldt = round_up(T, 8)
        Att = self.empty(M, D)
        if self.use_flash(T, dh):
            # fused attention: no (B*H, T, T) tensors; lse kept for the backward
            lse = torch.empty(B * H, T, dtype=torch.float32, device=self.dev)
            s_att = salt()
            tag = self._dtag("attn_fwd", "", T)
            if tag:
                self._tic(tag)
            ops.attn_fwd(QKV, 3 * D, key_pad, B, H, T, dh, 1.0 / math.sqrt(dh), p_drop, seed,
                         s_att, Att, D, lse, dt=self.dt)
            if tag:
                self._toc(tag)
            Pm = Pd = None
            ctx.update(lse=lse, key_pad=key_pad)
        else:
            S = torch.empty(B * H, T, ldt, dtype=torch.float32, device=self.dev)
            ops.gemm(T, T, dh, QKV, 3 * D, QKV[:, D:], 3 * D, S, ldt, dt=self.dt, c_fp32=1,
                     batch=B * H, batch_div=H,
                     strides=(T * 3 * D, dh, T * 3 * D, dh, H * T * ldt, T * ldt, 0, 0))
            Pm = self.empty(B * H, T, ldt)
            Pd = self.empty(B * H, T, ldt) if p_drop > 0 else Pm
            s_att = salt()
            ops.softmax_fwd(S, key_pad, B, H, T, T, ldt, 1.0 / math.sqrt(dh), p_drop, seed, s_att,
                            Pm, Pd if p_drop > 0 else None, dt=self.dt)
            del S
            ops.gemm(T, dh, ldt, Pd, ldt, QKV[:, 2 * D:], 3 * D, Att, D, dt=self.dt, b_kmajor=0,
                     kvalid=T, batch=B * H, batch_div=H,
                     strides=(H * T * ldt, T * ldt, T * 3 * D, dh, T * D, dh, 0, 0))
        Ao = self.empty(M, D)
        self._fwd(Att, D, M, T, prefix + "self_att.att.out_proj.weight", Ao, D,
                  bias=P[prefix + "self_att.att.out_proj.bias"])
        X1, s1 = self.empty(M, D), self.empty(M, D)
        mean1 = torch.empty(M, dtype=torch.float32, device=self.dev)
        rstd1 = torch.empty_like(mean1)
        s_r1 = salt()
        w1 = prefix + "pos_ffn.0.conv.weight"
        F, _, KW1 = self._wspecs[w1]
        P1 = (KW1 - 1) // 2
        # the FFN conv1 forward's reflect-padded X1 image, written by the LayerNorm that makes
        # X1 (fs2_ln_fwd img).  Its 2P tail rows are read only by the dropped pad-row outputs of
        # the last utterance (c_row = (T, -2P); each output row sums its own 2P+1 image rows):
        # one image per shape, reused layer after layer, its tail zeroed once at allocation
        img = self._fwd_image(B * (T + 2 * P1), 2 * P1, D) if self._pad_fwd(w1, M, T) else None
        ops.ln_fwd(X, D, P[prefix + "norm1.norm.weight"], P[prefix + "norm1.norm.bias"], 1e-6, X1, D,
                   mean1, rstd1, M, D, dt=self.dt, seed=seed, r=Ao, ldr=D, p_r=p_drop, salt_r=s_r1,
                   s_out=s1, img=img if _LN_IMG else None, img_t=T, img_p=P1)
        if img is not None and not _LN_IMG:
            ops.pad_rows(X1, D, B, T, D, P1, 1, 2 * P1, img, D, dt=self.dt)
        del Ao
        Hc = self.empty(M, F)
        X1in = X1 if img is None else (img,)
        tag = "ffn_conv1_fwd." + prefix.split(".")[0]
        self._tic(tag)
        self._fwd(X1in, D, M, T, w1, Hc, F, bias=P[prefix + "pos_ffn.0.conv.bias"], relu=1)
        self._toc(tag)
        del X1in, img
        Y = self.empty(M, D)
        self._fwd(Hc, F, M, T, prefix + "pos_ffn.2.conv.weight", Y, D,
                  bias=P[prefix + "pos_ffn.2.conv.bias"])
        X2, s2 = self.empty(M, D), self.empty(M, D)
        mean2 = torch.empty(M, dtype=torch.float32, device=self.dev)
        rstd2 = torch.empty_like(mean2)
        s_r2 = salt()
        ops.ln_fwd(X1, D, P[prefix + "norm2.norm.weight"], P[prefix + "norm2.norm.bias"], 1e-6, X2, D,
                   mean2, rstd2, M, D, dt=self.dt, seed=seed, r=Y, ldr=D, p_r=p_drop, salt_r=s_r2,
                   s_out=s2)
        ctx.update(QKV=QKV, Pm=Pm, Pd=Pd, Att=Att, X1=X1, s1=s1, mean1=mean1, rstd1=rstd1, Hc=Hc,
                   s2=s2, mean2=mean2, rstd2=rstd2, s_att=s_att, s_r1=s_r1, s_r2=s_r2, F=F,
                   ldt=ldt)
        return X2, ctx

    def _fft_bwd(self, dX2, ctx, B, T, prefix, H, p_drop, seed):
        D = self.cfg.enc_d_model
        dh = D // H
        M = B * T
        F, ldt = ctx["F"], ctx["ldt"]
        P, G = self.params, self.grads
        lnws = self.ws(ops.ln_ws(M, D))
        ds2, dY = self.empty(M, D), self.empty(M, D)
        ops.ln_bwd(dX2, D, ctx["s2"], D, ctx["mean2"], ctx["rstd2"], P[prefix + "norm2.norm.weight"],
                   P[prefix + "norm2.norm.bias"], ds2, D, M, D, dt=self.dt, ws=lnws, seed=seed,
                   dr=dY, p_r=p_drop, salt_r=ctx["s_r2"], dgamma=G[prefix + "norm2.norm.weight"],
                   dbeta=G[prefix + "norm2.norm.bias"], dcol=G[prefix + "pos_ffn.2.conv.bias"])
        w2 = prefix + "pos_ffn.2.conv.weight"
        w1 = prefix + "pos_ffn.0.conv.weight"
        pad = self._pad_dgrad(w1)
        if pad and not self._pad_dgrad_fits(w1, B, T):
            # the weight images of this conv were built tap-reversed for the padded path
            raise ValueError(f"{w1}: batch of {B} x {T} tokens exceeds the 32-bit offsets of the "
                             "padded conv data gradient; split the batch")
        if pad:   # conv2's data gradient lands in the zero-padded image conv1's reads
            P1 = (self._wspecs[w1][2] - 1) // 2
            img, dHc = self._dy_image(prefix, B, T, P1, F)
            crow = {"c_row": (T, 2 * P1)}
        else:
            img, crow = None, {}
            dHc = self.empty(M, F)
        dX1 = self.empty(M, D)
        # weight gradients enqueued as soon as their operands exist (the side stream waits for
        # everything queued on main so far): conv2's before its data gradient, conv1's right
        # after dHc, so the two big conv1 GEMMs overlap instead of the conv1 weight gradient
        # holding every CU while main's out-projection waits behind it
        self._wgrad(dY, D, ctx["Hc"], F, M, T, w2)
        self._dgrad(dY, D, M, T, w2, dHc, F, gate=ctx["Hc"], ldg=F, **crow)
        self._wgrad(dHc, F, ctx["X1"], D, M, T, w1,
                    gemm_tag="ffn_conv1_wgrad." + prefix.split(".")[0],
                    bias=prefix + "pos_ffn.0.conv.bias", dy_img=img)
        self._dgrad((img,) if pad else dHc, F, M, T, w1, dX1, D, residual=ds2, ldr=D)
        del dY, dHc, ds2, img
        lnws = self.ws(ops.ln_ws(M, D))
        ds1, dAo = self.empty(M, D), self.empty(M, D)
        ops.ln_bwd(dX1, D, ctx["s1"], D, ctx["mean1"], ctx["rstd1"], P[prefix + "norm1.norm.weight"],
                   P[prefix + "norm1.norm.bias"], ds1, D, M, D, dt=self.dt, ws=lnws, seed=seed,
                   dr=dAo, p_r=p_drop, salt_r=ctx["s_r1"], dgamma=G[prefix + "norm1.norm.weight"],
                   dbeta=G[prefix + "norm1.norm.bias"],
                   dcol=G[prefix + "self_att.att.out_proj.bias"])
        del dX1
        wo = prefix + "self_att.att.out_proj.weight"
        dAtt = self.empty(M, D)
        self._wgrad(dAo, D, ctx["Att"], D, M, T, wo)
        self._dgrad(dAo, D, M, T, wo, dAtt, D)
        del dAo
        QKV, Pm, Pd = ctx["QKV"], ctx["Pm"], ctx["Pd"]
        if "lse" in ctx:     # fused attention backward (dQ, dK, dV in one pass each)
            dQKV = self.empty(M, 3 * D)
            tag = self._dtag("attn_bwd", "", T)
            if tag:
                self._tic(tag)
            args = (QKV, 3 * D, ctx["key_pad"], ctx["Att"], D, dAtt, D, ctx["lse"], B, H, T, dh,
                    1.0 / math.sqrt(dh), p_drop, seed, ctx["s_att"], dQKV, 3 * D)
            ws = self.ws(ops.attn_ws(B, H, T))
            ops.attn_bwd(*args, dt=self.dt, ws=ws)
            if tag:
                self._toc(tag)
            return self._qkv_bwd(dQKV, ctx, M, T, D, prefix, ds1)
        # ---- attention backward over the materialised probabilities
        dPd = torch.empty(B * H, T, ldt, dtype=torch.float32, device=self.dev)
        ops.gemm(T, T, dh, dAtt, D, QKV[:, 2 * D:], 3 * D, dPd, ldt, dt=self.dt, c_fp32=1,
                 batch=B * H, batch_div=H,
                 strides=(T * D, dh, T * 3 * D, dh, H * T * ldt, T * ldt, 0, 0))
        dQKV = self.empty(M, 3 * D)
        # dV = Pd^T dO
        ops.gemm(ldt, dh, ldt, Pd, ldt, dAtt, D, dQKV[:, 2 * D:], 3 * D, dt=self.dt, a_kmajor=0,
                 b_kmajor=0, kvalid=T, mvalid=T, batch=B * H, batch_div=H,
                 strides=(H * T * ldt, T * ldt, T * D, dh, T * 3 * D, dh, 0, 0))
        dS = self.empty(B * H, T, ldt)
        ops.softmax_bwd(dPd, Pm, B, H, T, T, ldt, 1.0 / math.sqrt(dh), p_drop, seed, ctx["s_att"], dS,
                        dt=self.dt)
        del dPd
        # dQ = dS K
        ops.gemm(T, dh, ldt, dS, ldt, QKV[:, D:], 3 * D, dQKV, 3 * D, dt=self.dt, b_kmajor=0,
                 kvalid=T, batch=B * H, batch_div=H,
                 strides=(H * T * ldt, T * ldt, T * 3 * D, dh, T * 3 * D, dh, 0, 0))
        # dK = dS^T Q
        ops.gemm(ldt, dh, ldt, dS, ldt, QKV, 3 * D, dQKV[:, D:], 3 * D, dt=self.dt, a_kmajor=0,
                 b_kmajor=0, kvalid=T, mvalid=T, batch=B * H, batch_div=H,
                 strides=(H * T * ldt, T * ldt, T * 3 * D, dh, T * 3 * D, dh, 0, 0))
        del dS
        return self._qkv_bwd(dQKV, ctx, M, T, D, prefix, ds1)

    def _qkv_bwd(self, dQKV, ctx, M, T, D, prefix, ds1):
        wi = prefix + "self_att.att.in_proj_weight"
        dX = self.empty(M, D)
        self._wgrad(dQKV, 3 * D, ctx["X"], D, M, T, wi)
        self._bias_grad(dQKV, 3 * D, M, 3 * D, prefix + "self_att.att.in_proj_bias")
        self._dgrad(dQKV, 3 * D, M, T, wi, dX, D, residual=ds1, ldr=D)
        return dX

    # ------------------------------------------------------------------ variance predictor
    def _pred_fwd(self, Zin, keep, B, T, name, rate, p_drop, seed, salt, a1=None, lda1=None,
                  salts=None):
        """one variance predictor (model.py:208-240).  ``a1`` / ``lda1``: its conv1 output
        already computed (the fused duration / pitch conv1, a column slice of row pitch lda1);
        ``salts``: its two dropout salts, drawn in advance"""
        D = self.cfg.enc_d_model
        M = B * T
        P = self.params
        c = {"Zin": Zin}
        if a1 is None:
            a1, lda1 = self.empty(M, D), D
            self._fwd(Zin, D, M, T, name + ".conv1.conv.weight", a1, D,
                      bias=P[name + ".conv1.conv.bias"], relu=1)
        v1 = self.empty(M, D)
        m1 = torch.empty(M, dtype=torch.float32, device=self.dev)
        r1 = torch.empty_like(m1)
        s1 = salts[0] if salts else salt()
        ops.ln_fwd(a1, lda1, P[name + ".ln1.norm.weight"], P[name + ".ln1.norm.bias"], 1e-5, v1, D, m1,
                   r1, M, D, dt=self.dt, seed=seed, p_o=p_drop, salt_o=s1, row_mask=keep)
        a2 = self.empty(M, D)
        self._fwd(v1, D, M, T, name + ".conv2.conv.weight", a2, D,
                  bias=P[name + ".conv2.conv.bias"], relu=1)
        v2 = self.empty(M, D)
        m2 = torch.empty(M, dtype=torch.float32, device=self.dev)
        r2 = torch.empty_like(m2)
        s2 = salts[1] if salts else salt()
        ops.ln_fwd(a2, D, P[name + ".ln2.norm.weight"], P[name + ".ln2.norm.bias"], 1e-5, v2, D, m2, r2,
                   M, D, dt=self.dt, seed=seed, p_o=p_drop, salt_o=s2, row_mask=keep)
        y = self.empty(B, T)
        ops.rowdot_fwd(v2, D, P[name + ".linear.w.weight"], P[name + ".linear.w.bias"], float(rate),
                       M, D, y, dt=self.dt)
        c.update(a1=a1, lda1=lda1, v1=v1, m1=m1, r1=r1, a2=a2, v2=v2, m2=m2, r2=r2, s1=s1, s2=s2,
                 rate=float(rate))
        return y, c

    def _pred_pair_fwd(self, Zin, keep, B, T, pitch_rate, p_drop, seed, salt):
        """duration and pitch predictors (model.py:366-381), their conv1 as one conv with 768
        output channels over the shared input (columns 0..383 duration, 384..767 pitch); the
        dropout salts are drawn in the sequential order (duration's two, then pitch's)"""
        if self.PRED1 not in self._wspecs:
            pd, dctx = self._pred_fwd(Zin, keep, B, T, "durPred", 1.0, p_drop, seed, salt)
            pp, pctx = self._pred_fwd(Zin, keep, B, T, "pitchPred", pitch_rate, p_drop, seed, salt)
            return pd, dctx, pp, pctx
        D = self.cfg.enc_d_model
        M = B * T
        a1 = self.empty(M, 2 * D)
        self._fwd(Zin, D, M, T, self.PRED1, a1, 2 * D, bias=self.params[self.PRED1 + ".bias"],
                  relu=1)
        sd = (salt(), salt())
        sp = (salt(), salt())
        pd, dctx = self._pred_fwd(Zin, keep, B, T, "durPred", 1.0, p_drop, seed, salt,
                                  a1=a1[:, :D], lda1=2 * D, salts=sd)
        pp, pctx = self._pred_fwd(Zin, keep, B, T, "pitchPred", pitch_rate, p_drop, seed, salt,
                                  a1=a1[:, D:], lda1=2 * D, salts=sp)
        dctx["a1_pair"] = a1
        return pd, dctx, pp, pctx

    def _pred_pair_bwd(self, d_dur, dctx, d_pitch, pctx, keep, B, T, p_drop, seed, residual=None,
                       post_mask=False):
        """backward of _pred_pair_fwd: dZ = keep * (dZ_dur + dZ_pitch) [+ residual, * keep]; the
        fused conv1's data gradient sums both predictors' input gradients inside one GEMM"""
        if "a1_pair" not in dctx:
            dZa = self._pred_bwd(d_pitch, pctx, keep, B, T, "pitchPred", p_drop, seed,
                                 residual=residual)
            return self._pred_bwd(d_dur, dctx, keep, B, T, "durPred", p_drop, seed, residual=dZa,
                                  post_mask=post_mask)
        D = self.cfg.enc_d_model
        M = B * T
        da1 = self.empty(M, 2 * D)
        self._pred_bwd(d_pitch, pctx, keep, B, T, "pitchPred", p_drop, seed, da1=da1[:, D:])
        self._pred_bwd(d_dur, dctx, keep, B, T, "durPred", p_drop, seed, da1=da1[:, :D])
        dZ = self.empty(M, D)
        self._dgrad(da1, 2 * D, M, T, self.PRED1, dZ, D, row_scale=keep, residual=residual,
                    ldr=D if residual is not None else 0,
                    row_scale_post=keep if post_mask else None)
        self._wgrad(da1, 2 * D, dctx["Zin"], D, M, T, self.PRED1)
        return dZ

    def _pred_bwd(self, dy, c, keep, B, T, name, p_drop, seed, residual=None, post_mask=False,
                  da1=None):
        """returns dZin (masked by keep) [+ residual] for the predictor input; ``da1``: write the
        conv1 output gradient there (a column slice of the fused conv1's, row pitch 2 D) and
        stop -- the fused conv1's own backward follows (_pred_pair_bwd)"""
        D = self.cfg.enc_d_model
        M = B * T
        P, G = self.params, self.grads
        dv2 = self.empty(M, D)
        nb = min(256, max(1, (M + 31) // 32))
        ops.rowdot_bwd(dy, c["v2"], D, P[name + ".linear.w.weight"], c["rate"], M, D, dv2,
                       G[name + ".linear.w.weight"], G[name + ".linear.w.bias"], dt=self.dt,
                       ws=self.ws(nb * (D + 1)))
        da2 = self.empty(M, D)
        ops.ln_bwd(dv2, D, c["a2"], D, c["m2"], c["r2"], P[name + ".ln2.norm.weight"],
                   P[name + ".ln2.norm.bias"], da2, D, M, D, dt=self.dt, ws=self.ws(ops.ln_ws(M, D)),
                   seed=seed, p_o=p_drop, salt_o=c["s2"], row_mask=keep, relu_gate_in=1,
                   dgamma=G[name + ".ln2.norm.weight"], dbeta=G[name + ".ln2.norm.bias"],
                   dcol=G[name + ".conv2.conv.bias"])
        w2 = name + ".conv2.conv.weight"
        dv1 = self.empty(M, D)
        self._dgrad(da2, D, M, T, w2, dv1, D)
        self._wgrad(da2, D, c["v1"], D, M, T, w2)
        fused = da1 is not None
        if not fused:
            da1 = self.empty(M, D)
        ld1 = 2 * D if fused else D
        ops.ln_bwd(dv1, D, c["a1"], c["lda1"], c["m1"], c["r1"], P[name + ".ln1.norm.weight"],
                   P[name + ".ln1.norm.bias"], da1, ld1, M, D, dt=self.dt, ws=self.ws(ops.ln_ws(M, D)),
                   seed=seed, p_o=p_drop, salt_o=c["s1"], row_mask=keep, relu_gate_in=1,
                   dgamma=G[name + ".ln1.norm.weight"], dbeta=G[name + ".ln1.norm.bias"],
                   dcol=G[name + ".conv1.conv.bias"])
        if fused:
            return None
        w1 = name + ".conv1.conv.weight"
        dZ = self.empty(M, D)
        self._dgrad(da1, D, M, T, w1, dZ, D, row_scale=keep, residual=residual,
                    ldr=D if residual is not None else 0,
                    row_scale_post=keep if post_mask else None)
        self._wgrad(da1, D, c["Zin"], D, M, T, w1)
        return dZ

    # ------------------------------------------------------------------ PostNet
    def _postnet_fwd(self, mel, B, T, p_drop, seed, salt):
        c = self.cfg
        E, NM = c.postnet_embedding_dim, c.n_mels
        M = B * T
        P = self.params
        ctx = {"in": mel}
        x, ldx = mel, NM
        convs = ["postnet.conv_pre"] + [f"postnet.convs_intermedite.{i}"
                                        for i in range(c.postnet_n_convolutions - 2)]
        outs = []
        for i, name in enumerate(convs):
            p = self.empty(M, E)
            self._fwd(x, ldx, M, T, name + ".conv.weight", p, E, bias=P[name + ".conv.bias"])
            outs.append((name, x, ldx, p))
            if i == 0:
                q = self.empty(M, E)
                mn = torch.empty(M, dtype=torch.float32, device=self.dev)
                rs = torch.empty_like(mn)
                s = salt()
                ops.ln_fwd(p, E, P["postnet.ln1.weight"], P["postnet.ln1.bias"], 1e-5, q, E, mn, rs, M,
                           E, dt=self.dt, seed=seed, do_tanh=1, p_o=p_drop, salt_o=s)
                ctx["ln1"] = (p, mn, rs, s)
                x, ldx = q, E
            else:
                x, ldx = p, E
        q3 = self.empty(M, E)
        mn = torch.empty(M, dtype=torch.float32, device=self.dev)
        rs = torch.empty_like(mn)
        s = salt()
        ops.ln_fwd(x, E, P["postnet.ln2.weight"], P["postnet.ln2.bias"], 1e-5, q3, E, mn, rs, M, E,
                   dt=self.dt, seed=seed, do_tanh=1, p_o=p_drop, salt_o=s)
        ctx["ln2"] = (x, mn, rs, s)
        p4 = self.empty(M, NM)
        self._fwd(q3, E, M, T, "postnet.conv_post.conv.weight", p4, NM,
                  bias=P["postnet.conv_post.conv.bias"])
        post = self.empty(M, NM)
        mn3 = torch.empty(M, dtype=torch.float32, device=self.dev)
        rs3 = torch.empty_like(mn3)
        s3 = salt()
        ops.ln_fwd(p4, NM, P["postnet.ln3.weight"], P["postnet.ln3.bias"], 1e-5, post, NM, mn3, rs3, M,
                   NM, dt=self.dt, seed=seed, p_o=p_drop, salt_o=s3, post_add=mel, ldp=NM)
        ctx.update(convs=outs, q3=q3, p4=p4, ln3=(p4, mn3, rs3, s3))
        return post, ctx

    def _postnet_bwd(self, d_post, d_mel_total, keep, ctx, B, T, p_drop, seed):
        """d_mel_total: grad already accumulated on mel (loss + residual); returns masked d_mel."""
        c = self.cfg
        E, NM = c.postnet_embedding_dim, c.n_mels
        M = B * T
        P, G = self.params, self.grads
        p4, mn3, rs3, s3 = ctx["ln3"]
        dp4 = self.empty(M, NM)
        ops.ln_bwd(d_post, NM, p4, NM, mn3, rs3, P["postnet.ln3.weight"], P["postnet.ln3.bias"], dp4,
                   NM, M, NM, dt=self.dt, ws=self.ws(ops.ln_ws(M, NM)), seed=seed, p_o=p_drop,
                   salt_o=s3, dgamma=G["postnet.ln3.weight"], dbeta=G["postnet.ln3.bias"],
                   dcol=G["postnet.conv_post.conv.bias"])
        wname = "postnet.conv_post.conv.weight"
        dq3 = self.empty(M, E)
        self._dgrad(dp4, NM, M, T, wname, dq3, E)
        self._wgrad(dp4, NM, ctx["q3"], E, M, T, wname)
        x, mn, rs, s = ctx["ln2"]
        dx = self.empty(M, E)
        ops.ln_bwd(dq3, E, x, E, mn, rs, P["postnet.ln2.weight"], P["postnet.ln2.bias"], dx, E, M, E,
                   dt=self.dt, ws=self.ws(ops.ln_ws(M, E)), seed=seed, do_tanh=1, p_o=p_drop,
                   salt_o=s, dgamma=G["postnet.ln2.weight"], dbeta=G["postnet.ln2.bias"],
                   dcol=G[ctx["convs"][-1][0] + ".conv.bias"] if len(ctx["convs"]) > 1 else None)
        # ln2's input is the last intermediate conv's output (if any): its bias gradient came
        # with ln2's backward
        bias_done = len(ctx["convs"]) - 1 if len(ctx["convs"]) > 1 else -1
        for i, (name, xin, ldx, p) in reversed(list(enumerate(ctx["convs"]))):
            if i == 0:
                p0, mn1, rs1, s1 = ctx["ln1"]
                dp0 = self.empty(M, E)
                ops.ln_bwd(dx, E, p0, E, mn1, rs1, P["postnet.ln1.weight"], P["postnet.ln1.bias"], dp0,
                           E, M, E, dt=self.dt, ws=self.ws(ops.ln_ws(M, E)), seed=seed, do_tanh=1,
                           p_o=p_drop, salt_o=s1, dgamma=G["postnet.ln1.weight"],
                           dbeta=G["postnet.ln1.bias"],
                           dcol=G[name + ".conv.bias"] if i != bias_done else None)
                dx = dp0
                dmel = self.empty(M, NM)
                self._dgrad(dx, E, M, T, name + ".conv.weight", dmel, NM, residual=d_mel_total,
                            ldr=NM, row_scale_post=keep)
                self._wgrad(dx, E, xin, ldx, M, T, name + ".conv.weight")
                return dmel
            dprev = self.empty(M, E)
            self._dgrad(dx, E, M, T, name + ".conv.weight", dprev, E)
            self._wgrad(dx, E, xin, ldx, M, T, name + ".conv.weight",
                        bias=name + ".conv.bias" if i != bias_done else None)
            dx = dprev

    # ------------------------------------------------------------------ full forward
    def forward(self, tokens, speakers, durations=None, pitch=None, energy=None, pace=1.0,
                pitch_rate=1.0, energy_rate=1.0, intensity=None, training=True, seed=0,
                mel_len_max=None):
        """Model forward (model.py:279-441).  Returns (outputs tuple, ctx for backward)."""
        c = self.cfg
        self.prepare_weights()
        D, H_e, H_d = c.enc_d_model, c.enc_num_head, c.dec_num_head
        NM = c.n_mels
        P = self.params
        tokens = tokens.contiguous()
        speakers = speakers.contiguous()
        B, Tp = tokens.shape
        Mp = B * Tp
        salt = _Salt()
        pe_enc_p = c.enc_dropout if training else 0.0
        pe_dec_p = c.dec_dropout if training else 0.0
        pv = c.variance_predictor_dropout if training else 0.0
        pp_ = c.postnet_dropout if training else 0.0
        ctx = {"B": B, "Tp": Tp, "seed": seed, "training": training, "tokens": tokens,
               "speakers": speakers}
        # encoder prenet + PE + mask (model.py:331-337)
        X = self.empty(Mp, D)
        keep_p = torch.empty(Mp, dtype=torch.float32, device=self.dev)
        ops.embed_fwd(tokens, P["encPreNet.token_embedding.Embedding.weight"], self.pe_enc,
                      c.padding_idx, B, Tp, D, X, keep_p, dt=self.dt)
        kp_enc = torch.empty(Mp, dtype=torch.uint8, device=self.dev)
        ops.keypad_from_tokens(tokens, c.padding_idx, Mp, kp_enc)
        enc_ctx = []
        for i in range(c.enc_num_layers):
            X, lc = self._fft_fwd(X, B, Tp, kp_enc, f"encoder.layers.{i}.", H_e, pe_enc_p, seed, salt)
            enc_ctx.append(lc)
        Xe = self.empty(Mp, D)
        me = torch.empty(Mp, dtype=torch.float32, device=self.dev)
        re_ = torch.empty_like(me)
        ops.ln_fwd(X, D, P["encoder.norm.norm.weight"], P["encoder.norm.norm.bias"], 1e-6, Xe, D, me,
                   re_, Mp, D, dt=self.dt, row_mask=keep_p)                       # :344-347
        # speaker + emotion-intensity conditioning (model.py:352-360)
        E_int = 5
        ldc = round_up(2 * D + E_int, self.epc)
        cat = self.empty(Mp, ldc)
        if intensity is None:
            raise ValueError("intensity (B, T_phon, 5) is required (model.py:356-358)")
        intensity = intensity.to(device=self.dev, dtype=torch.float32).contiguous()
        ops.concat_fwd(Xe, P["speaker_emb.Embedding.weight"], speakers, intensity, B, Tp, D, E_int,
                       cat, ldc, dt=self.dt)
        Z = self.empty(Mp, D)
        self._fwd(cat, ldc, Mp, Tp, "concat_proj.w.weight", Z, D, row_scale=keep_p)
        # variance adaptor (model.py:365-403)
        # with the duration and pitch targets given (training), nothing downstream but the loss
        # reads durPred / pitchPred, so they run on the aux stream (same salt order as sequential)
        aux_h = (self._aux_fork(Z, keep_p) if (self._aux is not None and pitch is not None
                                                and durations is not None) else None)
        pd, dctx, pp, pctx = self._pred_pair_fwd(Z, keep_p, B, Tp, pitch_rate, pv, seed, salt)
        if aux_h is not None:
            self._aux_exit(aux_h)
        kwp = c.pitch_pred_kernel_size
        if pitch is not None:
            pitch = pitch.to(torch.float32).contiguous()
            avg_p = torch.empty(B, Tp, dtype=torch.float32, device=self.dev)
            ops.avg_over_durations(pitch, pitch.shape[1], durations.contiguous(), B, Tp, avg_p,
                                   self.ws(ops.avg_ws(B, pitch.shape[1])))
            a_p = avg_p
        else:
            avg_p = None
            a_p = pp.float()
        Z2 = self.empty(Mp, D)
        ops.embed1d_fwd(Z, a_p, P["pitchEmbed.conv.weight"], P["pitchEmbed.conv.bias"], B, Tp, D, kwp,
                        Z2, dt=self.dt)
        Z2m = Z2.clone()
        ops.mask_rows(Z2m, D, keep_p, Mp, D, dt=self.dt)
        # with the energy target given, the energy predictor's output too only reaches the loss:
        # it joins the duration / pitch chain on the aux stream
        aux_e = (self._aux_fork(Z2m, keep_p) if (aux_h is not None and energy is not None
                                                 and _AUX_ENERGY) else None)
        pe_, ectx = self._pred_fwd(Z2m, keep_p, B, Tp, "energyPred", energy_rate, pv, seed, salt)
        if aux_e is not None:
            self._aux_exit(aux_e)
        kwe = c.energy_pred_kernel_size
        if energy is not None:
            energy = energy.to(torch.float32).contiguous()
            avg_e = torch.empty(B, Tp, dtype=torch.float32, device=self.dev)
            ops.avg_over_durations(energy, energy.shape[1], durations.contiguous(), B, Tp, avg_e,
                                   self.ws(ops.avg_ws(B, energy.shape[1])))
            a_e = avg_e
        else:
            avg_e = None
            a_e = pe_.float()
        Z3 = self.empty(Mp, D)
        ops.embed1d_fwd(Z2, a_e, P["energyEmbed.conv.weight"], P["energyEmbed.conv.bias"], B, Tp, D,
                        kwe, Z3, dt=self.dt)
        # LengthRegulator (model.py:406-413)
        if durations is not None:
            durs, d_is_float = durations.contiguous(), 0
        else:
            durs = torch.clamp(torch.special.expm1(pd.float()), min=0).contiguous()
            d_is_float = 1
        mel_len = torch.empty(B, dtype=torch.int64, device=self.dev)
        cum = torch.empty(B, Tp, dtype=torch.int32, device=self.dev)
        if mel_len_max is None:
            ops.lr_index(durs, d_is_float, float(pace), B, Tp, 0, mel_len, cum, None)
            mel_lens_host = mel_len.cpu()
            Tm = int(mel_lens_host.max())
        else:
            Tm = int(mel_len_max)
            mel_lens_host = None
        frame_src = torch.empty(B, Tm, dtype=torch.int32, device=self.dev)
        ops.lr_index(durs, d_is_float, float(pace), B, Tp, Tm, mel_len, cum, frame_src)
        Mm = B * Tm
        S0 = self.empty(Mm, D)
        keep_m = torch.empty(Mm, dtype=torch.float32, device=self.dev)
        ops.lr_gather(Z3, frame_src, self.pe_dec, B, Tp, Tm, D, S0, keep_m, dt=self.dt)  # :422-423
        kp_dec = torch.empty(Mm, dtype=torch.uint8, device=self.dev)
        ops.keypad_from_lengths(mel_len, B, Tm, kp_dec)
        Xd = S0
        dec_ctx = []
        for i in range(c.dec_num_layers):
            Xd, lc = self._fft_fwd(Xd, B, Tm, kp_dec, f"decoder.layers.{i}.", H_d, pe_dec_p, seed, salt)
            dec_ctx.append(lc)
        Xo = self.empty(Mm, D)
        md = torch.empty(Mm, dtype=torch.float32, device=self.dev)
        rd = torch.empty_like(md)
        ops.ln_fwd(Xd, D, P["decoder.norm.norm.weight"], P["decoder.norm.norm.bias"], 1e-6, Xo, D, md,
                   rd, Mm, D, dt=self.dt)
        mel = self.empty(Mm, NM)
        self._fwd(Xo, D, Mm, Tm, "linear.w.weight", mel, NM, bias=P["linear.w.bias"],
                  row_scale=keep_m)                                                # :430
        post, pn_ctx = self._postnet_fwd(mel, B, Tm, pp_, seed, salt)            # :431
        if aux_h is not None:
            self._aux_join(aux_h[1], pd, pp, pe_, *[t for cc in (dctx, pctx, ectx)
                                                    for t in cc.values()
                                                    if isinstance(t, torch.Tensor)])
        ctx.update(keep_p=keep_p, enc_ctx=enc_ctx, Xenc_last=X, me=me, re=re_, cat=cat, ldc=ldc,
                   Z=Z, dctx=dctx, pctx=pctx, ectx=ectx, a_p=a_p, a_e=a_e, Z2m=Z2m, Tm=Tm,
                   cum=cum, keep_m=keep_m, dec_ctx=dec_ctx, Xdec_last=Xd, md=md, rd=rd, Xo=Xo,
                   pn_ctx=pn_ctx, p_enc=pe_enc_p, p_dec=pe_dec_p, p_var=pv, p_post=pp_,
                   mel_len=mel_len)
        out = (mel.view(B, Tm, NM), post.view(B, Tm, NM), pd.view(B, Tp), pp.view(B, Tp, 1),
               None if avg_p is None else avg_p.view(B, Tp, 1), pe_.view(B, Tp, 1),
               None if avg_e is None else avg_e.view(B, Tp, 1),
               mel_lens_host if mel_lens_host is not None else mel_len)
        return out, ctx

    # ------------------------------------------------------------------ full backward
    def backward(self, ctx, d_mel, d_post, d_dur, d_pitch, d_energy):
        """Backward of ``forward`` for upstream gradients of (mel, postnet, log-dur, pitch,
        energy) outputs; parameter gradients are ACCUMULATED into model._gflat."""
        c = self.cfg
        D, H_e, H_d, NM = c.enc_d_model, c.enc_num_head, c.dec_num_head, c.n_mels
        B, Tp, Tm, seed = ctx["B"], ctx["Tp"], ctx["Tm"], ctx["seed"]
        Mp, Mm = B * Tp, B * Tm
        P, G = self.params, self.grads
        keep_p, keep_m = ctx["keep_p"], ctx["keep_m"]
        def notify(tag):
            # a bucket's all-reduce must see this group's gradients on the main stream and on
            # the weight-gradient side stream: the bucketer makes its communication stream wait
            # on both (events), so the main stream itself never blocks on the side stream
            if self.on_grads_ready is not None:
                self.on_grads_ready(tag, self.grad_streams())
                if (self.dp_late is not None and self.adam_split is not None
                        and not self._adam_late_done and self._aux is not None
                        and self._side is not None and _ADAM_OVERLAP and self.dp_late[0]()):
                    self._adam_launch_late(self.dp_late[1])
        d_mel = d_mel.reshape(Mm, NM).to(self.adt).contiguous()
        d_post = d_post.reshape(Mm, NM).to(self.adt).contiguous()
        d_pitch = d_pitch.reshape(Mp).to(self.adt).contiguous()
        d_dur = d_dur.reshape(Mp).to(self.adt).contiguous()
        aux_h, dZd, dZp, dZe = None, None, None, None
        d_energy = d_energy.reshape(Mp).to(self.adt).contiguous()
        if self._aux is not None:
            # duration, pitch and energy predictor backward chains depend only on the loss
            # gradients and the forward context: run them beside the PostNet / decoder backward
            aux_h = self._aux_fork(d_pitch, d_dur, d_energy, keep_p)
            dZpd = self._pred_pair_bwd(d_dur, ctx["dctx"], d_pitch, ctx["pctx"], keep_p, B, Tp,
                                       ctx["p_var"], seed)
            if _AUX_ENERGY:
                dZe = self._pred_bwd(d_energy, ctx["ectx"], keep_p, B, Tp, "energyPred",
                                     ctx["p_var"], seed)
            self._aux_exit(aux_h)
        # mel receives the loss gradient and the PostNet residual (model.py:431)
        d_mel_total = d_mel.clone()
        ops.add(d_mel_total, d_post, Mm * NM, 1.0, dt=self.dt)
        dmel = self._postnet_bwd(d_post, d_mel_total, keep_m, ctx["pn_ctx"], B, Tm, ctx["p_post"],
                                 seed)
        notify("postnet")
        # mel linear (masked output, model.py:430)
        dXo = self.empty(Mm, D)
        self._dgrad(dmel, NM, Mm, Tm, "linear.w.weight", dXo, D)
        self._wgrad(dmel, NM, ctx["Xo"], D, Mm, Tm, "linear.w.weight")
        self._bias_grad(dmel, NM, Mm, NM, "linear.w.bias")
        dX = self.empty(Mm, D)
        ops.ln_bwd(dXo, D, ctx["Xdec_last"], D, ctx["md"], ctx["rd"], P["decoder.norm.norm.weight"],
                   P["decoder.norm.norm.bias"], dX, D, Mm, D, dt=self.dt, ws=self.ws(ops.ln_ws(Mm, D)),
                   dgamma=G["decoder.norm.norm.weight"], dbeta=G["decoder.norm.norm.bias"])
        notify("linear")
        for i in reversed(range(c.dec_num_layers)):
            dX = self._fft_bwd(dX, ctx["dec_ctx"][i], B, Tm, f"decoder.layers.{i}.", H_d,
                               ctx["p_dec"], seed)
            notify(f"decoder.layers.{i}")
        # LengthRegulator backward: segment sums (masked by the decoder input mask)
        dZ3 = self.empty(Mp, D)
        ops.lr_scatter(dX, ctx["cum"], keep_m, B, Tp, Tm, D, dZ3, dt=self.dt)
        def wg_side(fn, *tensors):
            # a weight-gradient-only pass on the side stream; its inputs stay unmodified after
            h = self._side_enter(*tensors) if _SIDE_SMALL else None
            fn()
            self._side_exit(h)
        kwe = c.energy_pred_kernel_size
        wg_side(lambda: ops.embed1d_bwd(dZ3, ctx["a_e"], B, Tp, D, kwe, G["energyEmbed.conv.weight"],
                                        G["energyEmbed.conv.bias"], dt=self.dt,
                                        ws=self.ws(128 * (kwe + 1) * D)), dZ3, ctx["a_e"])
        if dZe is not None:
            # dZ2 = dZ3 + keep * dZ_energy-input (the sequential chain's residual epilogue, here
            # one add of the aux chain's result, into its buffer: dZ3 stays as the side stream
            # reads it)
            self._aux_join(aux_h[1], dZpd, dZe)
            dZ2 = dZe
            ops.add(dZ2, dZ3, Mp * D, 1.0, dt=self.dt)
        else:
            dZ2 = self._pred_bwd(d_energy, ctx["ectx"], keep_p, B, Tp, "energyPred", ctx["p_var"],
                                 seed, residual=dZ3)
        kwp = c.pitch_pred_kernel_size
        wg_side(lambda: ops.embed1d_bwd(dZ2, ctx["a_p"], B, Tp, D, kwp, G["pitchEmbed.conv.weight"],
                                        G["pitchEmbed.conv.bias"], dt=self.dt,
                                        ws=self.ws(128 * (kwp + 1) * D)), dZ2, ctx["a_p"])
        if aux_h is not None:
            self._aux_join(aux_h[1], dZpd)
            # dZ = keep * (dZ_dur + dZ_pitch + dZ2), as the sequential chain's residual
            # epilogues, summed in fp32 with one rounding (the fused conv1's data gradient
            # already holds dZ_dur + dZ_pitch), into dZpd's buffer (dZ2 stays for the side stream)
            dZ = dZpd
            ops.add3_mask_rows(dZ, dZ2, None, D, keep_p, Mp, D, dt=self.dt)
        else:
            dZ = self._pred_pair_bwd(d_dur, ctx["dctx"], d_pitch, ctx["pctx"], keep_p, B, Tp,
                                     ctx["p_var"], seed, residual=dZ2, post_mask=True)
        notify("variance")
        if (self.adam_split is not None and self._aux is not None and self._side is not None
                and self.on_grads_ready is None and _ADAM_OVERLAP
                and not torch.cuda.is_current_stream_capturing()):
            self._adam_launch_late()
        # concat projection (Z = proj(cat) * keep) -- dZ is already masked
        ldc = ctx["ldc"]
        dcat = self.empty(Mp, 2 * D)
        self._dgrad(dZ, D, Mp, Tp, "concat_proj.w.weight", dcat, 2 * D, n_out=2 * D)
        self._wgrad(dZ, D, ctx["cat"], ldc, Mp, Tp, "concat_proj.w.weight", n_cols=ldc)
        wg_side(lambda: ops.concat_bwd_spk(dcat, 2 * D, ctx["speakers"], B, Tp, D, c.n_speakers,
                                           G["speaker_emb.Embedding.weight"], dt=self.dt,
                                           ws=self.ws(B * D)), dcat, ctx["speakers"])
        dXl = self.empty(Mp, D)
        ops.ln_bwd(dcat, 2 * D, ctx["Xenc_last"], D, ctx["me"], ctx["re"], P["encoder.norm.norm.weight"],
                   P["encoder.norm.norm.bias"], dXl, D, Mp, D, dt=self.dt,
                   ws=self.ws(ops.ln_ws(Mp, D)), row_mask=keep_p,
                   dgamma=G["encoder.norm.norm.weight"], dbeta=G["encoder.norm.norm.bias"])
        notify("conditioning")
        dX = dXl
        for i in reversed(range(c.enc_num_layers)):
            dX = self._fft_bwd(dX, ctx["enc_ctx"][i], B, Tp, f"encoder.layers.{i}.", H_e,
                               ctx["p_enc"], seed)
            notify(f"encoder.layers.{i}")
        ops.embed_bwd(ctx["tokens"], dX, keep_p, Mp, D, c.n_char,
                      G["encPreNet.token_embedding.Embedding.weight"], dt=self.dt,
                      ws=self.ws(ops.embed_bwd_ws(D, c.n_char)))
        self.side_join()
        notify("prenet")
