"""Train step (emo_rank_tts/fastspeech2/train.py:54-109, 232) and its data-parallel form.

* ``train_step`` is the reference loop body verbatim in structure -- model forward ->
  ``Loss`` -> ``optim.zero_grad()`` -> ``loss['total_loss'].backward()`` -> ``optim.step()``
  (train.py:72-81) -- and works with ``torch.optim.AdamW`` or ``FusedAdamW``.
* ``FusedTrainer`` is the same step without autograd bookkeeping: engine forward, fused loss,
  engine backward into the flat gradient buffer, a bucketed RCCL all-reduce (SUM, averaged in
  the optimizer) launched per bucket as soon as the backward has produced it; the fused AdamW
  of the decoder / mel-linear / PostNet parameters runs on the aux stream during the encoder
  backward (one process: right after the decoder; DP: once their buckets are reduced), the
  rest after the backward (DP: after the last bucket).  One process per GPU, ``torch.distributed`` with the nccl (= RCCL) backend.
"""

import os

import torch
import torch.distributed as dist

from . import ops
from .loss import fused_loss
from .optim import FusedAdamW


def train_step(model, criterion, optim, batch, intensity, epoch=0):
    """train.py:60-81 loop body (intensity given as an input)."""
    (phoneme, spk_ids, phon_len, mel_tgt, pitch_tgt, energy_tgt, duration_tgt, mel_len) = batch[:8]
    predictions = model(phoneme, spk_ids, duration_tgt, pitch_tgt, energy_tgt, intensity=intensity)
    targets = (mel_tgt, duration_tgt, pitch_tgt, energy_tgt, mel_len, phon_len)
    loss = criterion(predictions, targets, epoch)
    optim.zero_grad()
    loss["total_loss"].backward()
    optim.step()
    return predictions, loss


class GradBucketer:
    """Bucketed all-reduce of a flat gradient buffer, overlapped with the backward.

    ``ranges`` are the model's (tag, start, end) backward groups in completion order; they
    are merged into contiguous buckets of at least ``bucket_bytes``.  ``ready(tag, streams)``
    is called by the backward when a group's gradients are queued; a bucket is reduced (async,
    SUM) once its last group is ready.  The reduction is issued from a communication stream
    that first waits (stream-ordered events, no host sync) on every stream in ``streams`` that
    may still be writing gradients -- the main stream and the weight-gradient side stream --
    so neither the host nor the main stream waits for it.  ``finish()`` makes the current
    stream wait for every outstanding reduction.
    """

    def __init__(self, flat, ranges, bucket_bytes=32 << 20, group=None):
        self.flat, self.group = flat, group
        self.comm = torch.cuda.Stream(flat.device) if flat.is_cuda else None
        self.buckets = []          # [(start, end, last_tag)]
        cur = None
        for tag, s, e in ranges:
            if cur is None:
                cur = [s, e, tag]
            else:
                cur[1], cur[2] = e, tag
            if (cur[1] - cur[0]) * flat.element_size() >= bucket_bytes:
                self.buckets.append(tuple(cur))
                cur = None
        if cur is not None:
            self.buckets.append(tuple(cur))
        self.by_tag = {}
        for i, (_, _, tag) in enumerate(self.buckets):
            self.by_tag.setdefault(tag, []).append(i)
        self.handles = {}          # bucket index -> async all-reduce work
        self.launched = set()
        self.late_end = 0          # set_late(): flat end of the parameters updated early

    def _reduce(self, i, streams):
        s, e, _ = self.buckets[i]
        if self.comm is None:
            self.handles[i] = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM,
                                              group=self.group, async_op=True)
        else:
            for st in streams or [torch.cuda.current_stream(self.flat.device)]:
                self.comm.wait_stream(st)
            with torch.cuda.stream(self.comm):
                self.handles[i] = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM,
                                                  group=self.group, async_op=True)
        self.launched.add(i)

    # -- the late parameters' AdamW under DP (FusedTrainer.step): the decoder / mel-linear /
    # PostNet gradients occupy the front of the flat buffer (backward-completion order); once
    # every bucket that holds any of them is reduced, their update may run on the engine's aux
    # stream during the encoder backward, as the one-process step does
    def set_late(self, end):
        self.late_end = int(end)

    def late_launched(self):
        return self.late_end > 0 and all(i in self.launched for i, (s, _, _) in
                                         enumerate(self.buckets) if s < self.late_end)

    def wait_late(self, stream):
        """make ``stream`` wait (stream-ordered) for the all-reduce of every bucket that holds
        late gradients"""
        with torch.cuda.stream(stream):
            for i, (s, _, _) in enumerate(self.buckets):
                if s < self.late_end:
                    self.handles[i].wait()

    def ready(self, tag, streams=None):
        for i in self.by_tag.get(tag, []):
            if i not in self.launched:
                self._reduce(i, streams)

    def finish(self, streams=None):
        for i in range(len(self.buckets)):
            if i not in self.launched:   # groups that never reported (defensive)
                self._reduce(i, streams)
        for h in self.handles.values():
            h.wait()
        if self.comm is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.comm)
        self.handles, self.launched = {}, set()


# opt-in: measured slower on ROCm 7 / MI355X (bench A/B, profiles/r02_graph_ab.txt: B=32 21.88 ms
# eager vs 22.16 ms graph, B=16 14.02 vs 14.46 ms; GPU-idle time per step 0.63 ms eager vs
# 1.50 ms graph): the replayed multi-stream graph leaves more gaps between kernels than the
# eager launches, whose host issue time (8-12 ms/step) is already below the GPU time
_GRAPH = os.environ.get("FS2_GRAPH", "0") not in ("", "0")


class _StepGraph:
    """One captured forward + loss + backward for a fixed batch shape.

    The graph owns static copies of the batch tensors (refreshed by a device copy per step, so
    a caller may hand in a new batch of the same shape every step), the loss vector it writes,
    and every intermediate (torch's graph-private memory pool).  Launch arguments are frozen at
    capture, so the dropout seed is captured as 0 and each replay first writes the step's seed
    into the kernels' device-resident seed base (``ops.set_dropout_seed``); AdamW, whose bias
    corrections change every step, runs eagerly after the replay."""

    def __init__(self, trainer, batch, intensity, mel_len_max):
        self.static = [t.clone() for t in batch[:8]] + [intensity.clone()]
        self.mel_len_max = mel_len_max
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            # one eager pass on the capture stream: workspaces and lazily built tables exist
            # before capture, as torch.cuda.graphs recommends
            trainer.forward_backward(self.static[:8], self.static[8], mel_len_max, seed=0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            self.loss = trainer.forward_backward(self.static[:8], self.static[8], mel_len_max,
                                                 seed=0)
        torch.cuda.synchronize()

    def replay(self, batch, intensity, seed):
        for dst, src in zip(self.static, list(batch[:8]) + [intensity]):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        ops.set_dropout_seed(seed)
        self.graph.replay()
        ops.set_dropout_seed(0)
        return self.loss


class FusedTrainer:
    """One optimiser step of the FastSpeech2 train path on this rank's shard of the batch.

    ``graph=True`` (or FS2_GRAPH=1 on one rank) replays forward + loss + backward as a captured
    HIP graph per batch shape: one host launch instead of ~500 ctypes calls per step.  Off by
    default: measured slower than the eager launches on this stack (see ``_GRAPH``)."""

    def __init__(self, model, loss_weights=(1.0,) * 6, lr=1e-4, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=1e-2, bucket_bytes=32 << 20, graph=None):
        self.model = model
        self.eng = model.engine()
        self.opt = FusedAdamW(model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.weights = tuple(float(w) for w in loss_weights)
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.bucketer = None
        if self.world > 1:
            self.bucketer = GradBucketer(model._gflat, model.group_ranges(), bucket_bytes)
            self.eng.on_grads_ready = self.bucketer.ready
            # the late parameters' AdamW runs inside the backward once their buckets are
            # reduced (engine.dp_late), as the one-process step's does after the decoder
            self.bucketer.set_late(self.eng.late_param_end())
            self.eng.dp_late = (self.bucketer.late_launched, self.bucketer.wait_late)
        self.seed = 0
        # DP steps stay eager: their bucketed all-reduces are issued from the backward hooks,
        # and a captured step would record none of them (its warm-up pass already fired every
        # bucket), so graph replay is refused there rather than silently unreduced
        if graph and self.world > 1:
            raise ValueError("FusedTrainer(graph=True) needs world size 1")
        self.use_graph = (self.world == 1 and _GRAPH) if graph is None else bool(graph)
        self._graphs = {}
        self._torn = False         # a failed split step left the optimizer half-applied

    def _graph_for(self, batch, intensity, mel_len_max):
        key = tuple(tuple(t.shape) for t in batch[:8]) + (tuple(intensity.shape), mel_len_max)
        g = self._graphs.get(key)
        if g is None:
            if len(self._graphs) >= 4:          # shape buckets kept resident
                self._graphs.pop(next(iter(self._graphs)))
            g = self._graphs[key] = _StepGraph(self, batch, intensity, mel_len_max)
        return g

    def forward_backward(self, batch, intensity, mel_len_max=None, seed=None):
        """Forward + fused loss + backward of this rank's shard; the gradients are left in the
        model's flat buffer (with DP on, their bucket all-reduces are queued as the backward
        produces them).  Returns the loss vector."""
        (phoneme, spk_ids, phon_len, mel_tgt, pitch_tgt, energy_tgt, duration_tgt, mel_len) = batch[:8]
        m = self.model
        m._gflat.zero_()
        out, ctx = self.eng.forward(phoneme, spk_ids, duration_tgt, pitch_tgt, energy_tgt,
                                    intensity=intensity, training=True,
                                    seed=self.seed if seed is None else seed,
                                    mel_len_max=mel_len_max if mel_len_max is not None
                                    else mel_tgt.shape[1])
        mel, post, pd, pp, avg_p, pe, avg_e, _ = out
        loss, grads = fused_loss(mel, post, pd, pp.view(pd.shape), pe.view(pd.shape), mel_tgt,
                                 duration_tgt, avg_p.view(pd.shape), avg_e.view(pd.shape), mel_len,
                                 phon_len, self.weights)
        self.eng.backward(ctx, *grads)
        return loss

    def apply(self):
        """Wait for the gradient all-reduce (stream-ordered) and run AdamW with the 1/N mean."""
        if self.bucketer is not None:
            self.bucketer.finish(self.eng.grad_streams())
        self.opt.step(grad_scale=1.0 / self.world)

    def step(self, batch, intensity, mel_len_max=None):
        self.seed += 1
        if self.use_graph:
            if self.world > 1:
                raise RuntimeError("FusedTrainer: graph replay under data parallelism is not "
                                   "supported (the bucket all-reduces are issued from the "
                                   "backward hooks); use the eager step")
            mlm = mel_len_max if mel_len_max is not None else batch[3].shape[1]
            loss = self._graph_for(batch, intensity, mlm).replay(batch, intensity, self.seed)
        else:
            # the AdamW scalars are fixed before the backward, which updates the decoder /
            # PostNet parameters on the aux stream during the encoder backward (under DP once
            # the all-reduce of their gradient buckets is done, GradBucketer.wait_late)
            if self._torn:
                raise RuntimeError("FusedTrainer: an earlier step failed after the decoder / "
                                   "PostNet half of its AdamW update was applied; the optimizer "
                                   "state is inconsistent -- restore it from a checkpoint")
            split = self.opt.fused_images()
            if split:
                scal = self.opt.begin_step(1.0 / self.world)
                self.eng.adam_split = (self.opt, scal)
            try:
                loss = self.forward_backward(batch, intensity, mel_len_max)
            except BaseException:
                if split:
                    if self.eng._adam_late_done:
                        # the late parameters are already updated (aux stream): the step cannot
                        # be undone, and retrying it in place would update them twice
                        self._torn = True
                    else:    # nothing applied: undo the step count, the step may be retried
                        self.opt.step_count -= 1
                    self.eng._adam_late_done = False
                raise
            finally:
                self.eng.adam_split = None
            if split:
                if self.bucketer is not None:
                    self.bucketer.finish(self.eng.grad_streams())
                self.eng.adamw_step_split(self.opt, scal)
                return loss
        self.apply()
        return loss
