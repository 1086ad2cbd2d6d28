"""GPU, world size 2 on the one MI355X: the data-parallel train path end to end.

Two processes (gloo backend over GPU tensors -- RCCL cannot put two ranks on one device) each
run ``FusedTrainer.step`` on their own shard: the engine's ``on_grads_ready`` hooks, the
bucketed async all-reduce issued from the communication stream after it waited on the main and
weight-gradient side streams, the decoder / PostNet AdamW on the aux stream once their buckets
are reduced (during the encoder backward, as in the one-process step), ``finish()``, the rest of
AdamW and its ``grad_scale = 1/N``.  A single process
then computes each shard's gradient separately with the same seeds and applies one AdamW step
to their mean.  SURVEY 8e: the N-rank gradient equals the mean of the per-shard gradients.

Tolerances: the summed gradient per tensor max|a-b|/max|b| <= 1e-4 (fp32 split-K atomics make
weight gradients non-bit-reproducible); AdamW's first moment likewise; parameters after the step
within fp32 rounding except on elements whose gradient is itself rounding noise (the first
Adam step moves each weight by ~lr * sign(g)): max 2.1 lr, and <= 0.1 % of elements off by
more than 1e-6.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

B, LR = 4, 1e-4


def _setup_path():
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)


def _model_and_batch(rank_seed, dt):
    from fastspeech2 import load_config
    from fastspeech2.model import FastSpeech2
    from fastspeech2.synthetic import make_batch, as_tuple
    cfg = load_config()
    kw = dict(cfg["model"]["fastspeech2"], enc_num_layers=2, dec_num_layers=2)
    torch.manual_seed(0)
    m = FastSpeech2(**kw, n_speakers=4, act_dtype=dt).cuda().train()
    b = make_batch(B=B, tp_min=40, tp_max=60, t_mel_cap=300, seed=100 + rank_seed, device="cuda")
    return m, as_tuple(b)


def _worker(rank, world, port, out_dir, dtname):
    _setup_path()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)   # before any GPU work
    torch.cuda.set_device(0)
    from fastspeech2.train import FusedTrainer
    m, (bt, inten) = _model_and_batch(rank, getattr(torch, dtname))
    tr = FusedTrainer(m, lr=LR, bucket_bytes=4 << 20)
    assert tr.bucketer is not None and len(tr.bucketer.buckets) > 2
    tr.step(bt, inten)
    torch.cuda.synchronize()
    # the decoder / mel-linear / PostNet AdamW ran on the aux stream inside the backward, after
    # the all-reduce of their buckets (the one-process schedule), not after finish()
    assert tr.eng.n_adam_late == 1
    torch.save({"gsum": m._gflat.cpu(), "param": m._flat.cpu(),
                "exp_avg": tr.opt.exp_avg.cpu()}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


@pytest.mark.parametrize("dtname", ["bfloat16"])
def test_two_rank_fused_trainer_equals_mean_gradient_step(cuda, tmp_path, dtname):
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), dtname))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True)
           for r in range(world)]
    # single-process reference: per-shard gradients with the step's seed, then AdamW on the mean
    from fastspeech2.train import FusedTrainer
    grads = []
    for r in range(world):
        m, (bt, inten) = _model_and_batch(r, getattr(torch, dtname))
        tr = FusedTrainer(m, lr=LR)
        tr.seed = 1                       # FusedTrainer.step's first seed
        tr.forward_backward(bt, inten)
        torch.cuda.synchronize()
        grads.append(m._gflat.clone())
    gsum = grads[0] + grads[1]
    m._gflat.copy_(gsum)
    p0 = m._flat.clone()
    # m holds rank 1's model, whose initial parameters equal every rank's (same seed)
    tr.opt.step(grad_scale=1.0 / world)
    torch.cuda.synchronize()
    lay = m._layout
    for r in range(world):
        g = got[r]
        for n, o, k, _, _ in lay:
            ref = gsum[o:o + k].cpu()
            assert _rel(g["gsum"][o:o + k], ref) <= 1e-4, (r, n)
            assert _rel(g["exp_avg"][o:o + k], tr.opt.exp_avg[o:o + k].cpu()) <= 1e-4, (r, n)
        dp = (g["param"] - m._flat.cpu()).abs()
        # an element whose gradient is rounding noise (e.g. the key bias: softmax shift
        # invariance) may take the other sign of +-lr; everything else agrees to fp32 rounding
        assert dp.max().item() <= 2.1 * LR, (r, dp.max().item())
        assert (dp > 1e-6).float().mean().item() <= 1e-3, r
        assert not torch.equal(g["param"], p0.cpu())     # the step moved the weights
    # both ranks hold identical parameters after the step
    assert torch.equal(got[0]["param"], got[1]["param"])
