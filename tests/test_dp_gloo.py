"""CPU, world_size 2, gloo: the data-parallel gradient path.

Each rank computes the oracle gradients of its own shard (per-shard parity),
packs them into the flat buffer in the product's backward-completion layout, announces the
groups in backward order through ``GradBucketer`` (the same object FusedTrainer drives on the
GPU with RCCL) and the reduced buffer, divided by the world size as FusedAdamW does, must
equal the mean of the per-shard gradients computed in a single process.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

TINY = dict(enc_num_layers=1, enc_num_head=2, enc_d_model=16, enc_ffn_dim=32, enc_k_dim=16,
            enc_v_dim=16, enc_dropout=0.1, dec_num_layers=1, dec_num_head=2, dec_d_model=16,
            dec_ffn_dim=32, dec_k_dim=16, dec_v_dim=16, dec_dropout=0.1, normalize_before=False,
            ffn_type="1dcnn", ffn_cnn_kernel_size_list=[9, 1], n_char=20, n_mels=16,
            postnet_embedding_dim=16, postnet_kernel_size=5, postnet_n_convolutions=5,
            postnet_dropout=0.5, padding_idx=0, dur_pred_kernel_size=3, pitch_pred_kernel_size=3,
            energy_pred_kernel_size=3, variance_predictor_dropout=0.5)
LOSS = dict(log_scale_durations=True, ssim_loss_weight=1.0, duration_loss_weight=1.0,
            pitch_loss_weight=1.0, energy_loss_weight=1.0, mel_loss_weight=1.0,
            postnet_mel_loss_weight=1.0)


def _shard_grads(rank):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle.fs2_oracle import FastSpeech2Oracle, LossOracle
    from fastspeech2.synthetic import make_batch, as_tuple
    torch.manual_seed(0)
    m = FastSpeech2Oracle(**TINY, n_speakers=4).eval()
    b = make_batch(B=2, tp_min=12, tp_max=14, t_mel_cap=60, n_mels=16, n_char=20, seed=100 + rank)
    bt, inten = as_tuple(b)
    pred = m(bt[0], bt[1], bt[6], bt[4], bt[5], intensity=inten)
    loss = LossOracle(**LOSS)(pred, (bt[3], bt[6], bt[4], bt[5], bt[7], bt[2]), 0)
    loss["total_loss"].backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


def _layout():
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from fastspeech2.model import FastSpeech2, _group_key, group_tag
    m = FastSpeech2(**TINY, n_speakers=4)
    params = dict(m.named_parameters())
    order = sorted(params, key=lambda n: _group_key(n, 1, 1))
    layout, off = [], 0
    for n in order:
        k = params[n].numel()
        layout.append((n, off, k, group_tag(_group_key(n, 1, 1))))
        off += (k + 15) // 16 * 16
    ranges = []
    for n, o, k, tag in layout:
        end = o + (k + 15) // 16 * 16
        if ranges and ranges[-1][0] == tag:
            ranges[-1] = (tag, ranges[-1][1], end)
        else:
            ranges.append((tag, o, end))
    return layout, off, ranges


def _worker(rank, world, port, out_path):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastspeech2.train import GradBucketer
    g = _shard_grads(rank)
    layout, total, ranges = _layout()
    flat = torch.zeros(total)
    for n, o, k, _ in layout:
        flat[o:o + k] = g[n].reshape(-1)
    bk = GradBucketer(flat, ranges, bucket_bytes=4096)
    for tag, _, _ in ranges:          # backward-completion order
        bk.ready(tag)
    bk.finish()
    flat /= world                     # FusedAdamW grad_scale = 1/world
    if rank == 0:
        torch.save(flat, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_dp_allreduce_equals_mean_of_shard_grads(tmp_path):
    world = 2
    out = str(tmp_path / "flat.pt")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    layout, total, _ = _layout()
    ref = [_shard_grads(r) for r in range(world)]
    for n, o, k, _ in layout:
        mean = (ref[0][n] + ref[1][n]).reshape(-1) / world
        torch.testing.assert_close(got[o:o + k], mean, rtol=1e-5, atol=1e-7)
