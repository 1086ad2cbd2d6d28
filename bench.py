"""Benchmark: train mel-frames/sec of the FastSpeech2-with-emotion-intensity train step
(BASELINE.json metric) at B=32 utterances per GPU, 80-bin mel, default model dims, bf16.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

N>1: one process per GPU with the nccl (= RCCL) backend.  Under torch.distributed.run (the
driver's launch: WORLD_SIZE/RANK/LOCAL_RANK in the environment) WORLD_SIZE must equal --gpus.
Started directly with --gpus N > 1, bench.py first checks that N devices are visible (without
initialising the GPU) and then runs itself under ``torch.distributed.run --nproc-per-node N``
as a child process, exiting with its status.  A step is forward + loss + backward + bucketed
all-reduce + AdamW over one synthetic EmoV-DB-shaped batch per rank, inputs
resident in HBM.  Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist


def _build_record():
    """which sources the loaded library was built from (fs2_source_hash) against this tree's
    (fastspeech2/_native.py refuses a mismatch at load, so these two are equal in any line)"""
    from fastspeech2 import _native
    return {"library": _native.LIB_PATH, "library_source_hash": _native.lib().fs2_source_hash().decode(),
            "tree_source_hash": _native.source_hash()}


MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md)


class LaunchError(RuntimeError):
    pass


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus, env, visible_devices, argv, port=None):
    """What ``bench.py --gpus N`` does in this process: ``None`` = run the bench here (this
    process is one rank, or N == 1), else the child command line that runs N ranks.

    * WORLD_SIZE set (launched by torch.distributed.run): it must equal ``gpus``.
    * WORLD_SIZE unset and gpus > 1: needs ``visible_devices >= gpus``, then returns
      ``python -m torch.distributed.run --nnodes=1 --nproc-per-node gpus --master-addr
      127.0.0.1 --master-port P bench.py <argv>``."""
    if gpus < 1:
        raise LaunchError(f"--gpus {gpus}: need at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise LaunchError(f"WORLD_SIZE={ws} but --gpus {gpus}: the launcher and the "
                              f"bench disagree on the number of ranks")
        return None
    if gpus == 1:
        return None
    if visible_devices < gpus:
        raise LaunchError(f"--gpus {gpus} but only {visible_devices} GPU(s) visible: refusing "
                          f"to measure fewer GPUs than asked")
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
            f"--master-port={port or _free_port()}", os.path.abspath(__file__)] + list(argv)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--plumbing-check", action="store_true",
                    help="CPU test of the launcher: each rank joins a gloo group, rank 0 prints "
                         "the world size and the ranks seen; no GPU is touched")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--max-shape", action="store_true", help="all T_phon=200, d=5 (T_mel=1000)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-utts", type=int, default=0,
                    help="CPU baseline batch size (default: the bench batch itself)")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--single-speaker", action="store_true",
                    help="every utterance speaker 0 (BASELINE config 2 with --batch 16)")
    ap.add_argument("--no-fp32-leg", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="eager launches even if FS2_GRAPH=1 selects the captured HIP graph step")
    ap.add_argument("--no-config2-leg", action="store_true")
    ap.add_argument("--scaled", action="store_true",
                    help="BASELINE config 4: scaled FastSpeech2, hidden 512, FFN 2048, 6+6 layers")
    ap.add_argument("--detail", action="store_true",
                    help="HIP-event time every GEMM / attention call site; table on stderr")
    ap.add_argument("--no-extractor", action="store_true",
                    help="skip the second timed loop that adds the frozen IntensityExtractor")
    return ap.parse_args(argv)


def scaled_config(cfg_all):
    """BASELINE config 4 / SURVEY 8d: hidden 512, FFN 2048 (k/v dims follow), 6+6 layers."""
    import copy
    c = copy.deepcopy(cfg_all)
    m = c["model"]["fastspeech2"]
    for k in ("enc_d_model", "enc_k_dim", "enc_v_dim", "dec_d_model", "dec_k_dim", "dec_v_dim"):
        m[k] = 512
    m["enc_ffn_dim"] = m["dec_ffn_dim"] = 2048
    return c


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may run on (sched affinity),
    capped by OMP_NUM_THREADS when the box sets it (the GPU pool gives one GPU's job a 16-core
    share of a much larger host: os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(cfg_all, args):
    """Oracle (op-for-op PyTorch-CPU fp32 restatement of the reference train step) on
    the SAME synthetic B-utterance batch as the GPU line (rank 0's, seed 0), 1 warm-up step then
    the median of ``cpu_steps`` timed steps."""
    from oracle.fs2_oracle import FastSpeech2Oracle, LossOracle, train_step
    from fastspeech2.synthetic import make_batch, as_tuple
    cores = cpu_threads()
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    model = FastSpeech2Oracle(**cfg_all["model"]["fastspeech2"], n_speakers=4).train()
    crit = LossOracle(**cfg_all["loss"])
    opt = torch.optim.AdamW(model.parameters(), lr=cfg_all["train"]["learning_rate"])
    b = make_batch(B=args.cpu_utts or args.batch, seed=0, max_shape=args.max_shape,
                   single_speaker=args.single_speaker)
    bt, inten = as_tuple(b)
    train_step(model, crit, opt, bt, inten)
    ts = []
    for _ in range(args.cpu_steps):
        t0 = time.perf_counter()
        train_step(model, crit, opt, bt, inten)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    frames = int(b["mel_len"].sum())
    return {"value": frames / t, "unit": "mel-frames/s", "cores": cores, "kind": "port",
            "host_cpu_count": os.cpu_count(),
            "sample": f"the bench batch itself: B={b['mel'].shape[0]} utterances ({frames} valid mel "
                      f"frames, T_mel_max={b['mel'].shape[1]}), fp32, dropout on, {cores} threads "
                      f"(sched affinity / OMP_NUM_THREADS; os.cpu_count()={os.cpu_count()}), "
                      f"median of {len(ts)} steps after 1 warm-up ({t:.2f} s/step); "
                      f"oracle/fs2_oracle.py"}


def timed_leg(trainer, bt, inten, Tm, frames_local, steps, warmup, world):
    """K timed steps of ``trainer`` on one resident batch (barrier + synchronize on both sides,
    max over ranks); returns (whole-job frames/s, ms per step)."""
    for _ in range(warmup):
        trainer.step(bt, inten, mel_len_max=Tm)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.step(bt, inten, mel_len_max=Tm)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device="cuda")
    fr = torch.tensor([frames_local], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(fr, op=dist.ReduceOp.SUM)
    el = float(el.item())
    return float(fr.item()) * steps / el, el / steps * 1e3


def secondary_legs(cfg_all, args, rank, world):
    """Secondary lines beside ``value``: the fp32 train step (the reference trains in fp32, no
    AMP: train.py:72-81) at the same batch, and BASELINE config 2 (B=16, single speaker 'bea',
    bf16)."""
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    out = {}
    legs = []
    if not args.no_fp32_leg and args.dtype != "fp32":
        legs.append(("fp32", torch.float32, args.batch, args.single_speaker, 3, 1))
    if not args.no_config2_leg and not (args.batch == 16 and args.single_speaker):
        legs.append(("config2_b16_single_speaker_bf16", torch.bfloat16, 16, True, args.steps, 3))
    for name, dt, B, single, steps, warm in legs:
        torch.manual_seed(0)
        model = FastSpeech2(**cfg_all["model"]["fastspeech2"], n_speakers=4, act_dtype=dt).cuda().train()
        tr = FusedTrainer(model, lr=cfg_all["train"]["learning_rate"])
        b = make_batch(B=B, seed=rank, max_shape=args.max_shape, device="cuda",
                       single_speaker=single)
        bt, inten = as_tuple(b)
        v, ms = timed_leg(tr, bt, inten, b["mel"].shape[1], int(b["mel_len"].sum()), steps, warm,
                          world)
        out[name] = {"value": v, "unit": "mel-frames/s", "ms_per_step": ms, "steps": steps,
                     "batch_per_gpu": B, "single_speaker": single,
                     "dtype": "fp32" if dt == torch.float32 else "bf16",
                     "T_mel_max": int(b["mel"].shape[1])}
        del tr, model
        torch.cuda.empty_cache()
    return out


def pmc_traffic(kind="roofline", kernel=None):
    """HBM bytes per launch of a roofline kernel from the newest committed PMC summary of that
    kernel: profiles/r*_<kind>_traffic.json (written by tools/rocprof_summary.py traffic from two
    separate rocprofv3 --pmc passes of this same bench command), or -- on the GPU box, where
    profiles/ is not shipped -- its copy in bench_pmc.json at the repository root (refreshed by
    tools/rocprof_summary.py pin)."""
    import glob
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{kind}_traffic.json")))
    for h in reversed(hits):
        d = json.load(open(h))
        if kernel is None or d.get("kernel_substr", "").startswith(kernel):
            return d["hbm_bytes_per_launch"], os.path.relpath(h, ROOT)
    pinned = os.path.join(ROOT, "bench_pmc.json")
    if os.path.exists(pinned):
        d = json.load(open(pinned)).get(kind)
        if d and (kernel is None or d.get("kernel_substr", "").startswith(kernel)):
            return d["hbm_bytes_per_launch"], d["source"]
    return None, None


def detail_table(ks, eng, B, steps, elapsed):
    """Per-call-site time (ms/step) and achieved TFLOP/s of every tagged GEMM / attention."""
    rows = []
    D = eng.cfg.enc_d_model
    for tag, (n, ms) in ks.items():
        if ":" not in tag:
            continue
        kind, wname, T = tag.split(":")
        T = int(T[1:])
        M = B * T
        if kind.startswith("attn"):
            H = eng.cfg.dec_num_head
            fl = 4.0 * B * T * T * D * (1 if kind == "attn_fwd" else 2.5)
        else:
            O, C, KW = eng._wspecs[wname.replace("layers.*", "layers.0")]
            fl = 2.0 * M * O * C * KW
        per_step = n / steps
        rows.append((ms * per_step, tag, per_step, ms, fl / (ms * 1e-3) / 1e12))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"# detail: step {elapsed / steps * 1e3:.2f} ms; tagged {tot:.2f} ms/step", file=sys.stderr)
    for r in rows:
        print(f"{r[0]:8.3f} ms/step {r[2]:5.1f}x {r[3] * 1e3:8.1f} us {r[4]:7.1f} TF/s  {r[1]}",
              file=sys.stderr)


def extractor_leg(cfg_all, args, trainer, b, bt, Tm, dt, world, frames_local):
    """The reference train loop body INCLUDING the frozen IntensityExtractor forward + phoneme
    averaging (train.py:69-81), timed the same way over ``steps`` steps.  Reported
    beside ``value`` (whose definition, SURVEY 8d, excludes the extractor)."""
    from fastspeech2.intensity import IntensityExtractor, get_intensity_representation
    from fastspeech2.flops import extractor_flops
    from fastspeech2.synthetic import as_collate
    rc = cfg_all["model"]["rank_model"]
    torch.manual_seed(1)
    ext = IntensityExtractor(cfg_all["audio"]["n_mels"], rc["n_heads"], 5, rc["n_encoder_layers"],
                             rc["hidden_dim"], rc["kernel_size"], rc["dropout"],
                             act_dtype=dt).cuda()
    coll = as_collate(b)
    for _ in range(2):
        rep = get_intensity_representation(ext, coll)
        trainer.step(bt, rep, mel_len_max=Tm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        get_intensity_representation(ext, coll)
    torch.cuda.synchronize()
    t_ext = (time.perf_counter() - t0) / args.steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rep = get_intensity_representation(ext, coll)
        trainer.step(bt, rep, mel_len_max=Tm)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device="cuda")
    fr = torch.tensor([frames_local], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(fr, op=dist.ReduceOp.SUM)
    el = float(el.item())
    fl = extractor_flops(args.batch, Tm, rc["hidden_dim"], rc["n_encoder_layers"],
                         rc["kernel_size"])
    return {"value": float(fr.item()) * args.steps / el, "unit": "mel-frames/s",
            "ms_per_step": el / args.steps * 1e3,
            "extractor_ms": t_ext * 1e3, "extractor_flop": fl,
            "extractor_tflops": fl / t_ext / 1e12,
            "note": "train step + frozen IntensityExtractor fwd + phoneme averaging "
                    "(train.py:69-81); extractor weights random-init, rank_X from the batch"}


def plumbing_check(world, rank, local):
    """--plumbing-check: the rank environment the launcher produced, gathered over gloo."""
    if world > 1:
        dist.init_process_group("gloo")
    mine = torch.tensor([rank, local, world], dtype=torch.int64)
    got = [torch.zeros_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(got, mine)
    else:
        got = [mine]
    if rank == 0:
        print(json.dumps({"plumbing": True, "n_gpus": world, "parallelism": f"dp{world}",
                          "ranks": [int(g[0]) for g in got],
                          "local_ranks": [int(g[1]) for g in got],
                          "world_sizes": [int(g[2]) for g in got]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    try:
        # torch.cuda.device_count() does not initialise the GPU on this stack, so the child
        # ranks start from a process that never touched the device
        visible = args.gpus if args.plumbing_check else torch.cuda.device_count()
        cmd = launch_plan(args.gpus, os.environ, visible, sys.argv[1:])
    except LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    if cmd is not None:
        sys.exit(subprocess.run(cmd).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing_check:
        plumbing_check(world, rank, local)
        return
    # FS2_BENCH_REHEARSE=1 under torch.distributed.run: every rank on GPU 0 over gloo -- a
    # rehearsal of the N > 1 code path (launcher, bucketed gradient all-reduce, barriers,
    # max-over-ranks timing, rank-0 line) on a one-GPU box; never a measurement
    rehearse = world > 1 and os.environ.get("FS2_BENCH_REHEARSE") == "1"
    if local >= torch.cuda.device_count() and not rehearse:
        print(f"bench.py: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) "
              f"visible", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(0 if rehearse else local)
    if rehearse:
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from fastspeech2 import load_config
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple, as_collate
    from fastspeech2.timing import KernelTimer
    from fastspeech2.flops import train_flops, extractor_flops
    cfg_all = load_config()
    if args.scaled:
        cfg_all = scaled_config(cfg_all)
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    model = FastSpeech2(**cfg_all["model"]["fastspeech2"], n_speakers=4, act_dtype=dt).cuda().train()
    trainer = FusedTrainer(model, lr=cfg_all["train"]["learning_rate"])
    b = make_batch(B=args.batch, seed=rank, max_shape=args.max_shape, device="cuda",
                   single_speaker=args.single_speaker)
    bt, inten = as_tuple(b)
    Tm = b["mel"].shape[1]
    Tp = b["phoneme"].shape[1]
    frames_local = int(b["mel_len"].sum())
    if args.detail or args.no_graph:
        trainer.use_graph = False
    for _ in range(args.warmup):
        trainer.step(bt, inten, mel_len_max=Tm)
    torch.cuda.synchronize()
    timer = KernelTimer()
    timer.detail = args.detail
    # FS2_BENCH_NO_TIMER=1 (A/B runs): no HIP-event brackets in the timed region
    trainer.eng.timer = None if os.environ.get("FS2_BENCH_NO_TIMER") else timer
    if trainer.eng.timer is not None:
        # one more untimed step counts the brackets; their events are created before t0
        trainer.step(bt, inten, mel_len_max=Tm)
        torch.cuda.synchronize()
        n_ev = timer.n_events()
        timer.reset()
        timer.reserve(n_ev * args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(bt, inten, mel_len_max=Tm)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    trainer.eng.timer = None
    ks = timer.summary()
    graphed = trainer.use_graph
    if graphed:
        # a graph replay runs the captured launches without the host-side HIP-event brackets:
        # time the roofline kernel in an eager pass of the same step (same kernels, arguments
        # and inputs), on the stream the kernel is launched on
        trainer.use_graph = False
        timer = KernelTimer()
        trainer.eng.timer = timer
        for _ in range(args.steps):
            trainer.step(bt, inten, mel_len_max=Tm)
        torch.cuda.synchronize()
        trainer.eng.timer = None
        ks = timer.summary()
        trainer.use_graph = True
    # host time to issue one step's launches, from an idle queue: 3 steps enqueued right after
    # a synchronize (inside the timed loop the host runs ~10 steps ahead of the GPU and then
    # blocks on the HIP queue's back-pressure, which made "host time" track the GPU's)
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(3):
        trainer.step(bt, inten, mel_len_max=Tm)
    host_enqueue = (time.perf_counter() - h0) / 3
    torch.cuda.synchronize()
    if args.detail and rank == 0:
        detail_table(ks, trainer.eng, args.batch, args.steps, elapsed)
    tmax = torch.tensor([elapsed], device="cuda")
    ftot = torch.tensor([frames_local], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(ftot, op=dist.ReduceOp.SUM)
    elapsed = float(tmax.item())
    frames_all = float(ftot.item())
    loss_v = loss.float().cpu().tolist()
    ext_info = None
    if not args.no_extractor:
        ext_info = extractor_leg(cfg_all, args, trainer, b, bt, Tm, dt, world, frames_local)
    legs = secondary_legs(cfg_all, args, rank, world)
    if rank == 0:
        c = model.cfg
        D, F, KW = c.dec_d_model, c.dec_ffn_dim, c.ffn_cnn_kernel_size_list[0]
        n, ms = ks.get("ffn_conv1_fwd.decoder", (0, float("nan")))
        kflop = 2.0 * (args.batch * Tm) * F * (KW * D)
        achieved = kflop / (ms * 1e-3) / 1e12 if n else None
        traffic, traffic_src = (pmc_traffic("roofline", "gemm_w4b_kernel<false, 8>")
                                if not args.scaled else (None, None))
        # second entry: the decoder FFN conv1 weight gradient, the largest GEMM bucket of the
        # step (2 M F 9D per launch like the forward); it runs on the side stream beside the
        # main stream's conv1 data gradient, so its duration is the shared-GPU one
        wn, wms = ks.get("ffn_conv1_wgrad.decoder", (0, float("nan")))
        wach = kflop / (wms * 1e-3) / 1e12 if wn else None
        wtraffic, wtraffic_src = (pmc_traffic("wgrad", "gemm_ps_kernel<0, 64, 0, 1>")
                                  if not args.scaled else (None, None))
        step_ms = elapsed / args.steps * 1e3
        step_tflops = train_flops(c, args.batch, Tp, Tm) * world / (step_ms * 1e-3) / 1e12
        fpf = train_flops(c, 1, 200, 1000) / 1000.0
        line = {
            "metric": "train mel-frames/sec at B=32, 80-bin mel; 1/2/4/8 MI355X",
            "value": frames_all * args.steps / elapsed,
            "unit": "mel-frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": step_ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic (seeded EmoV-DB-shaped batches, random-init weights)",
            "config": {"workload": f"FastSpeech2 train step (fwd+loss+bwd+allreduce+AdamW), "
                                   f"B={args.batch}/GPU, T_phon_max={Tp}, T_mel_max={Tm}, "
                                   f"D={c.enc_d_model} F={c.enc_ffn_dim} "
                                   f"{c.enc_num_layers}+{c.dec_num_layers} FFT layers, 80 mels"
                                   + (", max-shape" if args.max_shape else "")
                                   + (", single speaker" if args.single_speaker else ""),
                       "global_batch": args.batch * world, "seq_len": Tm,
                       "valid_mel_frames_per_step": frames_all, "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "kernel": "decoder FFN conv1 (k=9) fwd: a plain GEMM with overlapping A rows over the reflect-padded token image (gemm_w4b_kernel<false, 8>: 256x256 tiles on 4 waves of 128x128, 64-deep stages through 2 LDS-DMA slots, bias + ReLU + pad-row drop in the epilogue); flop counted on the B*T_mel valid rows; the padded image is written by the LayerNorm before it (fs2_ln_fwd img), no separate copy",
                         "achieved": achieved, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved / MFMA_BF16_PEAK_TFLOPS) if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "launches": n, "avg_ms": ms,
                         "flop_per_launch": kflop,
                         "timing": ("HIP events on the engine stream around each launch, in an "
                                    "eager pass of the same steps after the graph-replayed "
                                    "timed region" if graphed else
                                    "HIP events on the engine stream over the timed region")},
            "roofline_conv1_wgrad": {
                "bound": "mfma", "kernel": "decoder FFN conv1 (k=9) weight gradient: K-major GEMM "
                                           "over channel-major padded dY / X images (conv_mode 6, "
                                           "gemm_ps_kernel<0, 64, 0, 1>), split-K fp32 slices; "
                                           "the two image transposes are separate launches",
                "achieved": wach, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": (wach / MFMA_BF16_PEAK_TFLOPS) if wach else None,
                "traffic": wtraffic, "traffic_source": wtraffic_src,
                "launches": wn, "avg_ms": wms, "flop_per_launch": kflop,
                "timing": "HIP events on the weight-gradient side stream around the GEMM launch; "
                          "it is enqueued beside the main stream's conv1 data gradient (a "
                          "persistent kernel holding one block per CU), so the duration includes "
                          "its wait for CUs (DESIGN.md 6.4 has the standalone time)"},
            "hip_graph": graphed,
            **({"rehearsal": f"gloo, {world} ranks on one GPU: the N > 1 code path, NOT a "
                             "measurement"} if rehearse else {}),
            "build": _build_record(),
            # the step-level roofline on VALID frames -- frames/s x the train FLOPs
            # of one mel frame at T_phon=200, T_mel=1000 (338.8 MFLOP at default dims) / peak
            "roofline_step": {"bound": "mfma",
                              "achieved": frames_all * args.steps / elapsed * fpf / 1e12 / world,
                              "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s per GPU",
                              "frac": frames_all * args.steps / elapsed * fpf / 1e12 / world
                              / MFMA_BF16_PEAK_TFLOPS,
                              "flop_per_valid_frame": fpf,
                              "definition": "SURVEY 8(d): frames/s x train FLOP per mel frame "
                                            "(fwd + 2x bwd at T_phon=200, T_mel=1000) / peak"},
            "step_mfma_frac": step_tflops / (MFMA_BF16_PEAK_TFLOPS * world),
            "host_enqueue_ms_per_step": host_enqueue * 1e3,
            "kernel_ms": {k: v[1] for k, v in ks.items()},
            "loss_total_last": loss_v[0],
        }
        if ext_info is not None:
            line["with_intensity_extractor"] = ext_info
        line.update(legs)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(cfg_all, args)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
