"""CPU: ``bench.py --gpus N`` launches N ranks (BASELINE metric "1/2/4/8 MI355X").

* ``launch_plan``: --gpus -> the torch.distributed.run command, WORLD_SIZE cross-check, the
  refusal to measure fewer devices than asked;
* end to end: ``bench.py --gpus 2 --plumbing-check`` started without a launcher re-runs itself
  under torch.distributed.run and each rank sees RANK / LOCAL_RANK / WORLD_SIZE (gloo, no GPU);
* ``bench.py --gpus 2`` on a box with fewer GPUs exits non-zero instead of measuring one.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env():
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e["OMP_NUM_THREADS"] = "1"
    return e


def test_launch_plan_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, 0, []) is None
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, 1, []) is None


def test_launch_plan_builds_torchrun_command():
    cmd = bench.launch_plan(8, {}, 8, ["--gpus", "8", "--steps", "3"], port=29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3"]


def test_launch_plan_under_launcher_checks_world_size():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, 8, []) is None
    with pytest.raises(bench.LaunchError):
        bench.launch_plan(8, {"WORLD_SIZE": "1"}, 8, [])


def test_launch_plan_refuses_missing_devices():
    with pytest.raises(bench.LaunchError, match="only 1 GPU"):
        bench.launch_plan(2, {}, 1, [])
    with pytest.raises(bench.LaunchError):
        bench.launch_plan(0, {}, 8, [])


def test_bench_gpus2_spawns_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--plumbing-check"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout          # rank 0 only
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["parallelism"] == "dp2"
    assert sorted(d["ranks"]) == [0, 1] and sorted(d["local_ranks"]) == [0, 1]
    assert d["world_sizes"] == [2, 2]


def test_bench_gpus1_plumbing_unchanged():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plumbing-check"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["ranks"] == [0]


def test_bench_refuses_more_gpus_than_visible():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has >= 2 GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr


@pytest.mark.gpu
def test_bench_two_rank_path_rehearsed_on_one_gpu():
    """GPU: the N > 1 bench path end to end -- torch.distributed.run, two ranks, the bucketed
    gradient all-reduce, barriers, max-over-ranks timing and the rank-0 line -- with both ranks
    on GPU 0 over gloo (FS2_BENCH_REHEARSE=1; RCCL needs one GPU per rank).  Not a
    measurement: the line says so."""
    e = _env()
    e["FS2_BENCH_REHEARSE"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={bench._free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-extractor", "--no-fp32-leg", "--no-config2-leg"]
    r = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout          # rank 0 only
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 64
    assert d["config"]["parallelism"] == "dp2" and "rehearsal" in d
    assert d["value"] > 0 and d["build"]["library_source_hash"] == d["build"]["tree_source_hash"]
