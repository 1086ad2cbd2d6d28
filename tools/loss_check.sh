set -o pipefail
mkdir -p gpurun_out/loss
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "loss" 2>&1 | tail -2
timeout -k 10 120 python -u tools/loss_bench.py 2>&1 | grep -v amdgpu.ids
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/loss/prof -o run -- python $GRAFT_REPO_ROOT/tools/loss_bench.py > /dev/null 2>&1
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py stats $GRAFT_REPO_ROOT/gpurun_out/loss/prof 23 $GRAFT_REPO_ROOT/gpurun_out/loss/stats.txt | head -12
