# GPU: serial (single-stream) rocprofv3 kernel stats of the bench step -> gpurun_out/${1:-ser}
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-ser} && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py stats $GRAFT_REPO_ROOT/$O/prof 13 $GRAFT_REPO_ROOT/$O/kernel_stats.txt | head -${2:-45}
