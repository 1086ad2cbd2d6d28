# GPU: eager vs HIP-graph step A/B (B=32 and B=16) + kernel trace / gaps of the graph step
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-gab} && mkdir -p $O
for B in 32 16; do
for G in "--no-graph" ""; do
timeout -k 10 300 python -u bench.py --batch $B --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg $G > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json; d=json.load(open('$O/b.json')); print('B=$B $G ms/step %.3f host %.2f graph %s' % (d['ms_per_step'], d['host_enqueue_ms_per_step'], d['hip_graph']))"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py gaps $GRAFT_REPO_ROOT/$O/prof adamw_vec_kernel 20 $GRAFT_REPO_ROOT/$O/gaps.json
