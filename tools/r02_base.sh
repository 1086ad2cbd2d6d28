# GPU: baseline of round 2 -- bench line, per-call-site detail, kernel trace + GPU-idle gaps
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-base} && mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extractor > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('ms/step %.3f  value %.0f  roofline %.3f host %.2f' % (d['ms_per_step'], d['value'], d['roofline']['frac'], d['host_enqueue_ms_per_step']))"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --detail > $O/detail.json 2> $O/detail.txt || { tail -20 $O/detail.txt; exit 1; }
grep -v amdgpu.ids $O/detail.txt | head -50
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py stats $GRAFT_REPO_ROOT/$O/prof 13 $GRAFT_REPO_ROOT/$O/kernel_stats.txt | head -40
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py gaps $GRAFT_REPO_ROOT/$O/prof adamw_prep_tiles 10 $GRAFT_REPO_ROOT/$O/gaps.json
