# GPU: selected parity tests ($1 = pytest -k expression, "all" = every gpu test) + bench line +
# kernel stats of a short profiled bench.  Usage: bash tools/quick_check.sh "<expr>" [tag]
cd $GRAFT_REPO_ROOT && O=gpurun_out/${2:-quick} && mkdir -p $O
if [ "$1" == "all" ]; then K=(); else K=(-k "$1"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu "${K[@]}" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('ms/step %.3f  value %.0f  roofline %.3f' % (d['ms_per_step'], d['value'], d['roofline']['frac']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py stats $GRAFT_REPO_ROOT/$O/prof 13 $GRAFT_REPO_ROOT/$O/kernel_stats.txt | head -${3:-25}
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py timeline $GRAFT_REPO_ROOT/$O/prof 2 $GRAFT_REPO_ROOT/$O/stream_timeline.txt | tail -1
