#!/bin/bash
# bench line + rocprofv3 kernel trace / stats of the product library (no tests)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04p}
O=$(pwd)/gpurun_out/$TAG; mkdir -p $O; R=$(pwd)
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['ms_per_step'], d['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $O/prof_bench.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
python $R/tools/rocprof_summary.py stats $O/prof 17 $O/kernel_stats.txt | head -30
python $R/tools/rocprof_summary.py gaps $O/prof adamw_prep_tiles 10 $O/gaps.json | tail -2
