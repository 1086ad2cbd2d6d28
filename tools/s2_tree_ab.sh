#!/bin/bash
# same-box A/B of two trees: the session-start tree (scratch/base, built in place) vs this one
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
for rep in 1 2 3; do
  for t in base final; do
    D=$R; [ "$t" == "base" ] && D=$R/scratch/base
    cd $D && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $R/gpurun_out/ab/tb.json 2> $R/gpurun_out/ab/tb.err || { tail -20 $R/gpurun_out/ab/tb.err; exit 1; }
    python -c "import json; d=json.load(open('$R/gpurun_out/ab/tb.json')); print('$t: ms/step %.3f  value %.0f  conv1 fwd %.1f us' % (d['ms_per_step'], d['value'], d['roofline']['avg_ms']*1e3))"
  done
done
