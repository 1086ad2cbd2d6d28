#!/bin/bash
# session-2 LayerNorm A/B: tests ($1), ln_bench per FS2_LN_PIPE mode, bench A/B ($2..)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab gpurun_out/gab
if [ "$1" != "-" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$1" > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
  tail -2 gpurun_out/ab/t.log
fi
for m in 0 1 2; do
  echo "== FS2_LN_PIPE=$m"
  FS2_LN_PIPE=$m LN_VARIANTS=1 timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/gab/ln.txt 2>&1 || { tail -20 gpurun_out/gab/ln.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gab/ln.txt | grep -v torch
done
shift
for rep in 1 2; do
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$cfg: ms/step %.3f  value %.0f' % (d['ms_per_step'], d['value']))"
done
done
