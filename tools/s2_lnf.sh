#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab gpurun_out/gab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "layernorm or model or fullsize" > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
tail -2 gpurun_out/ab/t.log
for r in 1 2 4; do
  echo "== FS2_LN_FWD_ROWS=$r"
  FS2_LN_FWD_ROWS=$r timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/gab/ln.txt 2>&1 || { tail -20 gpurun_out/gab/ln.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gab/ln.txt | grep fwd
done
for rep in 1 2; do
for cfg in FS2_AB_DEFAULT=1 FS2_LN_FWD_ROWS=1 FS2_LN_FWD_ROWS=4; do
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$cfg: ms/step %.3f  value %.0f' % (d['ms_per_step'], d['value']))"
done
done
