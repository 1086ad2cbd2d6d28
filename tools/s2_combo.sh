#!/bin/bash
# session-2: test subset ($1, "-" = none), GEMM call sites under $2 (space-separated env
# settings, "-" = defaults), then interleaved bench A/B over the remaining args
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab gpurun_out/gab
if [ "$1" != "-" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$1" > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
  tail -2 gpurun_out/ab/t.log
fi
for cfg in $2; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  echo "== gemm $cfg"
  env $cfg timeout -k 10 200 python -u tools/gemm_bench.py decoder > gpurun_out/gab/g.txt 2>&1 || { tail -20 gpurun_out/gab/g.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gab/g.txt | grep -v blas
done
shift; shift
for rep in 1 2; do
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$cfg: ms/step %.3f  value %.0f' % (d['ms_per_step'], d['value']))"
done
done
