#!/bin/bash
# GEMM call sites (filter $1) under env settings ($2..; "-" = defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gab
F=$1; shift
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u tools/gemm_bench.py $F > gpurun_out/gab/g.txt 2>&1 || { tail -20 gpurun_out/gab/g.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gab/g.txt | grep -v blas
done
