#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gab
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  echo "== $cfg"
  env $cfg timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/gab/ln.txt 2>&1 || { tail -20 gpurun_out/gab/ln.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gab/ln.txt | grep bwd
done
