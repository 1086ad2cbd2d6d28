#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gab
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  echo "== $cfg"
  env LN_POSTNET=1 $cfg timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/gab/lnp.txt 2>&1 || { tail -20 gpurun_out/gab/lnp.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gab/lnp.txt
done
