#!/bin/bash
# persistent short-K kernel tile configurations on the encoder-size shapes (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04pk
for c in auto 44 24 22; do
  if [ $c == auto ]; then
    timeout -k 10 120 python -u tools/pk_small_bench.py || exit 1
  else
    FS2_PK_CFG=$c timeout -k 10 120 python -u tools/pk_small_bench.py || exit 1
  fi
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04pk/pk.txt
