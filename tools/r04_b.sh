#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04b
timeout -k 10 120 python -u tools/pk_small_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04b/pk_auto.txt &&
timeout -k 10 300 python -u tools/wgrad1x1_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04b/wgrad1x1.txt
