#!/bin/bash
# session-2 baseline: tests + bench + rocprof (tools/gpu_check.sh), then the GEMM call-site
# microbench with hipBLASLt on the same shapes as a ceiling reference
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh s2base || exit 1
cd $R && FS2_GB_BLAS=1 timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/s2base/gemm_blas.txt 2>&1 || { tail -20 gpurun_out/s2base/gemm_blas.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s2base/gemm_blas.txt
