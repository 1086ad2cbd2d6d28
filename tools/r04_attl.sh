#!/bin/bash
# attention kernels with the next tile's DMA issued after the barrier (FS2_ATTN_FLAGS=8,
# experiments library): parity tests under the flag, standalone timings, step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export FS2_HIP_LIB=$(pwd)/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
FS2_ATTN_FLAGS=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "attention or attn or flash" 2>&1 | tail -2 &&
for f in 0 8 0 8; do FS2_ATTN_FLAGS=$f ATTN_T=977 ATTN_P=0.1 timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/flags=$f /" | tail -4 || exit 1; done &&
bash tools/ab_env.sh 3 "FS2_ATTN_FLAGS=0" "FS2_ATTN_FLAGS=8"
