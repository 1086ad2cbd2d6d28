#!/bin/bash
# attention forward timing-only variants (experiments library): FS2_ATTN_FLAGS 1 = no softmax VALU,
# 2 = no K/V DMA after the first tile, 3 = both
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export FS2_HIP_LIB=$(pwd)/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so ATTN_T=977 ATTN_P=0.0
for f in ${FLAGS:-0 1 2 3}; do echo "flags $f"; FS2_ATTN_FLAGS=$f timeout -k 10 60 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
