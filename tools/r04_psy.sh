#!/bin/bash
# gemm_ps_kernel with phase 0's DMA in the MFMA section by default: parity tests (product
# library), bit-exactness against the old placement (FS2_PS_FLAGS=64), step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread 2>&1 | tail -2 &&
FS2_PS_FLAGS=0 timeout -k 10 200 python -u tools/g4r_bench.py > /dev/null && cp /tmp/g4r_11.pt /tmp/ps_new.pt &&
FS2_PS_FLAGS=64 timeout -k 10 200 python -u tools/g4r_bench.py > /dev/null &&
python -c "
import torch
a=torch.load('/tmp/ps_new.pt'); b=torch.load('/tmp/g4r_11.pt')
for k in a: print(k, 'bit-exact' if torch.equal(a[k], b[k]) else 'DIFF')
" && bash tools/ab_env.sh 2 "FS2_PS_FLAGS=64" "FS2_PS_FLAGS=0"
