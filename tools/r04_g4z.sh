#!/bin/bash
# gemm256r_kernel after a schedule change: GEMM / model parity tests, bit-exactness against
# gemm256_kernel (FS2_G4R=0), step A/B of the experiments flag that restores the old placement
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "gemm or conv or big or persistent or padded or model or graph" 2>&1 | tail -2 &&
FS2_G4R=1 timeout -k 10 200 python -u tools/g4r_bench.py > /dev/null && FS2_G4R=0 timeout -k 10 200 python -u tools/g4r_bench.py > /dev/null &&
python -c "
import torch
a=torch.load('/tmp/g4r_11.pt'); b=torch.load('/tmp/g4r_01.pt')
for k in a: print(k, 'bit-exact' if torch.equal(a[k], b[k]) else 'DIFF')
" && bash tools/ab_env.sh 2 "FS2_G4_FLAGS=16384" "FS2_G4_FLAGS=0"
