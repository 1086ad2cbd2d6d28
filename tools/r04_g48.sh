#!/bin/bash
# 256x192 gemm256r instance: GEMM parity tests (product library), bit-exactness and timing
# against gemm_ps_kernel at the decoder conv1 data-gradient shape, step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "gemm or conv or big or persistent or padded" 2>&1 | tail -2 &&
for v in 1 0 1 0; do FS2_G4R48=$v G4R_ONLY=dgrad timeout -k 10 120 python -u tools/g4r_bench.py || exit 1; done &&
python -c "
import torch
a=torch.load('/tmp/g4r_11.pt') if False else None
" && FS2_G4R48=1 timeout -k 10 200 python -u tools/g4r_bench.py > /dev/null && FS2_G4R48=0 timeout -k 10 200 python -u tools/g4r_bench.py > /dev/null &&
python -c "
import torch
a=torch.load('/tmp/g4r_11.pt'); b=torch.load('/tmp/g4r_10.pt')
for k in a:
    d=(a[k].float()-b[k].float()).abs().max().item()
    print(k, 'bit-exact' if torch.equal(a[k], b[k]) else 'DIFF max %g (ref max %g)' % (d, b[k].float().abs().max().item()))
" && bash tools/ab_env.sh 3 "FS2_G4R48=0" "FS2_G4R48=1"
