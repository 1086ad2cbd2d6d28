#!/bin/bash
# gemm256r_kernel: GEMM parity tests (product library), kernel timings and bit-exactness against
# gemm256_kernel, then the step with either kernel (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "gemm or conv or big or persistent or padded" 2>&1 | tail -2 &&
FS2_G4R=1 timeout -k 10 200 python -u tools/g4r_bench.py && FS2_G4R=0 timeout -k 10 200 python -u tools/g4r_bench.py &&
python -c "
import torch
a=torch.load('/tmp/g4r_1.pt'); b=torch.load('/tmp/g4r_0.pt')
for k in a: print(k, 'bit-exact' if torch.equal(a[k], b[k]) else 'DIFF max %g' % (a[k].float()-b[k].float()).abs().max().item())
" && bash tools/ab_env.sh 3 "FS2_G4R=0" "FS2_G4R=1"
