#!/bin/bash
# gemm256r_kernel epilogues: GEMM parity tests (product library), bit-exactness of the
# register-direct epilogue (TR) against gemm256_kernel, conv1 forward timings
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "gemm or conv or big or persistent or padded" 2>&1 | tail -2 &&
FS2_G4R=1 timeout -k 10 200 python -u tools/g4r_bench.py && FS2_G4R=0 timeout -k 10 200 python -u tools/g4r_bench.py &&
python -c "
import torch
a=torch.load('/tmp/g4r_1.pt'); b=torch.load('/tmp/g4r_0.pt')
for k in a: print(k, 'bit-exact' if torch.equal(a[k], b[k]) else 'DIFF max %g' % (a[k].float()-b[k].float()).abs().max().item())
" &&
for tr in 1 0 1 0; do FS2_G4R_TR=$tr G4R_ONLY=conv1 G4R_DATA=act timeout -k 10 120 python -u tools/g4r_bench.py || exit 1; done &&
FS2_G4R_TR=0 FS2_G4_FLAGS=4096 G4R_ONLY=conv1 G4R_DATA=act timeout -k 10 120 python -u tools/g4r_bench.py &&
bash tools/ab_env.sh 2 "FS2_G4R_TR=0" "FS2_G4R_TR=1"
