#!/bin/bash
# gemm_ps_kernel: DMA regions inside the MFMA section (FS2_PS_FLAGS 64 / 128), dgrad microbench
# and the step (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for f in 0 64 128 192 0 64 128 192; do FS2_PS_FLAGS=$f G4R_ONLY=dgrad timeout -k 10 120 python -u tools/g4r_bench.py | sed "s/^/psflags=$f /" || exit 1; done &&
bash tools/ab_env.sh 3 "FS2_PS_FLAGS=0" "FS2_PS_FLAGS=64" "FS2_PS_FLAGS=128" "FS2_PS_FLAGS=192"
