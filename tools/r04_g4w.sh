#!/bin/bash
# gemm256r_kernel: more DMA regions issued inside the MFMA section (experiments flags), step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for f in 0 32768 65536 98304; do FS2_G4_FLAGS=$f G4R_ONLY=conv1 G4R_DATA=act timeout -k 10 120 python -u tools/g4r_bench.py || exit 1; done &&
bash tools/ab_env.sh 3 "FS2_G4_FLAGS=0" "FS2_G4_FLAGS=32768" "FS2_G4_FLAGS=65536" "FS2_G4_FLAGS=98304"
