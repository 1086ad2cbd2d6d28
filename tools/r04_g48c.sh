#!/bin/bash
# encoder FFN conv1 forward: implicit reflect conv on 256x192 gemm256r tiles (FS2_G4R48C) vs the
# padded-image persistent path; microbench, then the step (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in 0 1 0 1; do FS2_G4R48C=$v G4R_ONLY=enc G4R_DATA=act timeout -k 10 120 python -u tools/g4r_bench.py || exit 1; done &&
bash tools/ab_env.sh 3 "FS2_G4R48C=0" "FS2_PAD_FWD=0 FS2_G4R48C=1" "FS2_PAD_FWD=0 FS2_G4R48C=0"
