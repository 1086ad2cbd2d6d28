#!/bin/bash
# gemm256r_kernel timing switches at the decoder conv1 forward shape (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export G4R_ONLY="${G4R_ONLY:-conv1}"
for d in rand act zero; do
  for f in ${FLAGS:-0 24 4096 1024 3072 3096 7192}; do
    G4R_DATA=$d FS2_G4_FLAGS=$f timeout -k 10 120 python -u tools/g4r_bench.py || exit 1
  done
done
