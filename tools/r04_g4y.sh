#!/bin/bash
# gemm256r_kernel: DMA pieces issued inside the MFMA section (experiments flags 8192 / 16384),
# conv1 forward timings, then the step
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for r in 1 2; do for f in 0 8192 16384 24576; do
  G4R_ONLY=conv1 G4R_DATA=act FS2_G4_FLAGS=$f timeout -k 10 120 python -u tools/g4r_bench.py || exit 1
done; done
