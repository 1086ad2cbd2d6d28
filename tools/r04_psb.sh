#!/bin/bash
# gemm_ps_kernel: B fragments of the second k-half read in phase 1 (FS2_PS_FLAGS=1024):
# bit-exactness, dgrad timing, step A/B (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for f in 0 1024; do FS2_PS_FLAGS=$f timeout -k 10 200 python -u tools/g4r_bench.py > /tmp/psb_$f.txt && cp /tmp/g4r_11.pt /tmp/psb_$f.pt || exit 1; grep dgrad /tmp/psb_$f.txt | sed "s/^/psflags=$f /"; done &&
python -c "
import torch
a=torch.load('/tmp/psb_0.pt'); b=torch.load('/tmp/psb_1024.pt')
print('bit-exact', all(torch.equal(a[k], b[k]) for k in a))
" && bash tools/ab_env.sh 3 "FS2_PS_FLAGS=0" "FS2_PS_FLAGS=1024"
