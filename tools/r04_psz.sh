#!/bin/bash
# gemm_ps_kernel: phase 1 / 3 DMA inside the MFMA section (FS2_PS_FLAGS 256 / 512): parity of
# the dgrad / projections against the default placement (bit-exact), step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for f in 0 256 512 768; do FS2_PS_FLAGS=$f timeout -k 10 200 python -u tools/g4r_bench.py > /tmp/psz_$f.txt && cp /tmp/g4r_11.pt /tmp/psz_$f.pt || exit 1; grep dgrad /tmp/psz_$f.txt | sed "s/^/psflags=$f /"; done &&
python -c "
import torch
a=torch.load('/tmp/psz_0.pt')
for f in (256, 512, 768):
    b=torch.load('/tmp/psz_%d.pt' % f)
    print(f, all(torch.equal(a[k], b[k]) for k in a))
" && bash tools/ab_env.sh 3 "FS2_PS_FLAGS=0" "FS2_PS_FLAGS=256" "FS2_PS_FLAGS=512" "FS2_PS_FLAGS=768"
