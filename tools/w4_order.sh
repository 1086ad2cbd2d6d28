#!/bin/bash
# GPU: conv1 forward block order A/B (tools/w4_order.py) + FETCH_SIZE per launch for each order
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/w4o
for f in 0 8 0 8; do
  FS2_W4_FLAGS=$f timeout -k 10 120 python -u tools/w4_order.py 2>&1 | grep -v amdgpu.ids || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 0 8; do
  FS2_W4_FLAGS=$f timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/w4o/f$f -o run -- python3 tools/w4_order.py > gpurun_out/w4o/f$f.log 2>&1 || exit 1
  FS2_W4_FLAGS=$f timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/w4o/w$f -o run -- python3 tools/w4_order.py > gpurun_out/w4o/w$f.log 2>&1 || exit 1
  python3 tools/rocprof_summary.py pmc gpurun_out/w4o/pmc$f.json w4b gpurun_out/w4o/f$f gpurun_out/w4o/w$f | cut -c1-400
done
