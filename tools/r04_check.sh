#!/bin/bash
# Round-4 GPU pass: smoke + GPU tests + bench + kernel stats (gpu_check.sh), then the serial
# per-call-site detail (streams off, experiments library).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04a}
bash tools/gpu_check.sh $TAG "$2" nopmc && bash tools/detail.sh && cp gpurun_out/det/detail.txt gpurun_out/$TAG/serial_detail.txt
