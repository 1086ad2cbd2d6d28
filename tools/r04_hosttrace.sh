#!/bin/bash
# kernel trace + HIP runtime (API) trace of a short product bench: when did the host enqueue each
# launch relative to its start on the GPU (host-bound gaps vs dependency waits)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=$(pwd)/gpurun_out/hosttrace; mkdir -p $O; R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $O/bench.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
ls -la $O/prof/* | head; du -sh $O
