#!/bin/bash
# One rocprofv3 --pmc pass over a python script, summarised per (kernel, grid).
# Usage (repo root on the GPU box):
#   bash tools/pmc.sh TAG KERNEL_SUBSTRS "COUNTER ..." script.py [args ...]
# KERNEL_SUBSTRS: comma-separated kernel-name substrings ("" = every kernel).
# Keep within one pass's slots: 8 SQ_, 4 TCC_ (FETCH_SIZE 3, WRITE_SIZE 2), 2 GRBM_.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SUBS=$2; CNT=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $CNT --output-format csv -d $O/p -o run -- python $R/"$@" \
  > $O/run.log 2>&1 || { echo "pmc pass $TAG failed"; tail -20 $O/run.log; exit 1; }
python $R/tools/rocprof_summary.py pmc $O/pmc.json "$SUBS" $O/p
