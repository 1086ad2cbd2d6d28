#!/bin/bash
# LDS / MFMA counters of the conv1 weight-gradient operand-layout variants (tools/wgrad_bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/p -o run -- python $R/tools/wgrad_bench.py > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
grep -v amdgpu.ids $O/run.log | tail -8
python $R/tools/rocprof_summary.py pmc $O/wgrad_pmc.json gemm256_kernel,gemm_ps_kernel $O/p
