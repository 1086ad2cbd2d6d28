#!/bin/bash
# PMC counters of the fused attention kernels at the decoder shape (T=977, p=0): two passes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export ATTN_T=977 ATTN_P=0.0 ATTN_N=5
bash tools/pmc.sh r04ap1 attn_ "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" tools/attn_bench.py &&
bash tools/pmc.sh r04ap2 attn_ "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC" tools/attn_bench.py &&
cat gpurun_out/r04ap1/pmc.json gpurun_out/r04ap2/pmc.json
