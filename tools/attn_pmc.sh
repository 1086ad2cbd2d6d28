#!/bin/bash
# Attention counters at the decoder shape (B=32, H=2, dh=192, T=977, p=0.1): two --pmc passes
# over tools/attn_bench.py for the default kernels, and (experiments library) for the paired
# dK/dV kernel (FS2_ATTN_BWD=4).  Summaries: gpurun_out/attnpmc_*/pmc.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export ATTN_T=977 ATTN_P=0.1 ATTN_N=8
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
bash tools/pmc.sh attnpmc_p1 attn "$P1" tools/attn_bench.py > /dev/null || exit 1
bash tools/pmc.sh attnpmc_p2 attn "$P2" tools/attn_bench.py > /dev/null || exit 1
python tools/rocprof_summary.py pmc gpurun_out/attnpmc_default.json attn gpurun_out/attnpmc_p1/p gpurun_out/attnpmc_p2/p > /dev/null || exit 1
export FS2_HIP_LIB=$R/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so FS2_ATTN_BWD=4
bash tools/pmc.sh attnpmc_q1 attn "$P1" tools/attn_bench.py > /dev/null || exit 1
bash tools/pmc.sh attnpmc_q2 attn "$P2" tools/attn_bench.py > /dev/null || exit 1
python tools/rocprof_summary.py pmc gpurun_out/attnpmc_paired.json attn gpurun_out/attnpmc_q1/p gpurun_out/attnpmc_q2/p > /dev/null || exit 1
python - <<'PY'
import json
for tag in ("default", "paired"):
    for r in json.load(open(f"gpurun_out/attnpmc_{tag}.json")):
        w = r.get("SQ_WAIT_ANY", 0) / max(1.0, r.get("SQ_WAVE_CYCLES", 1))
        print(tag, r["kernel"][:60], "grid", r["grid"], "us %.1f" % r["avg_us"],
              "mfma_busy %.3f" % r.get("mfma_busy_frac", 0), "wait_any %.3f" % w)
PY
