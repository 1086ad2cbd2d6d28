# round-3 session-2: LDS / MFMA counters of the decoder GEMM call sites, then the serial
# per-kernel totals of the bench step (experiments library)
set -o pipefail
R=$GRAFT_REPO_ROOT
export FS2_HIP_LIB=$R/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
bash tools/pmc.sh pmc_lds "gemm" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU" tools/gemm_bench.py decoder || exit 1
python - <<'PY'
import json, os
d = json.load(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmc_lds/pmc.json"))
for k in d["kernels"]:
    print(k["kernel"][:58], k["grid"], round(k.get("avg_us", 0), 1),
          "conflict/LDS-cycles=%.3f" % (k["SQ_LDS_BANK_CONFLICT"] / max(1, k["SQ_LDS_IDX_ACTIVE"])),
          "mfma_busy=%.2f" % (k["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, 4 * k["SQ_BUSY_CYCLES"])),
          "wait=%.2f" % (k["SQ_WAIT_ANY"] / max(1, k["SQ_WAVE_CYCLES"])))
PY
mkdir -p gpurun_out/s2serial && cd /tmp && FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s2serial/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $R/gpurun_out/s2serial/bench.json 2> $R/gpurun_out/s2serial/err.txt || { tail -5 $R/gpurun_out/s2serial/err.txt; exit 1; }
python $R/tools/rocprof_summary.py stats $R/gpurun_out/s2serial/prof 13 $R/gpurun_out/s2serial/serial_kernel_stats.txt | head -30
