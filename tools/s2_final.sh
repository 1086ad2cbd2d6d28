#!/bin/bash
# session-2 final pass: smoke + all GPU tests + bench line + kernel stats (tools/gpu_check.sh),
# then the scaled (config 4) bench line and the inference / vocoder bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh r02s2final || exit 1
O=$R/gpurun_out/r02s2final
cd $R && timeout -k 10 300 python -u bench.py --scaled --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $O/bench_scaled.json 2> $O/bench_scaled.err || { tail -20 $O/bench_scaled.err; exit 1; }
tail -1 $O/bench_scaled.json
timeout -k 10 300 python -u tools/infer_bench.py --vocoder > $O/infer.json 2> $O/infer.err || { tail -20 $O/infer.err; exit 1; }
tail -1 $O/infer.json
