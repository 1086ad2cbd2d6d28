#!/bin/bash
# One GPU-box pass: GPU parity tests, bench line, rocprofv3 kernel stats of a short bench.
# Usage (from the repo root on the box): bash tools/gpu_check.sh [tag] [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
  tail -3 $O/smoke.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg \
  > $O/prof_bench.json 2> $O/prof.err || { echo "rocprof failed"; tail -20 $O/prof.err; exit 1; }
python $R/tools/rocprof_summary.py stats $O/prof 17 $O/kernel_stats.txt | head -40
# roofline kernel: the decoder FFN conv1 forward (4-wave kernel over the reflect-padded image:
# 124 x 6 tiles of 256 x 256)
python $R/tools/rocprof_summary.py kernel $O/prof "gemm_w4b_kernel<false, 8>" 190464 100 | tee $O/roofline_kernel_trace.txt
# second roofline kernel: the decoder FFN conv1 weight gradient (conv_mode 6 on the persistent
# kernel: 84 tiles x 2 splits on the 208-CU side-stream budget -> 168 blocks of 512; the encoder's, same grid, runs < 200 us)
python $R/tools/rocprof_summary.py kernel $O/prof "gemm_ps_kernel<0, 64, 0, 1>" 86016 200 | tee $O/wgrad_kernel_trace.txt
python $R/tools/rocprof_summary.py gaps $O/prof embed_fwd_kernel 10 $O/gaps.json | tail -3
python $R/tools/rocprof_summary.py timeline $O/prof 2 $O/stream_timeline.txt | tail -1
if [ "$3" == "pmc" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg \
      > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 $O/pmc_$C.log; exit 1; }
  done
  python $R/tools/rocprof_summary.py traffic $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE "gemm_w4b_kernel<false, 8>" 190464 100 $O/roofline_traffic.json
  python $R/tools/rocprof_summary.py traffic $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE "gemm_ps_kernel<0, 64, 0, 1>" 86016 200 $O/wgrad_traffic.json
  python $R/tools/rocprof_summary.py traffic $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE "gemm_w4b_kernel<true, 6>" 63488 100 $O/dgrad_traffic.json
fi
if [ "$4" == "detail" ]; then
  cd $R && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --detail > $O/detail.json 2> $O/detail.txt || { echo "detail failed"; tail -20 $O/detail.txt; exit 1; }
  grep -v amdgpu.ids $O/detail.txt | head -60
fi
if [ "$5" == "serial" ]; then
  # per-kernel totals with the weight-gradient and predictor streams off (experiments library):
  # the standalone work of the step, free of the in-step CU contention between streams
  cd /tmp && FS2_HIP_LIB=$R/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sprof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg \
    > $O/sprof_bench.json 2> $O/sprof.err || { echo "serial rocprof failed"; tail -20 $O/sprof.err; exit 1; }
  python $R/tools/rocprof_summary.py stats $O/sprof 17 $O/serial_kernel_stats.txt | head -45
fi
