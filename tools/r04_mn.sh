#!/bin/bash
# MN-major GEMMs without the compiler's DMA-ring drain: GEMM parity, 1x1 weight-gradient timings, bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04mn
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3 && timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 300 python -u tools/wgrad1x1_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04mn/wgrad1x1.txt &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > gpurun_out/r04mn/bench.json 2> gpurun_out/r04mn/bench.err && python -c "
import json; d=json.load(open('gpurun_out/r04mn/bench.json')); print('bench', d['ms_per_step'], d['value'])"
