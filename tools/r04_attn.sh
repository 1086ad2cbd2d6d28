#!/bin/bash
# fused attention: parity tests (fused vs torch incl. the dropout restatement, materialised path),
# then fwd / bwd timings at the bench shapes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04attn
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "attention or softmax or mask_quirk" 2>&1 | tail -5 &&
timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04attn/attn.txt
