#!/bin/bash
# gate / residual persistent instance: parity, then 256x192 (FS2_PS_EO_W=48) vs 256x128 timings
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "persistent or padded or gemm or conv" 2>&1 | tail -2 &&
export FS2_HIP_LIB=$(pwd)/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so &&
for w in 48 32 48 32; do echo "EO_W $w"; FS2_PS_EO_W=$w timeout -k 10 120 python -u tools/pk_bench.py 2>&1 | grep -E "gate|resid" || exit 1; done &&
for w in 48 32 48 32; do FS2_PS_EO_W=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null > /tmp/eo.json || exit 1; python -c "import json; d=json.load(open('/tmp/eo.json')); print('bench EO_W $w', round(d['ms_per_step'], 3))"; done
