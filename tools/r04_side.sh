#!/bin/bash
# side-stream persistent-GEMM grid budget A/B (experiments library, same box, interleaved)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export FS2_HIP_LIB=$(pwd)/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for rep in 1 2; do for c in ${CTAS:-256 224 192 160}; do
  FS2_SIDE_CTAS=$c timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('ctas $c', round(d['ms_per_step'],3))" || exit 1
done; done
