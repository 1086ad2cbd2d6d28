#!/bin/bash
# side-stream persistent-GEMM grid budget / CU mask A/B (experiments library, same box, interleaved)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export FS2_HIP_LIB=$(pwd)/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for rep in 1 2; do for c in ${CTAS:-256 224 192 160}; do for m in ${MASKS:-1}; do
  FS2_SIDE_CUMASK=$m FS2_SIDE_CTAS=$c timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null > /tmp/side_$c_$m.json || exit 1
  python -c "import json; d=json.load(open('/tmp/side_$c_$m.json')); print('ctas $c mask $m', round(d['ms_per_step'], 3))" || exit 1
done; done; done
