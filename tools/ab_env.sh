#!/bin/bash
# interleaved bench runs of the experiments library under env-variable variants:
#   bash tools/ab_env.sh REPS "VAR=1 VAR2=0" "VAR=0" ...   (ms/step per variant and rep)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=$1; shift
export FS2_HIP_LIB=$(pwd)/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
BA="--no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg"
for i in $(seq $REPS); do
  for v in "$@"; do
    env $v timeout -k 10 200 python -u bench.py $BA 2>/dev/null > /tmp/ab_env.json || exit 1
    python -c "import json; d=json.load(open('/tmp/ab_env.json')); print('[$v]', round(d['ms_per_step'], 3))"
  done
done
