#!/bin/bash
# late-parameter AdamW on the aux stream: model / DP tests (graph replay vs eager bit-exact,
# torch AdamW equivalence), then the step A/B (experiments library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 &&
bash tools/ab_env.sh 3 "FS2_ADAM_OVERLAP=0" "FS2_ADAM_OVERLAP=1"
