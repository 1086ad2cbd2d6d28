set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "four_wave or gemm_pad or conv1" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k "forward" 2>&1 | tail -3 || exit 1
bash tools/ab_lib.sh 4
