# model / full-size parity with the cached padded images, then the padded-dgrad A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "padded or reversed" 2>&1 | tail -2 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 &&
bash tools/s3_fwd_ab.sh
