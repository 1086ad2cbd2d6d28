# GPU: bf16 padded-domain data gradient + LN backward rows per block -- parity, then A/Bs
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "fold or layernorm or ln_ or four_wave" 2>&1 | tail -2 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_model.py 2>&1 | tail -2 || exit 1
rm -f gpurun_out/ab/log.txt
bash tools/step_ab.sh 2 "-" "FS2_DGRAD_BF16=0" || exit 1
bash tools/ab_lib.sh 3
