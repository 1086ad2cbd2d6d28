set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "embedding or rowdot or add3 or concat" 2>&1 | tail -2
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', round(d['ms_per_step'],3))"; done
