# host enqueue check: model tests, then bench lines (step time, host enqueue, config-2 leg)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 &&
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', round(d['ms_per_step'],3), 'host', round(d['host_enqueue_ms_per_step'],2), 'cfg2', round(d['config2_b16_single_speaker_bf16']['ms_per_step'],3))"; done
