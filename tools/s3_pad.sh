# padded-image conv1 data gradient: op tests, model + full-size parity, then the bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "reversed_taps or padded_image or weight_prep or persistent_short or nan_passes or fwd_padded" 2>&1 | tail -3 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 &&
EXP=$GRAFT_REPO_ROOT/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so &&
for v in 1 0 1 0; do echo "FS2_PAD_FWD=$v"; FS2_HIP_LIB=$EXP FS2_PAD_FWD=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', round(d['ms_per_step'],3), 'host', round(d['host_enqueue_ms_per_step'],2))" || exit 1; done
