set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "gemm or wgrad or conv" 2>&1 | tail -2
FS2_HIP_LIB=$R/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so timeout -k 10 200 python -u tools/gemm_bench.py wgrad 2>&1 | grep -v amdgpu.ids
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', round(d['ms_per_step'],3))"; done
