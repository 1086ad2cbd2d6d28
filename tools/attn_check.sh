# GPU: fused attention parity tests + per-call-site timing (bench --detail)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/attn
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn/pytest.log 2>&1 || { tail -30 gpurun_out/attn/pytest.log; exit 1; }
tail -2 gpurun_out/attn/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --detail > gpurun_out/attn/detail.json 2> gpurun_out/attn/detail.txt || { tail -20 gpurun_out/attn/detail.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/attn/detail.txt | head -14
python -c "import json; d=json.load(open('gpurun_out/attn/detail.json')); print('ms/step', d['ms_per_step'])"
