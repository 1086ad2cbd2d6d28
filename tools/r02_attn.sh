# GPU: attention parity tests, then A/B of the 32x32 attention kernels vs the 16x16 ones
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-attn} && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fullsize.py tests/test_gpu_model.py -m gpu -k "attention or fullsize or bf16 or attn" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -30
for E in "FS2_ATTN_V1=1" "FS2_ATTN_V1=0"; do
env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json; d=json.load(open('$O/b.json')); print('$E ms/step %.3f' % d['ms_per_step'])"
env $E FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --detail > $O/d.json 2> $O/d.txt || { tail -20 $O/d.txt; exit 1; }
grep attn $O/d.txt
done
