# LayerNorm backward rows per block A/B (experiments library): default 32 / 64 / 128
EXP=$GRAFT_REPO_ROOT/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for r in 0 64 128 0; do echo "== FS2_LN_RPB=$r"; FS2_HIP_LIB=$EXP FS2_LN_RPB=$r LN_VARIANTS=1 timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids | grep "31264"; done
for g in 0 1 0 1; do echo "== FS2_GRAPH=$g"; FS2_GRAPH=$g timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('hip_graph'), round(d.get('host_enqueue_ms_per_step') or -1, 2))"; done
