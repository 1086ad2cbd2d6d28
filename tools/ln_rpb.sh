# LayerNorm backward rows per block A/B (experiments library): default 32 / 64 / 128
EXP=$GRAFT_REPO_ROOT/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for r in 0 64 128 0; do echo "== FS2_LN_RPB=$r"; FS2_HIP_LIB=$EXP FS2_LN_RPB=$r LN_VARIANTS=1 timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids | grep "31264"; done
