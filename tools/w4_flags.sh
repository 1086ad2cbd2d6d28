# GPU: the 4-wave GEMM on the FFN conv1 shape with resources removed (experiments build,
# FS2_W4_FLAGS: 1 no barrier, 2 no DMA, 4 no fragment reads; results wrong) -- which one
# bounds a stage.  Usage: bash tools/w4_flags.sh "0 1 2 4 3 5 6 7"
cd $GRAFT_REPO_ROOT
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for f in ${1:-0 1 2 4 3 6 7}; do
  echo "== flags $f"; FS2_HIP_LIB=$EXP FS2_W4_FLAGS=$f GS_ONLY=2,0 timeout -k 10 100 python -u tools/gemm_square.py 2>&1 | grep -v amdgpu.ids || exit 1
done
