# GPU: tools/ln_bench.py (standalone LayerNorm kernels at the decoder / encoder shapes) on the
# experiments library under each FS2_* setting given ("-" = defaults).
# Usage: bash tools/ln_sweep.sh "-" "FS2_LN_ROWS=2" ...
cd $GRAFT_REPO_ROOT
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for e in "$@"; do
  V=(); [ "$e" != "-" ] && V=($e)
  echo "== [$e]"
  env FS2_HIP_LIB=$EXP LN_VARIANTS=1 "${V[@]}" timeout -k 10 120 python -u tools/ln_bench.py || exit 1
done
