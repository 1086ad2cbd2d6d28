#!/bin/bash
# PostNet (tanh-gated) LayerNorm backward microbench on the experiments library, per arm:
# default (exp-based tanh gate), exact tanhf gate, R = 2 rows kernel, both.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for e in "-" "FS2_LN_TANH_EXACT=1" "FS2_LN_TANH_ROWS=1" "FS2_LN_TANH_ROWS=1 FS2_LN_TANH_EXACT=1"; do
  V=(); [ "$e" != "-" ] && V=($e)
  echo "[$e]"
  env FS2_HIP_LIB=$EXP LN_POSTNET=1 "${V[@]}" timeout -k 10 120 python -u tools/ln_bench.py || exit 1
done
