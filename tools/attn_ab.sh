#!/bin/bash
# attention kernels: parity tests, then standalone timings of the product library and of the
# experiments library under FS2_ATTN_FLAGS variants.  Usage: bash tools/attn_ab.sh "FLAGS ..."
cd ${GRAFT_REPO_ROOT:-$(pwd)}
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "attention" 2>&1 | tail -2 || exit 1
echo "== product"; timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
for f in $1; do
  echo "== FS2_ATTN_FLAGS=$f"; FS2_HIP_LIB=$EXP FS2_ATTN_FLAGS=$f timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
