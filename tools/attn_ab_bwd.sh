# GPU: fused attention backward variants (experiments library, FS2_ATTN_BWD bits): bit-exactness
# against the default kernels, the torch parity test, then timing at the bench shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export FS2_HIP_LIB=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
V=${1:-4}
ATTN_VARIANT=$V timeout -k 10 120 python -u tools/attn_exact.py || exit 1
FS2_ATTN_BWD=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "fused_attention" 2>&1 | tail -3
for v in 0 $V; do
  echo "FS2_ATTN_BWD=$v"
  FS2_ATTN_BWD=$v timeout -k 10 120 python -u tools/attn_bench.py || exit 1
done
