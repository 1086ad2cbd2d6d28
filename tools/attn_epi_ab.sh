# GPU: attention output-store pairing -- parity, standalone timing, then step A/B of the product
# library against libfs2_hip_base.so; and the 4-wave min-K sweep on the experiments library
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "fused_attention" 2>&1 | tail -2 || exit 1
timeout -k 10 120 python -u tools/attn_bench.py || exit 1
FS2_HIP_LIB=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_base.so timeout -k 10 120 python -u tools/attn_bench.py || exit 1
bash tools/ab_lib.sh 3 || exit 1
rm -f gpurun_out/ab/log.txt
bash tools/step_ab.sh 2 "-" "FS2_W4_MIN_K=1024" "FS2_W4_MIN_K=384" "FS2_W4_MIN_K=384 FS2_W4_MIN_TILES=100"
