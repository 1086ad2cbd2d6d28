set -o pipefail
mkdir -p gpurun_out/attn
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
FS2_HIP_LIB=$EXP FS2_ATTN_STG=0 timeout -k 10 120 python -u tools/attn_ab.py gpurun_out/attn/a0.npz 2>&1 | grep -v amdgpu.ids
FS2_HIP_LIB=$EXP FS2_ATTN_STG=1 timeout -k 10 120 python -u tools/attn_ab.py gpurun_out/attn/a1.npz 2>&1 | grep -v amdgpu.ids
python tools/attn_ab.py --cmp gpurun_out/attn/a0.npz gpurun_out/attn/a1.npz
for s in 0 1 0 1; do echo "STG=$s"; FS2_HIP_LIB=$EXP FS2_ATTN_STG=$s timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | head -2; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "attention" 2>&1 | tail -2
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "kmajor or colsum" 2>&1 | tail -2
