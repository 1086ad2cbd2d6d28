set -o pipefail
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
echo "== gemm256r plain (FS2_GEMM_NO_PS=1)"; FS2_HIP_LIB=$EXP FS2_GEMM_NO_PS=1 timeout -k 10 200 python -u tools/gemm_square.py 2>&1 | grep -v amdgpu.ids || exit 1
C="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU"
GS_ONLY=2 bash tools/pmc.sh gpmc_ps "" "$C" tools/gemm_square.py || exit 1
FS2_HIP_LIB=$EXP FS2_GEMM_NO_PS=1 GS_ONLY=2 bash tools/pmc.sh gpmc_g4r "" "$C" tools/gemm_square.py || exit 1
