# GPU: 4-wave GEMM parity tests, GEMM shapes against hipBLASLt (w4 on / off), PMC of the w4
# kernel on the FFN conv1 shape.  Usage: bash tools/w4_check.sh [pytest -k expr] [ab]
cd $GRAFT_REPO_ROOT && O=gpurun_out/w4 && mkdir -p $O
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
timeout -k 10 300 python -u -m pytest tests -m gpu -k "${1:-four_wave or persistent_long_k}" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo "== w4 (product)"; timeout -k 10 200 python -u tools/gemm_square.py 2>&1 | grep -v amdgpu.ids || exit 1
if [ -n "$2" ]; then echo "== $2"; FS2_HIP_LIB=$EXP env $2 timeout -k 10 200 python -u tools/gemm_square.py 2>&1 | grep -v amdgpu.ids || exit 1; fi
C="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU"
GS_ONLY=2 bash tools/pmc.sh w4pmc "w4" "$C" tools/gemm_square.py || exit 1
