# GPU: memory-path counters of the 4-wave GEMM vs hipBLASLt on the FFN conv1 shape.
cd $GRAFT_REPO_ROOT
GS_ONLY=2 bash tools/pmc.sh w4pmc2 "w4b,Cijk" "GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max TCC_HIT_sum TCC_MISS_sum" tools/gemm_square.py || exit 1
GS_ONLY=2 bash tools/pmc.sh w4pmc3 "w4b,Cijk" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES" tools/gemm_square.py || exit 1
