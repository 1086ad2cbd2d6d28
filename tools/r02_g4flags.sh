# GPU: gemm256 main-loop experiments (FS2_G4_FLAGS: 1 no stagger, 2 no setprio, 4 no vmcnt wait, 8 no DMA issue)
cd $GRAFT_REPO_ROOT
for f in 0 256 384; do echo "FS2_G4_FLAGS=$f"; FS2_G4_FLAGS=$f bash tools/r02_py.sh tools/gemm_square.py | grep -v "^$" || exit 1; done
