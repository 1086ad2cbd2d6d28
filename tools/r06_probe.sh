# GPU probe batch (round 6): attention PMC, serial per-call-site detail, LayerNorm rows-per-block
# sweep (standalone + step, experiments library)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/det
bash tools/detail.sh > gpurun_out/det/summary.txt || exit 1
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for r in 0 24 41 48 64; do
  echo "FS2_LN_RPB=$r"
  FS2_HIP_LIB=$EXP FS2_LN_RPB=$r timeout -k 10 120 python -u tools/ln_bench.py || exit 1
done
rm -f gpurun_out/ab/log.txt
bash tools/step_ab.sh 2 "-" "FS2_LN_RPB=41" "FS2_LN_RPB=24"
