# A/B of one FS2_* switch on gemm_bench call sites and on the bench step (experiments library)
# usage: bash tools/ab_small.sh VAR "filter words" 
set -o pipefail
V=$1; shift
EXP=$GRAFT_REPO_ROOT/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for s in 0 1; do echo "== $V=$s"; env $V=$s timeout -k 10 200 python -u tools/gemm_bench.py $@ 2>&1 | grep -v amdgpu.ids; done
for s in 0 1 0 1; do echo "== step $V=$s"; env FS2_HIP_LIB=$EXP $V=$s timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))"; done
