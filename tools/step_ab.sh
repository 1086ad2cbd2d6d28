# GPU: interleaved bench-step A/B runs on the experiments library.
# Usage: bash tools/step_ab.sh ROUNDS "ENV_A" "ENV_B" ["ENV_C" ...]   (ENV "-" = no variables)
# Prints ms/step per arm per round, then each arm's median.
cd $GRAFT_REPO_ROOT
EXP=$PWD/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
R=$1; shift
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/log.txt
ARMS=("$@")
NA=${#ARMS[@]}
for r in $(seq 1 $R); do
  # rotate the starting arm each round (the first run of a round measured consistently slower)
  for k in $(seq 0 $((NA - 1))); do
    i=$(( (k + r - 1) % NA ))
    e=${ARMS[$i]}
    V=(); [ "$e" != "-" ] && V=($e)
    env FS2_HIP_LIB=$EXP "${V[@]}" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
    ms=$(python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print(' '.join('%s=%.1f' % (k.split('.')[0][9:] + k.split('.')[1][:3], v * 1e3) for k, v in d.get('kernel_ms', {}).items()), d['ms_per_step'])")
    echo "$r arm$i [$e] $ms" | tee -a gpurun_out/ab/log.txt
  done
done
python - "$@" <<'PY'
import sys, statistics, collections
d = collections.defaultdict(list)
for line in open("gpurun_out/ab/log.txt"):
    p = line.split()
    d[p[1]].append(float(p[-1]))
for k in sorted(d):
    print(k, sys.argv[1 + int(k[3:])], "median %.3f" % statistics.median(d[k]), d[k])
PY
