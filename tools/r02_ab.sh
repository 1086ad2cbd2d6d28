# GPU: interleaved A/B of the default bench step under env settings ($@; "-" = defaults), x2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
for rep in 1 2; do
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$cfg: ms/step %.3f  value %.0f' % (d['ms_per_step'], d['value']))"
done
done
