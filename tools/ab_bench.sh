# GPU A/B of whole-step bench time for env settings ($@; "-" = defaults), interleaved twice
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abb
for rep in 1 2; do
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extractor > gpurun_out/abb/b.json 2> gpurun_out/abb/b.err || { tail -20 gpurun_out/abb/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abb/b.json')); print('$cfg: ms/step %.3f  value %.0f' % (d['ms_per_step'], d['value']))"
done
done
