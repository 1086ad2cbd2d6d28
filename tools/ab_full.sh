# GPU A/B of kernel-selection env flags: full per-call-site tables (no side stream, so the
# call sites do not share the chip) for each setting ($@ = settings, "-" = defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abf
i=0
for cfg in "$@"; do
  i=$((i+1))
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  echo "== $cfg"
  env FS2_NO_SIDE_STREAM=1 $cfg timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --detail > gpurun_out/abf/d$i.json 2> gpurun_out/abf/d$i.txt || { tail -20 gpurun_out/abf/d$i.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/abf/d$i.txt | head -1
done
