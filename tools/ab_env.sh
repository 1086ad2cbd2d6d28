# GPU A/B of kernel-selection env flags: per-call-site timing for each setting ($@ = settings)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --detail > gpurun_out/ab/d.json 2> gpurun_out/ab/d.txt || { tail -20 gpurun_out/ab/d.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab/d.txt | grep -E "detail|pos_ffn.0.conv.weight:T977|pos_ffn.0.conv.weight:T200" | head -8
done
