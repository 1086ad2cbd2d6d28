# GPU: per-call-site timing under alternative kernel-selection env flags
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/env
for cfg in "BASE=1" "FS2_GEMM_NO256=1" "FS2_GEMM_NO_BIG=1 FS2_GEMM_NO256=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --detail > gpurun_out/env/d.json 2> gpurun_out/env/d.txt || { tail -20 gpurun_out/env/d.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/env/d.txt | head -32
done
