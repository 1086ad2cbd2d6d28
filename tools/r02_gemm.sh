# GPU: GEMM call-site microbench under env variants ($@; "-" = defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gemm
for cfg in "$@"; do
  [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/gemm/g.txt 2>&1 || { tail -20 gpurun_out/gemm/g.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/gemm/g.txt
done
