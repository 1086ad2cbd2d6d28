# GPU: every fs2_gemm call site of a short bench run (FS2_GEMM_TRACE=1), largest first.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sites
FS2_GEMM_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --no-graph > gpurun_out/sites/b.json 2> gpurun_out/sites/err.log || { tail -20 gpurun_out/sites/err.log; exit 1; }
grep "^gemm" gpurun_out/sites/err.log > gpurun_out/sites/sites.txt; head -70 gpurun_out/sites/sites.txt
