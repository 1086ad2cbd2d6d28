# GPU: serial (no side / aux stream) per-call-site detail + PMC passes for the kernels below roofline
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-iso} && mkdir -p $O
FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --detail > $O/detail.json 2> $O/detail.txt || { tail -20 $O/detail.txt; exit 1; }
grep -v amdgpu.ids $O/detail.txt | head -60
python -c "import json; d=json.load(open('$O/detail.json')); print('serial ms/step %.3f' % d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py stats $GRAFT_REPO_ROOT/$O/prof 13 $GRAFT_REPO_ROOT/$O/kernel_stats.txt | head -45
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"; do
  i=$((i+1))
  FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc$i -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg > $GRAFT_REPO_ROOT/$O/pmc$i.log 2>&1 || { echo "pmc $C failed"; tail -20 $GRAFT_REPO_ROOT/$O/pmc$i.log; exit 1; }
done
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py pmc $GRAFT_REPO_ROOT/$O/pmc.json "attn_,gemm_big_kernel<true, true, 0, 0>,gemm256_kernel<true, true, 1,ln_bwd_rows,gemm256_kernel<false, false, 0, 0>" $GRAFT_REPO_ROOT/$O/pmc1 $GRAFT_REPO_ROOT/$O/pmc2 $GRAFT_REPO_ROOT/$O/pmc3 $GRAFT_REPO_ROOT/$O/pmc4 | head -40
