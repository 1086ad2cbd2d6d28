# GPU: kernel names + durations hipBLASLt picks for the square / conv-shaped GEMMs (tools/gemm_square.py)
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/blas && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python $GRAFT_REPO_ROOT/tools/gemm_square.py > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob('/root/repo/gpurun_out/blas/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:200], r['Calls'], r['AverageNs'])
PY
