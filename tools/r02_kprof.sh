# GPU: rocprofv3 kernel stats of one python tool ($1) -> gpurun_out/kprof/stats.txt
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/kprof && rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python $GRAFT_REPO_ROOT/$1 > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob('/root/repo/gpurun_out/kprof/**/run_kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:16]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us avg {int(r['Calls']):6d} calls  {r['Name'][:110]}")
PY
