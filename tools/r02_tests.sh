# GPU: selected tests ($1 = pytest -k expression or "all"; $2 = files) then the default bench line
cd $GRAFT_REPO_ROOT && O=gpurun_out/${3:-tests} && mkdir -p $O
if [ "$1" == "all" ]; then K=(); else K=(-k "$1"); fi
timeout -k 10 900 python -u -m pytest ${2:-tests} -m gpu "${K[@]}" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -40
if [ "$4" != "nobench" ]; then
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps({k: d[k] for k in ('ms_per_step','value','roofline','cpu_baseline','fp32','config2_b16_single_speaker_bf16','host_enqueue_ms_per_step') if k in d}))"
fi
