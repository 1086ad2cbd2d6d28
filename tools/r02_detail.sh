# GPU: per-call-site detail (serial streams) under env settings ($1, "-" = defaults), output tag $2
cd $GRAFT_REPO_ROOT && O=gpurun_out/${2:-detail} && mkdir -p $O
cfg="$1"; [ "$cfg" == "-" ] && cfg="FS2_AB_DEFAULT=1"
env $cfg FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --detail > $O/detail.json 2> $O/detail.txt || { tail -20 $O/detail.txt; exit 1; }
grep -v amdgpu.ids $O/detail.txt | head -${3:-24}
