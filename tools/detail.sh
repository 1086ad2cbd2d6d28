# Serial per-call-site times (bench.py --detail) with the weight-gradient and predictor streams
# off: needs the experiments library (make -C fine-grained-emotional-control-of-tts_amd/csrc
# experiments), whose FS2_* switches the product library compiles out.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/det
export FS2_HIP_LIB=$GRAFT_REPO_ROOT/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
FS2_NO_SIDE_STREAM=1 FS2_NO_AUX_STREAM=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg --detail > gpurun_out/det/detail.json 2> gpurun_out/det/detail.txt || { tail -20 gpurun_out/det/detail.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/det/detail.txt | head -80
