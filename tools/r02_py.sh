# GPU: run one python tool ($1) with args under a time limit, output to gpurun_out/py
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/py
timeout -k 10 300 python -u "$@" > gpurun_out/py/out.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/py/out.txt | tail -60; exit $rc
