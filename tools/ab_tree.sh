#!/bin/bash
# same-box product-library A/B: tree A = this tree with the files under ab_base/ put back
# (the baseline), tree B = this tree; interleaved bench runs, ms/step of each printed
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd); REPS=${1:-3}
A=/tmp/ab_A; rm -rf $A; mkdir -p $A
tar --exclude=./gpurun_out --exclude=./ab_base -cf - . | tar -xf - -C $A
(cd ab_base && tar -cf - .) | tar -xf - -C $A
BA="--no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg"
for i in $(seq $REPS); do
  for t in A B; do
    d=$R; [ $t = A ] && d=$A
    (cd $d && timeout -k 10 200 python -u bench.py $BA 2>/dev/null > /tmp/ab_$t.json) || exit 1
    python -c "import json; d=json.load(open('/tmp/ab_$t.json')); print('$t', round(d['ms_per_step'], 3), 'host', round(d.get('host_enqueue_ms_per_step', 0), 2))"
  done
done
