# same-box A/B of the product library: this tree, the tree without the padded forward
# (scratch/nofwd), without both padded convs (scratch/nopad), and the session start (scratch/old)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { (cd $1 && timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('step', round(d['ms_per_step'],3), 'fwd dec', round(k['ffn_conv1_fwd.decoder']*1e3,1), 'enc', round(k['ffn_conv1_fwd.encoder']*1e3,1))"); }
for i in 1 2 3; do for t in . scratch/nofwd scratch/nopad scratch/old; do echo "$t"; run $t || exit 1; done; done
