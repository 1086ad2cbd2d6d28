# padded conv1 data gradient (1: encoder + decoder, 2: decoder only) A/B (experiments library): step time and the conv1 forward HIP-event averages
set -o pipefail
cd $GRAFT_REPO_ROOT
EXP=$GRAFT_REPO_ROOT/fine-grained-emotional-control-of-tts_amd/fastspeech2/libfs2_hip_exp.so
for v in 1 2 1 2 1 2; do echo "FS2_PAD_DGRAD=$v"; FS2_HIP_LIB=$EXP FS2_PAD_DGRAD=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extractor --no-fp32-leg --no-config2-leg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('step', round(d['ms_per_step'],3), 'fwd dec', round(k['ffn_conv1_fwd.decoder']*1e3,1), 'enc', round(k['ffn_conv1_fwd.encoder']*1e3,1))" || exit 1; done
