# GPU: run a python tool under several flag values ($1 = tool, rest = values) set as both
# FS2_G4_FLAGS and FS2_PS_FLAGS (the 256x256 and persistent kernels' timing switches)
cd $GRAFT_REPO_ROOT
T=$1; shift
for f in "$@"; do echo "flags=$f"; FS2_PS_FLAGS=$f FS2_G4_FLAGS=$f bash tools/r02_py.sh $T | grep -v "^$" || exit 1; done
