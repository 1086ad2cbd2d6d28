# GPU: run a python tool ($1) under several env settings (rest; "-" = defaults)
cd $GRAFT_REPO_ROOT
T=$1; shift
for e in "$@"; do [ "$e" == "-" ] && e="FS2_AB_DEFAULT=1"; echo "== $e"; env $e bash tools/r02_py.sh $T | grep -v "^$" || exit 1; done
