# Timing of SGBM library variants (tooling): tools/bench_sgbm.py under FVO_LIB=exp/libfvo_<v>.so for
# each v in $VARIANTS (plus the in-tree library as "tree"), twice each; $SG_ARGS go to bench_sgbm.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgv
export TMPDIR=/tmp
for v in tree ${VARIANTS}; do
  lib=""; [ "$v" = tree ] || lib=exp/libfvo_$v.so
  for rep in 1 2; do
    echo -n "$v $SG_ARGS " >> gpurun_out/sgv/bench.log
    FVO_LIB=$lib timeout -k 10 120 python tools/bench_sgbm.py $SG_ARGS 2>/dev/null | tail -1 >> gpurun_out/sgv/bench.log || exit 1
  done
done
exit 0
