# Timing of ORB library variants (tooling): tools/bench_orb.py under FVO_LIB=exp/libfvo_<v>.so for
# each v in $VARIANTS (plus the in-tree library as "tree"), twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/orbv
export TMPDIR=/tmp
for v in tree ${VARIANTS}; do
  lib=""; [ "$v" = tree ] || lib=exp/libfvo_$v.so
  for rep in 1 2; do
    echo -n "$v " >> gpurun_out/orbv/bench.log
    FVO_LIB=$lib timeout -k 10 120 python tools/bench_orb.py 2>/dev/null | tail -1 >> gpurun_out/orbv/bench.log || exit 1
  done
done
exit 0
