# BA timing of library variants (tooling): tools/bench_ba.py (600p, and 1080p with HD=1) under
# FVO_LIB=exp/libfvo_<v>.so for each v in $VARIANTS (plus the in-tree library), twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bav
export TMPDIR=/tmp
for v in tree ${VARIANTS}; do
  lib=""; [ "$v" = tree ] || lib=exp/libfvo_$v.so
  for rep in 1 2; do
    for flag in "" ${HD:+--hd}; do
      echo -n "$v $flag " >> gpurun_out/bav/bench.log
      FVO_LIB=$lib timeout -k 10 150 python tools/bench_ba.py $flag 2>/dev/null | tail -1 >> gpurun_out/bav/bench.log || exit 1
    done
  done
done
exit 0
