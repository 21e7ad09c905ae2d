# Overlapped-bench A/B of library variants (tooling): bench.py under FVO_LIB=exp/libfvo_<v>.so for
# each v in $VARIANTS (plus the in-tree library as "tree"), $REPS times each, interleaved; extra
# bench arguments in $BENCH_ARGS.  -> gpurun_out/ablib/ab.log (variant, frames/s, ms per step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablib
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
  for v in tree ${VARIANTS}; do
    lib=""; [ "$v" = tree ] || lib=exp/libfvo_$v.so
    FVO_LIB=$lib timeout -k 10 240 python bench.py --cpu-frames 0 --ate-frames 0 --steps 20 $BENCH_ARGS 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])" \
      >> gpurun_out/ablib/ab.log || exit 1
  done
done
cat gpurun_out/ablib/ab.log
