# Overlapped-bench A/B of bench.py argument sets (tooling): for each set in $SETS (space-separated,
# commas between arguments), $REPS runs interleaved; extra common arguments in $BENCH_ARGS.
# -> gpurun_out/abargs/ab.log (argument set, frames/s, ms per step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abargs
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
  for a in $SETS; do
    timeout -k 10 300 python bench.py --cpu-frames 0 --ate-frames 0 --steps 20 $BENCH_ARGS $(echo $a | tr ',' ' ') 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$a', d['value'], d['ms_per_step'])" \
      >> gpurun_out/abargs/ab.log || exit 1
  done
done
cat gpurun_out/abargs/ab.log
