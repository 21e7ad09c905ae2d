set -o pipefail
mkdir -p gpurun_out/abb
rm -f gpurun_out/abb/ab.log
for rep in 1 2; do
  for b in 64 128 96; do
    timeout -k 10 300 python bench.py --cpu-frames 0 --ate-frames 0 --steps 12 --batch $b 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('batch=$b', d['value'], d['ms_per_step'])" >> gpurun_out/abb/ab.log || exit 1
  done
done
cat gpurun_out/abb/ab.log
