set -o pipefail
mkdir -p gpurun_out/ord
for rep in 1 2 3; do
  for sl in 0 1; do
    timeout -k 10 200 python bench.py --cpu-frames 0 --ate-frames 0 --steps 20 --sgbm-last $sl 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('sgbm_last=$sl', d['value'], d['ms_per_step'])" >> gpurun_out/ord/ab.log || exit 1
  done
done
cat gpurun_out/ord/ab.log
