#!/bin/bash
# SGBM batch chunks over two streams (cost pass of one chunk beside the row pass of the other)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for c in 1 2 4 1 2 4; do
  FVO_SG_CHUNKS=$c timeout -k 10 120 python -u "$R/tools/bench_sgbm.py" || { echo "bench_sgbm failed"; exit 1; }
done
for c in 1 2; do
  FVO_SG_CHUNKS=$c timeout -k 10 300 python -u "$R/bench.py" --steps 10 --warmup 3 --cpu-frames 0 --ate-frames 0 > "$R/gpurun_out/bench_ch$c.json" 2> "$R/gpurun_out/bench_ch$c.err" || { echo "bench failed"; tail -5 "$R/gpurun_out/bench_ch$c.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$R/gpurun_out/bench_ch$c.json" $c
done
