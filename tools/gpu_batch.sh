#!/bin/bash
# bench at several frames-per-step batch sizes
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for bs in 64 128 192; do
  timeout -k 10 300 python -u "$R/bench.py" --batch $bs --steps 6 --warmup 2 --cpu-frames 0 --ate-frames 0 > "$R/gpurun_out/bench_b$bs.json" 2> "$R/gpurun_out/bench_b$bs.err" || { echo "bench failed"; tail -5 "$R/gpurun_out/bench_b$bs.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['workspace_gb'], d['stages_ms_per_step'])" "$R/gpurun_out/bench_b$bs.json" $bs
done
