#!/bin/bash
# one iteration on the GPU box: every -m gpu test, SGBM alone, then the bench without the CPU/ATE legs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
mkdir -p "$R/gpurun_out"
timeout -k 10 500 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 120 --timeout-method thread > "$R/gpurun_out/gpu_tests_$TAG.log" 2>&1 || { echo "tests failed"; tail -30 "$R/gpurun_out/gpu_tests_$TAG.log"; exit 1; }
tail -1 "$R/gpurun_out/gpu_tests_$TAG.log"
timeout -k 10 120 python -u "$R/tools/bench_sgbm.py" || exit 1
timeout -k 10 300 python -u "$R/bench.py" --steps 10 --warmup 3 --cpu-frames 0 --ate-frames 0 > "$R/gpurun_out/bench_$TAG.json" 2> "$R/gpurun_out/bench_$TAG.err" || { echo "bench failed"; tail -5 "$R/gpurun_out/bench_$TAG.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'])" "$R/gpurun_out/bench_$TAG.json"
