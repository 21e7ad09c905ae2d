#!/bin/bash
# rocprofv3 collection for the committed profiles (run on the GPU box via gpurun).
#   pass 1: kernel trace + stats;  passes 2/3: FETCH_SIZE / WRITE_SIZE PMC (separate passes,
#   MI355X_MICROARCH.md §HBM: TCC FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Only summaries of libfvo kernels are kept (the raw traces include the renderer's torch
# kernels and exceed the gpurun copy-back limit).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r1}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-frames 0 --ate-frames 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_trace -o trace -- python3 "$R/bench.py" $ARGS > "$OUT/bench_under_trace.json" 2> "$OUT/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/p_fetch -o fetch -- python3 "$R/bench.py" $ARGS > /dev/null 2> "$OUT/fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/p_write -o write -- python3 "$R/bench.py" $ARGS > /dev/null 2> "$OUT/write.err"
python3 "$R/profiles/summarize.py" /tmp/p_trace /tmp/p_fetch /tmp/p_write "$OUT"
