#!/bin/bash
# In-order kernel trace of the default bench (no stream overlap): per-kernel durations
# without another stream's kernels sharing the CUs.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/inorder"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_io -o io -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-frames 0 --ate-frames 0 --overlap-sgbm 0 > "$R/gpurun_out/inorder/bench.json" 2> "$R/gpurun_out/inorder/bench.err" || { tail -5 "$R/gpurun_out/inorder/bench.err"; exit 1; }
f=$(find /tmp/p_io -name "*kernel_stats.csv" | head -1)
cp "$f" "$R/gpurun_out/inorder/kernel_stats.csv"
python3 "$R/tools/kstats.py" "$R/gpurun_out/inorder/kernel_stats.csv" k_ | head -40
