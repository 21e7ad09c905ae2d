#!/bin/bash
# Kernel timeline of the overlapped bench step on the GPU box (tooling only):
#   gpurun -- 'bash tools/gpu_timeline.sh [bench args]'
# -> gpurun_out/tl/timeline.txt (queue busy time, overlap, idle gaps, per-kernel totals over the
#    last 120 ms, i.e. the timed steps).  rocprof output stays in /tmp (a trace exceeds what
#    gpurun copies back).
set -e
root=$(pwd)
mkdir -p gpurun_out/tl
rm -rf /tmp/tl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- \
  python3 "$root/bench.py" --steps 10 --warmup 3 --cpu-frames 0 --ate-frames 0 "$@" > /tmp/tl.out 2>&1
cd "$root"
f=$(find /tmp/tl -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" --last-ms 120 --calls "${TL_CALLS:-k_pnp}" --queue "${TL_QUEUE:-}" > gpurun_out/tl/timeline.txt
grep '^{' /tmp/tl.out > gpurun_out/tl/bench_under_trace.json || true
