#!/bin/bash
# rocprofv3 kernel stats for the §8f-3 / §8f-4 kernels (motion blur, map transform, voxel
# downsample incl. hipcub's radix sort / scan) over their throughput tools.
#   gpurun -- 'bash tools/prof_rows.sh <tag>'
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
OUT=$R/gpurun_out/prof_rows_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_blur -o blur -- python3 "$R/tools/bench_blur.py" > "$OUT/bench_blur.jsonl"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_map -o map -- python3 "$R/tools/bench_map.py" > "$OUT/bench_map.jsonl"
mkdir -p "$OUT/blur" "$OUT/map"
python3 "$R/profiles/summarize.py" /tmp/p_blur /tmp/none /tmp/none "$OUT/blur"
python3 "$R/profiles/summarize.py" /tmp/p_map /tmp/none /tmp/none "$OUT/map"
cat "$OUT/blur/kernel_stats.csv" "$OUT/map/kernel_stats.csv"
