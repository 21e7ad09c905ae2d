#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes) of the §8f-3 / §8f-4 kernels
# over their throughput tools; summarised by profiles/summarize.py.
#   gpurun -- 'bash tools/pmc_rows.sh <tag>'
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
OUT=$R/gpurun_out/pmc_rows_$TAG
mkdir -p "$OUT/blur" "$OUT/map"
cd /tmp && export TMPDIR=/tmp
for t in blur map; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/f_$t -o f -- python3 "$R/tools/bench_$t.py" > /dev/null 2> "$OUT/$t/fetch.err"
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/w_$t -o w -- python3 "$R/tools/bench_$t.py" > /dev/null 2> "$OUT/$t/write.err"
  python3 "$R/profiles/summarize.py" /tmp/none /tmp/f_$t /tmp/w_$t "$OUT/$t"
  cat "$OUT/$t/pmc_per_kernel.csv"
done
