#!/bin/bash
# in-order per-kernel times of a tool script: rocprofv3 kernel trace + stats
#   gpurun -- 'bash tools/gpu_ktrace.sh <tag> tools/bench_ba.py'
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/kt_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$TAG -o kt -- python3 "$R/$1" > "$OUT/cmd.out" 2> "$OUT/cmd.err" || { echo "trace failed"; tail -5 "$OUT/cmd.err"; exit 1; }
f=$(find /tmp/kt_$TAG -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/kernel_stats.csv"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    n = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:60]
    print(f"{n:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e6:8.3f} ms")
PY
