#!/bin/bash
# Per-kernel stats of one tool run on the GPU box (tooling):
#   gpurun -- 'bash tools/gpu_kstats.sh <tag> <script.py> [args...]'
# -> gpurun_out/ks_<tag>/{kernel_stats.csv,run.out}.  rocprof output stays in /tmp.
set -uo pipefail
R=$(pwd); TAG=$1; shift
OUT=$R/gpurun_out/ks_$TAG; mkdir -p "$OUT"; rm -rf /tmp/ks_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks_$TAG -o run -- python3 "$R/$1" "${@:2}" > "$OUT/run.out" 2>&1 || { tail -5 "$OUT/run.out"; exit 1; }
find /tmp/ks_$TAG -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
# per-call listing of the kernels matching $KS_CALLS over the trace's last $KS_MS ms
if [ -n "${KS_CALLS:-}" ]; then
  f=$(find /tmp/ks_$TAG -name "*kernel_trace.csv" | head -1)
  python3 "$R/tools/timeline.py" "$f" --last-ms "${KS_MS:-50}" --calls "$KS_CALLS" --kernels 0 --gaps 0 > "$OUT/calls.txt" || true
fi
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "anonymous namespace" in r["Name"]]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
    print(f"{n:40s} {int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['AverageNs']) / 1e3:9.1f} us")
PY
