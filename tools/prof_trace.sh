#!/bin/bash
# Quick rocprofv3 kernel-trace summary of the bench (libfvo kernels only) -> gpurun_out/<tag>_stats.csv
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-trace}
shift || true
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt_$TAG -o trace -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-frames 0 --ate-frames 0 "$@" > "$R/gpurun_out/${TAG}_bench.json" 2> "$R/gpurun_out/${TAG}.err"
python3 - "$R" "$TAG" <<'PY'
import csv, glob, os, sys, re
R, tag = sys.argv[1], sys.argv[2]
f = glob.glob(f"/tmp/pt_{tag}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
out = open(os.path.join(R, "gpurun_out", f"{tag}_stats.csv"), "w")
out.write("name,calls,total_ms,avg_us\n")
for r in rows:
    m = re.search(r"\b(k_[a-z0-9_]+)(<[^>(]*>)?", r["Name"])
    if not m:
        continue
    out.write(f"{m.group(0)},{r['Calls']},{float(r['TotalDurationNs'])/1e6:.3f},{float(r['AverageNs'])/1e3:.1f}\n")
PY
cat "$R/gpurun_out/${TAG}_stats.csv" | head -40
