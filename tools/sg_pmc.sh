#!/bin/bash
# SQ counters of the SGBM kernels (standalone SGBM micro-bench), one rocprofv3 pass.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
B=16 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d /tmp/sgpmc -o sq -- python3 "$R/tools/bench_sgbm.py" > "$R/gpurun_out/sgpmc.out" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/sgpmc.out"; exit 1; }
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
f = glob.glob("/tmp/sgpmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_sg" not in k: continue
    import re; k = re.search(r"k_sg_\w+", k).group(0)
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = open(R + "/gpurun_out/sgpmc.csv", "w")
for k, d in acc.items():
    line = k + " " + " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items()))
    print(line); out.write(line + "\n")
PY
