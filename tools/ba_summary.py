#!/usr/bin/env python3
"""Summarise a tools/gpu_ba_check.sh run (tooling): BA stage times, per-kernel BA stats, bench line."""
import csv
import json
import os
import re
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ba"
for f in ("bench600.log", "bench1080.log"):
    p = os.path.join(D, f)
    if os.path.exists(p):
        print(f, [ln.strip() for ln in open(p) if ln.startswith("{")][-1:])
for sh in (600, 1080):
    p = os.path.join(D, f"kstats_{sh}.csv")
    if not os.path.exists(p):
        continue
    print("==", sh)
    for r in csv.DictReader(open(p)):
        m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", r["Name"])
        if m and ("k_ba" in m.group(1) or "k_sg" in m.group(1)):
            print(f"{m.group(1):28s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us "
                  f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms")
p = os.path.join(D, "bench_full.log")
if os.path.exists(p):
    j = json.loads([ln for ln in open(p) if ln.startswith("{")][-1])
    print("bench", j["value"], j["ms_per_step"], {k: v for k, v in list(j["stages_ms_per_step"].items())[:6]})
