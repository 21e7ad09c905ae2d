#!/usr/bin/env python3
"""Print the BA / PnP rows of rocprofv3 kernel_stats CSVs (tooling): kstats_ba.py DIR"""
import csv
import glob
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*kernel_stats.csv"))):
    print("==", os.path.basename(f))
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "k_ba" in n or "pnp" in n:
            short = n.split("::")[1].split("(")[0]
            print(f"{short:22s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us avg "
                  f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms tot")
