#!/usr/bin/env python3
"""Merge one collect.sh run (gpurun_out/prof_<tag>/) into a committed profile directory:
for each summary CSV, the rows of the run's shape replace that shape's rows, rows of other
shapes are kept.  Usage: tools/merge_profiles.py gpurun_out/prof_<tag> profiles/r2"""
import csv
import os
import shutil
import sys

FILES = ("kernel_stats.csv", "pmc_per_kernel.csv", "valu_per_kernel.csv", "mfma_per_kernel.csv")


def read(path):
    with open(path, newline="") as f:
        r = csv.DictReader(f)
        return r.fieldnames, list(r)


def main(src, dst):
    for name in FILES:
        s = os.path.join(src, name)
        if not os.path.exists(s):
            print(f"skip {name}: not in {src}")
            continue
        fields, rows = read(s)
        shapes = {r["shape"] for r in rows}
        d = os.path.join(dst, name)
        kept = []
        if os.path.exists(d):
            dfields, drows = read(d)
            if dfields != fields:
                raise SystemExit(f"{name}: columns differ between {s} and {d}")
            kept = [r for r in drows if r["shape"] not in shapes]
        with open(d, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=fields)
            w.writeheader()
            w.writerows(rows + kept)
        print(f"{name}: {len(rows)} rows of {sorted(shapes)} + {len(kept)} kept")
    # the bench line that ran under the trace pass; one file per shape (a 1080p run must not
    # overwrite the 600p one): bench_under_trace.json for the headline shape, else _1080p etc.
    b = os.path.join(src, "bench_under_trace.json")
    if os.path.exists(b):
        shapes = set()
        with open(os.path.join(src, "kernel_stats.csv"), newline="") as f:
            shapes = {r["shape"] for r in csv.DictReader(f)}
        name = "bench_under_trace.json"
        if any(sh.startswith("1920x1080") for sh in shapes):
            name = "bench_under_trace_1080p.json"
        shutil.copy(b, os.path.join(dst, name))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
