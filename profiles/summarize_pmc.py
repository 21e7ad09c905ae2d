"""Generic per-kernel summary of one rocprofv3 --pmc pass (any counter set) joined with the
same pass's kernel-trace durations -> CSV: kernel, shape, dispatches, avg_ms, avg_<counter>...
plus, when the SQ counters are present, the VALU utilisation:
  valu_util = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction on a SIMD-32) /
              (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (GRBM_GUI_ACTIVE is summed over 8 XCDs)
  i.e. the fraction of the SIMDs' cycles spent issuing vector instructions (1.0 = every
  SIMD issues one wave64 VALU instruction every 2 cycles for the kernel's whole duration).
    usage: python profiles/summarize_pmc.py <rocprof dir> <out.csv> <shape> [kernel-prefix ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def find(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return f[0] if f else None


def short(name):
    m = re.search(r"\b(k_[a-z0-9_]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def main(d, out, shape, prefixes):
    cc = find(d, "*counter_collection.csv")
    kt = find(d, "*kernel_trace.csv")
    dur = {}
    if kt:
        for r in csv.DictReader(open(kt)):
            dur[r.get("Dispatch_Id")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    ctrs = set()
    for r in csv.DictReader(open(cc)):
        k = short(r["Kernel_Name"])
        if prefixes and not any(k.startswith(p) for p in prefixes):
            continue
        c = r["Counter_Name"]
        ctrs.add(c)
        per[k][c] += float(r["Counter_Value"])
        did = r.get("Dispatch_Id")
        if did not in disp[k]:
            disp[k].add(did)
            per[k]["_t"] += dur.get(did, 0.0)
    ctrs = sorted(ctrs)
    cols = ["kernel", "shape", "dispatches", "avg_ms"] + [f"avg_{c}" for c in ctrs] + ["valu_util"]
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        for k, v in sorted(per.items()):
            n = len(disp[k])
            avg = {c: v.get(c, 0.0) / n for c in ctrs}
            gui = avg.get("GRBM_GUI_ACTIVE", 0.0)
            cyc = gui / 8 * 1024 if gui else None
            util = round(avg["SQ_INSTS_VALU"] * 2 / cyc, 4) if cyc and "SQ_INSTS_VALU" in avg else None
            w.writerow([k, shape, n, round(v["_t"] / n * 1e3, 4)] + [round(avg[c], 1) for c in ctrs] + [util])
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:])
