"""Per-kernel averages of the MFMA PMC pass (tools/mfma_pmc.sh) for the libfvo BA kernels,
joined with the kernel-trace durations of the same pass -> mfma_per_kernel.csv.
MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs), kernel cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back').
F64 MFMA flops = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (MOPS counts 512 math ops)."""
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


def main(d, out, shape):
    cc = find(d, "*counter_collection.csv")
    kt = find(d, "*kernel_trace.csv")
    dur = {}
    if kt:
        for r in csv.DictReader(open(kt)):
            dur[r.get("Dispatch_Id")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(cc)):
        k = short(r["Kernel_Name"])
        if not k.startswith("k_ba_"):
            continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r.get("Dispatch_Id") not in disp[k]:
            disp[k].add(r.get("Dispatch_Id"))
            per[k]["_time_s"] += dur.get(r.get("Dispatch_Id"), 0.0)
    with open(os.path.join(out, "mfma_per_kernel.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "shape", "dispatches", "avg_ms", "avg_MFMA_BUSY_CYCLES", "avg_GRBM_GUI_ACTIVE",
                    "mfma_util", "avg_f64_mfma_flops", "f64_mfma_tflops"])
        for k, v in sorted(per.items()):
            n = len(disp[k])
            t = v["_time_s"] / n if n else 0.0
            busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / n
            gui = v.get("GRBM_GUI_ACTIVE", 0.0) / n
            util = busy / (gui / 8 * 1024) if gui else None
            fl = v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) / n * 512
            w.writerow([k, shape, n, round(t * 1e3, 4), round(busy), round(gui), None if util is None else round(util, 5),
                        round(fl), round(fl / t / 1e12, 3) if t else None])
    print(open(os.path.join(out, "mfma_per_kernel.csv")).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
