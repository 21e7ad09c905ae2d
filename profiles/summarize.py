"""Summarise rocprofv3 CSV output for the libfvo kernels (kernel names from the anonymous
namespace of forest-slam_amd/csrc/*.hip).  Writes kernel_stats.csv (rocprof's own stats,
filtered), pmc_per_kernel.csv (avg FETCH_SIZE / WRITE_SIZE per dispatch, raw and gfx950-
corrected) into the output directory; every row carries the workload shape key (bench.py
shape_key) so counters are never reported for another shape."""
import csv
import glob
import os
import sys
from collections import defaultdict


def find(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return f[0] if f else None


def ours(name):
    return any(k in name for k in ("k_sg_", "k_bf_", "k_pnp", "k_backproject", "k_brief", "k_blur", "k_angle",
                                   "k_harris", "k_select", "k_nms", "k_fast", "k_resize", "k_copy_level0",
                                   "k_row_scan", "k_offsets", "k_ba_", "k_em_", "k_ing_", "k_gather",
                                   "k_mb_", "k_map_", "k_vx_", "rocprim"))


def short(name):
    import re
    m = re.search(r"\b(k_[a-z0-9_]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def main(trace, fetch, write, out, shape):
    os.makedirs(out, exist_ok=True)
    st = find(trace, "*kernel_stats.csv")
    if st:
        rows = list(csv.DictReader(open(st)))
        keep = [r for r in rows if ours(r["Name"])]
        with open(os.path.join(out, "kernel_stats.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) + ["shape"])
            w.writeheader()
            for r in keep:
                r["Name"] = short(r["Name"])
                r["shape"] = shape
                w.writerow(r)
    pmc = defaultdict(lambda: {"FETCH_SIZE": [], "WRITE_SIZE": []})
    for d, ctr in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE")):
        f = find(d, "*counter_collection.csv")
        if not f:
            continue
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == ctr and ours(r["Kernel_Name"]):
                pmc[short(r["Kernel_Name"])][ctr].append(float(r["Counter_Value"]))
    with open(os.path.join(out, "pmc_per_kernel.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "shape", "dispatches", "avg_FETCH_SIZE_kB", "avg_WRITE_SIZE_kB",
                    "hbm_bytes_per_dispatch_corrected"])
        for k, v in sorted(pmc.items()):
            fe = sum(v["FETCH_SIZE"]) / max(len(v["FETCH_SIZE"]), 1)
            wr = sum(v["WRITE_SIZE"]) / max(len(v["WRITE_SIZE"]), 1)
            # gfx950: FETCH_SIZE reports 1/2 of the bytes read -- calibrated for 16-, 12-, 8-, 4- and
            # 2-B-per-lane streaming loads in the row pass's own pattern (tools/fetch_calib.hip,
            # profiles/r6/fetch_calib.csv: factor 0.500 for every width) -- so x2; WRITE_SIZE is taken
            # as is (1.000 for write-back 8-B stores; non-temporal 8-B stores in the cost pass's
            # pattern read 1.68x in the microbenchmark, 1.07x in the cost pass itself); units kB (x1024)
            w.writerow([k, shape, max(len(v["FETCH_SIZE"]), len(v["WRITE_SIZE"])), round(fe, 1), round(wr, 1),
                        int((2 * fe + wr) * 1024)])
    print("summaries written to", out)


if __name__ == "__main__":
    main(*sys.argv[1:6])
