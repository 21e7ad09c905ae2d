"""Join tools/fetch_calib's byte counts with its FETCH_SIZE / WRITE_SIZE passes:
    python tools/fetch_calib_summary.py run.jsonl <fetch dir> <write dir> out.csv
factor = counter bytes per dispatch (kB x 1024) / bytes the pattern moves; the SGBM traffic
correction in profiles/summarize.py applies 1 / factor per kernel (its load width)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = {"b128": "k_cal_b128", "b32": "k_cal_b32", "b96v": "k_cal_rows<3, false>", "b96vp": "k_cal_rows<3, true>",
          "b64v": "k_cal_rows<2, false>", "b16m": "k_cal_b16m", "st64": "k_cal_st64",
          "st64t": "k_cal_st64t<false>", "st128": "k_cal_st128"}


def counters(d, name):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    if not f:
        return per
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == name:
            k = r["Kernel_Name"]
            for pat, kn in KERNEL.items():
                if kn.replace(" ", "") + "(" in k.replace(" ", ""):
                    per[pat].append(float(r["Counter_Value"]) * 1024)
    return per


def main(run, fdir, wdir, out):
    rows = [json.loads(l) for l in open(run) if l.startswith("{")]
    fe, wr = counters(fdir, "FETCH_SIZE"), counters(wdir, "WRITE_SIZE")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["pattern", "kernel", "bytes", "ms", "GB/s", "FETCH_SIZE_bytes", "fetch_factor",
                    "WRITE_SIZE_bytes", "write_factor"])
        for r in rows:
            p = r["pattern"]
            fb = sum(fe[p]) / len(fe[p]) if fe[p] else 0.0
            wb = sum(wr[p]) / len(wr[p]) if wr[p] else 0.0
            w.writerow([p, KERNEL[p], int(r["bytes"]), r["ms"], r["gbs"], int(fb), round(fb / r["bytes"], 4),
                        int(wb), round(wb / r["bytes"], 4)])
    print(open(out).read())


if __name__ == "__main__":
    main(*sys.argv[1:5])
