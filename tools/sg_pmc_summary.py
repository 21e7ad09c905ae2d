#!/usr/bin/env python3
"""Summarise the SQ counters of gpurun_out/sgpmc/<mode>/pmc_counter_collection.csv per SGBM kernel
(tools/gpu_sgbm_pmc.sh): VALU / LDS instructions per dispatch, VALU utilisation, wait fractions."""
import collections
import csv
import re
import sys

for m in sys.argv[1:] or ["classic"]:
    rows = list(csv.DictReader(open(f"gpurun_out/sgpmc/{m}/pmc_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in rows:
        k = re.search(r"k_sg_\w+(<[^>]*>)?", r["Kernel_Name"]).group(0)
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            cnt[k] += 1
    for k, v in agg.items():
        n = cnt[k]
        g = v["GRBM_GUI_ACTIVE"] / n / 8
        print(f"{m} {k}: VALU/disp {v['SQ_INSTS_VALU'] / n:.3g}  LDS/disp {v['SQ_INSTS_LDS'] / n:.3g}  "
              f"valu_util {v['SQ_INSTS_VALU'] / n * 2 / (1024 * g):.3f}  wait_any {v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']:.2f}  "
              f"wait_inst {v['SQ_WAIT_INST_ANY'] / v['SQ_WAVE_CYCLES']:.2f}  cycles {g:.3g}")
