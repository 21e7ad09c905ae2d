"""Per-queue chain of the BA kernels in the last step of a rocprofv3 kernel trace (tooling):
each kernel's start / duration relative to the step's first BA kernel and the gap before it.
    python tools/ba_chain.py gpurun_out/bachain/ba_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id") or r.get("Queue_Id"), n))
    rows.sort()
    # the last step: from the last k_ba_build / k_ba_births-like first kernel of the step
    starts = [i for i, r in enumerate(rows) if r[3].startswith("k_ba_stereo")]
    rows = rows[starts[-1]:] if starts else rows
    t0 = rows[0][0]
    last = defaultdict(lambda: None)
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, q, n in rows:
        gap = (s - last[q]) / 1e3 if last[q] is not None else 0.0
        print(f"q{q:>3} {n:<22} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}")
        last[q] = e
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
    print(f"span {(max(r[1] for r in rows) - t0) / 1e3:.1f} us")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:<22} {c:4d} calls {t:9.1f} us")


if __name__ == "__main__":
    main()
