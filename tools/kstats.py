"""Per-kernel average durations from a rocprofv3 --stats CSV (tooling only).

    python tools/kstats.py gpurun_out/x/.../x_kernel_stats.csv [substring ...]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if len(sys.argv) > 2 and not any(s in n for s in sys.argv[2:]):
        continue
    rows.append((float(r["TotalDurationNs"]), n, int(r["Calls"]), float(r["AverageNs"])))
for tot, n, c, avg in sorted(rows, reverse=True):
    print(f"{n[:44]:44s} calls {c:5d}  avg {avg / 1e3:9.1f} us  total {tot / 1e6:8.3f} ms")
