"""Timeline of a rocprofv3 --kernel-trace CSV: how much the streams overlap and where the GPU idles.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o tl -- python3 bench.py ...
    python tools/timeline.py gpurun_out/tl/.../tl_kernel_trace.csv [--last-ms 200]

Reports, over the last --last-ms of the trace (the timed steps): the span, the time at least one
kernel runs (busy union), the time kernels of two or more queues run together, per-queue busy
time, and the longest idle gaps with the kernels either side.  Tooling only."""
import argparse
import csv
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, n.split("(")[0][:48]))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-ms", type=float, default=200.0)
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    rows = load(a.csv)
    t_end = max(r[1] for r in rows)
    t0 = t_end - int(a.last_ms * 1e6)
    rows = [r for r in rows if r[0] >= t0]
    span = t_end - rows[0][0]
    busy = union([(s, e) for s, e, _, _ in rows])
    per_q = defaultdict(list)
    for s, e, q, _ in rows:
        per_q[q].append((s, e))
    qb = {q: union(v) for q, v in per_q.items()}
    both = sum(qb.values()) - busy  # exact for two queues
    print(f"window {span / 1e6:.2f} ms, kernels {len(rows)}, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%)")
    for q, b in sorted(qb.items()):
        names = defaultdict(int)
        for s, e, qq, n in rows:
            if qq == q:
                names[n] += e - s
        top = ", ".join(f"{k} {v / 1e6:.1f}" for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:6])
        print(f"queue {q}: busy {b / 1e6:.2f} ms  [{top}]")
    print(f"overlap (>=2 queues busy, 2-queue estimate): {both / 1e6:.2f} ms")
    gaps = []
    end = rows[0][1]
    prev = rows[0]
    for r in rows[1:]:
        if r[0] > end:
            gaps.append((r[0] - end, prev[3], r[3]))
        if r[1] > end:
            end, prev = r[1], r
    gaps.sort(reverse=True)
    print(f"idle total {sum(g[0] for g in gaps) / 1e6:.2f} ms in {len(gaps)} gaps; longest:")
    for g, p, n in gaps[:a.gaps]:
        print(f"  {g / 1e3:8.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()
