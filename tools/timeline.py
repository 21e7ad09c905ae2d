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
    ap.add_argument("--kernels", type=int, default=40, help="per-kernel totals over the window (0: none)")
    ap.add_argument("--calls", default="", help="substring: list each call of matching kernels in the last 2 windows/10")
    ap.add_argument("--queue", default="", help="with --calls: only this queue's calls")
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
        top = ", ".join(f"{k} {v / 1e6:.1f}" for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:12])
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
    if a.calls:
        calls(rows, a.calls, int(a.last_ms * 1e6 / 5), a.queue)
    if a.kernels:
        tot = defaultdict(lambda: [0, 0])
        for s, e, _, n in rows:
            tot[n][0] += e - s
            tot[n][1] += 1
        print("kernel                                            calls    total     per call")
        for n, (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:a.kernels]:
            print(f"{n:48s} {c:6d} {t / 1e6:8.2f} ms {t / c / 1e3:9.1f} us")


def calls(rows, pat, span_ns, queue=""):
    t_hi = max(r[1] for r in rows)
    t_lo = t_hi - span_ns
    sel = [r for r in rows if (pat == "*" or pat in r[3]) and r[0] >= t_lo and (not queue or r[2] == queue)]
    print(f"calls of *{pat}* in the last {span_ns / 1e6:.1f} ms (start offset, duration, what else ran):")
    for s, e, q, n in sel:
        other = defaultdict(int)
        for s2, e2, q2, n2 in rows:
            if q2 != q and s2 < e and e2 > s:
                other[n2] += min(e, e2) - max(s, s2)
        top = ", ".join(f"{k} {v / 1e3:.0f}" for k, v in sorted(other.items(), key=lambda kv: -kv[1])[:3])
        print(f"  {(s - t_lo) / 1e3:9.1f} us  {n:24s} q{q}  {(e - s) / 1e3:8.1f} us   [{top}]")


if __name__ == "__main__":
    main()
