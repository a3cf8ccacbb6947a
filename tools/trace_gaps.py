"""Idle-gap analysis of a rocprofv3 kernel trace (run_kernel_trace.csv).

For the last N dispatches (the timed region): kernel busy time vs wall span,
the largest gaps between consecutive kernels and which kernels they separate,
and per-kernel-name gap totals (gap BEFORE each kernel).
Usage: python tools/trace_gaps.py TRACE_CSV [--last N]
"""
import argparse
import csv
import collections


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("mr::", "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--after", default="", help="start after the last dispatch of this kernel")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if a.after:
        idx = [i for i, r in enumerate(rows) if short(r[2]).startswith(a.after)]
        if idx:
            rows = rows[idx[-1] + 1:]
    if a.last:
        rows = rows[-a.last:]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    print(f"dispatches {len(rows)}  span {span/1e6:.3f} ms  busy {busy/1e6:.3f} ms  "
          f"idle {(span-busy)/1e6:.3f} ms ({100*(span-busy)/span:.1f} %)")
    gaps = []
    before = collections.defaultdict(lambda: [0, 0])
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = s1 - e0
        gaps.append((g, short(n0), short(n1)))
        before[short(n1)][0] += g
        before[short(n1)][1] += 1
    gaps.sort(reverse=True)
    print("largest gaps (us): prev -> next")
    for g, n0, n1 in gaps[:a.top]:
        print(f"  {g/1e3:9.1f}  {n0} -> {n1}")
    print("gap before kernel: total ms, count, mean us")
    for n, (t, c) in sorted(before.items(), key=lambda kv: -kv[1][0]):
        print(f"  {t/1e6:8.3f} {c:6d} {t/1e3/c:8.1f}  {n}")


if __name__ == "__main__":
    main()
