"""Durations of, and idle gaps before, the kernels of a rocprofv3 kernel trace
(``rocprofv3 --kernel-trace -d DIR -o run -- ...``; CSV files or the rocpd
database ``run_results.db`` this rocprofv3 writes by default): per kernel-name match,
the mean / median duration and the mean / median gap since the previous
kernel on the same queue ended -- what a chain of short dependent launches
(one CG iteration per launch at shard sizes) loses between kernels.

    python tools/trace_gaps.py DIR_OR_CSV_OR_DB [--match cg_onepass] [--skip 0]
                               [--stats-csv OUT.csv]
"""
import argparse
import csv
import glob
import os
import sqlite3
import statistics


def rows(path):
    """Kernel records of a CSV trace or of rocprofv3's rocpd database (.db)."""
    files = [path] if path.endswith((".csv", ".db")) else sorted(
        glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        + glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
    for f in files:
        if f.endswith(".db"):
            con = sqlite3.connect(f)
            for name, s, e, q in con.execute("select name, start, end, queue_id from kernels"):
                yield {"Kernel_Name": name, "Start_Timestamp": s, "End_Timestamp": e, "Queue_Id": q}
            con.close()
            continue
        with open(f) as fh:
            for r in csv.DictReader(fh):
                yield r


def top_kernels(path, out_csv):
    """rocprofv3's per-kernel summary (the rocpd `top_kernels` view) as a CSV."""
    con = sqlite3.connect(path)
    with open(out_csv, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for r in con.execute("select name, total_calls, total_duration, average, percentage "
                             "from top_kernels"):
            w.writerow(r)
    con.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", action="append", default=[])
    ap.add_argument("--skip", type=int, default=0, help="drop the first N matches (warm-up)")
    ap.add_argument("--stats-csv", default=None,
                    help="also write the per-kernel summary of a .db to this CSV")
    a = ap.parse_args()
    if a.stats_csv:
        top_kernels(a.path, a.stats_csv)
    ks = []
    for r in rows(a.path):
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        s, e = int(r.get("Start_Timestamp", 0)), int(r.get("End_Timestamp", 0))
        q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
        ks.append((s, e, q, name))
    ks.sort()
    last_end = {}
    stats = {}
    for s, e, q, name in ks:
        gap = s - last_end[q] if q in last_end else None
        last_end[q] = max(e, last_end.get(q, 0))
        for m in a.match or [""]:
            if m in name:
                st = stats.setdefault(m or "all", {"dur": [], "gap": []})
                st["dur"].append((e - s) / 1e3)
                if gap is not None:
                    st["gap"].append(gap / 1e3)
    for m, st in stats.items():
        d, g = st["dur"][a.skip:], st["gap"][a.skip:]
        if not d:
            continue
        print(f"{m}: n={len(d)} dur mean {statistics.mean(d):.2f} median {statistics.median(d):.2f} us"
              + (f"; gap before mean {statistics.mean(g):.2f} median {statistics.median(g):.2f} us"
                 if g else ""))


if __name__ == "__main__":
    main()
