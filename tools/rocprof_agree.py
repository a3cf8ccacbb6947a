"""Check the bench's HIP-event kernel table against a rocprofv3 kernel trace
of the same command (bench.py under `rocprofv3 --kernel-trace --stats`).

The resident CG solve runs a whole solve per launch, so a launch's duration
depends on its CG iteration count, and rocprof's per-kernel average over the
whole process (warmup, timed steps, the instrumented replay, same_window,
trajectory) is not the replay's average.  The replay's launches are a known
slice of the dispatch sequence: per side, launch i of the process is ALS
iteration i, in the order warmup (W), timed (K), replay (K), same_window (3),
trajectory (max(3, W + K)).  This picks the replay slice from the trace and
compares its mean duration -- and, with the bench's CG counts, its time per
CG iteration -- with the bench's own numbers for the same launches.

Usage: python tools/rocprof_agree.py TRACE_DIR BENCH_JSON [--out FILE]
"""
import argparse
import csv
import glob
import json
import os

CLASSES = {
    "resident_users": ("cg_resident_kernel<", "true"),
    "resident_items": ("cg_resident_kernel<", "false"),
    "gram_users": ("gram_kernel<", "true"),
    "gram_items": ("gram_kernel<", "false"),
}


def side_of(name, prefix):
    """USER template argument (second of cg_resident_kernel / gram_kernel)."""
    args = name.split(prefix, 1)[1].split(">", 1)[0].split(",")
    return args[1].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("bench_json")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    b = json.load(open(a.bench_json))
    W, K = b["warmup"], b["steps"]
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = {"source": os.path.relpath(files[0]) if files else None, "warmup": W, "steps": K,
           "slice": f"launches {W + K} .. {W + 2 * K - 1} of each class (the instrumented replay)",
           "classes": {}}
    for cls, (prefix, user) in CLASSES.items():
        seq = [r for r in rows if prefix in r["Kernel_Name"] and side_of(r["Kernel_Name"], prefix) == user]
        if len(seq) < W + 2 * K or cls not in b.get("kernels", {}):
            continue
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in seq]
        rep = dur[W + K:W + 2 * K]
        ev = b["kernels"][cls]
        ent = {"rocprof_all_launches": len(dur),
               "rocprof_mean_all_us": round(sum(dur) / len(dur), 2),
               "rocprof_mean_replay_us": round(sum(rep) / len(rep), 2),
               "events_mean_replay_us": ev["avg_us"],
               "ratio": round((sum(rep) / len(rep)) / ev["avg_us"], 4)}
        if ev.get("cg_iterations"):
            ent["rocprof_us_per_cg_iteration"] = round(sum(rep) / ev["cg_iterations"], 2)
            ent["events_us_per_cg_iteration"] = ev["us_per_cg_iteration"]
        out["classes"][cls] = ent
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
