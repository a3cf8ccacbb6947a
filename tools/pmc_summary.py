"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into per-kernel HBM
bytes per launch (profiles/pmc_<round>.json, read by bench.py).

    python tools/pmc_summary.py --fetch DIR_FETCH --write DIR_WRITE --out profiles/pmc_r03.json

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) reports
half the bytes of wide (16 B/lane) coalesced streaming reads -> x2; WRITE_SIZE
(KB) is exact for 16 B/lane streaming stores.  Dispatches whose counter is
below 5 % of the kernel's maximum are early-exit CG launches and are ignored.
"""
import argparse
import csv
import glob
import json
import os
import re

CLASSES = [
    ("gram_users", r"gram_kernel<\d+, true|gram_pair_kernel<true"),
    ("gram_items", r"gram_kernel<\d+, false|gram_pair_kernel<false"),
    ("matvec_users", r"(cg_matvec_kernel|cg_onepass_kernel)<\d+, true"),
    ("matvec_items", r"(cg_matvec_kernel|cg_onepass_kernel)<\d+, false"),
    ("resident_users", r"cg_resident_kernel<\d+, true"),
    ("resident_items", r"cg_resident_kernel<\d+, false"),
    ("slab_reduce", r"slab_reduce_kernel"),
    ("cg_update", r"cg_update_kernel"),
    ("cg_control", r"cg_control_kernel"),
    ("rec_score", r"rec_score_kernel"),
    ("rec_select", r"rec_select_kernel"),
]


def classify(name):
    for cls, pat in CLASSES:
        if re.search(pat, name):
            return cls
    return None


def read_counter(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            cls = classify(row.get("Kernel_Name", ""))
            if cls is None:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals.setdefault(cls, {}).setdefault(key, 0.0)
            vals[cls][key] += float(row["Counter_Value"])
    out = {}
    for cls, disp in vals.items():
        v = sorted(disp.values())
        mx = max(v) if v else 0.0
        act = [x for x in v if x >= 0.05 * mx]
        out[cls] = {"mean_kb": sum(act) / max(1, len(act)), "dispatches": len(act)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--shape", default="ml-full", help="bench workload the passes ran")
    ap.add_argument("--k", type=int, default=64)
    a = ap.parse_args()
    fe = read_counter(a.fetch, "FETCH_SIZE")
    wr = read_counter(a.write, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                     "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per active dispatch",
           "workload": {"shape": a.shape, "k": a.k},
           "per_kernel": {}, "hbm_bytes_per_launch": {}}
    for cls in sorted(set(fe) | set(wr)):
        f = fe.get(cls, {}).get("mean_kb", 0.0)
        w = wr.get(cls, {}).get("mean_kb", 0.0)
        b = (2.0 * f + w) * 1024.0
        res["per_kernel"][cls] = {"fetch_kb": f, "write_kb": w, "bytes_corrected": b,
                                  "dispatches": fe.get(cls, {}).get("dispatches", 0)}
        res["hbm_bytes_per_launch"][cls] = int(b)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["hbm_bytes_per_launch"]))


if __name__ == "__main__":
    main()
