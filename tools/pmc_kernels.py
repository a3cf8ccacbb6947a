"""Per-kernel means of arbitrary rocprofv3 --pmc counters.
    python tools/pmc_kernels.py DIR [DIR ...]"""
import csv, glob, os, re, sys
from collections import defaultdict
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import classify

acc = defaultdict(lambda: defaultdict(dict))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            cls = classify(row.get("Kernel_Name", ""))
            if cls is None:
                continue
            key = row.get("Dispatch_Id")
            c = row["Counter_Name"]
            acc[cls][c][key] = acc[cls][c].get(key, 0.0) + float(row["Counter_Value"])
for cls in sorted(acc):
    print(cls)
    for c in sorted(acc[cls]):
        v = sorted(acc[cls][c].values())
        mx = max(v)
        act = [x for x in v if x >= 0.05 * mx] or v
        print(f"   {c:32s} mean {sum(act)/len(act):16.1f}  n={len(act)}")
