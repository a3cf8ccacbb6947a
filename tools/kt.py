"""Print a bench JSON line's headline numbers and kernel table."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e9, 3), "G/s", d["ms_per_step"], "ms", "cg/step",
          d["cg_iterations"]["per_step_users"], d["cg_iterations"]["per_step_items"],
          "with events", d.get("ms_per_step_with_kernel_events"))
    for k, v in d["kernels"].items():
        print("   %-15s %9.2f us x%4d  %s GB/s" % (k, v["avg_us"], v["launches"], v["alg_GBps"]))
