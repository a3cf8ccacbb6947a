"""The committed measurement records agree with each other (CPU): the
bench's HIP-event kernel table and the rocprofv3 kernel trace of the same
command (profiles/r06/final, tools/rocprof_agree.py), and the PMC summaries
the bench lines read their `traffic` from."""
import json
import os
import subprocess
import sys

from conftest import ROOT

FINAL = os.path.join(ROOT, "profiles", "r06", "final")


def test_rocprof_trace_agrees_with_hip_events():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rocprof_agree.py"), FINAL,
                        os.path.join(FINAL, "bench_under_rocprof.json")],
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    cls = out["classes"]
    assert {"resident_users", "resident_items", "gram_users", "gram_items"} <= set(cls)
    for name, c in cls.items():
        assert abs(c["ratio"] - 1.0) < 0.02, (name, c)
    # the replay slice, not the whole-process mean, is what the bench reports
    ru = cls["resident_users"]
    assert abs(ru["rocprof_us_per_cg_iteration"] - ru["events_us_per_cg_iteration"]) \
        < 0.02 * ru["events_us_per_cg_iteration"]


def test_resident_traffic_matches_launch_per_iteration_counters():
    res = json.load(open(os.path.join(ROOT, "profiles", "r06", "pmc_resident_k64.json")))
    for side in ("users", "items"):
        direct = res[side]["bytes_per_cg_iteration"]
        per_launch = res["launch_per_iteration_pmc_bytes"][side]
        assert abs(direct / per_launch - 1.0) < 0.01, (side, direct, per_launch)


def test_bench_cg_traffic_from_committed_pmc():
    sys.path.insert(0, ROOT)
    import bench_cg
    a = bench_cg.pmc_traffic("spmv_a", 27_000_000, 2_800_000, 10)
    assert a is not None and 3.5e9 < a < 4.2e9
    assert bench_cg.pmc_traffic("spmv_a", 1000, 100, 10) is None   # other shapes: unmeasured
