"""The compiled reference's CG trajectory on the bench workload -- TEST INFRA.

    python tools/ref_trajectory.py [--iterations 25] [--threads 8] [--out F]

Replays ``als()`` (``cpp/ls_lib/matrix.cpp:814-892``) around the reference's
own ``cg_least_squares`` (``oracle/ref_replay.als_replay``, bit-identical to
``als_from_python``) on bench.py's data (ML-full shape, k = 64, the cached
synthetic set) from bench.py's start (``RandomState(0)``: U0 then V0, the
order of ``cpp/python/cpp_ls.py:147-148``), with the outer stop test switched
off (min_r_decrease = -inf) so every one of ``--iterations`` ALS iterations
runs; the inner CG keeps the reference's (0.01, 200).  Writes one JSON
record per ALS iteration (CG iterations and seconds per half-step, final rr)
as it goes, so a long run can be read while it runs.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ref  # noqa: E402
from oracle.ref_replay import als_replay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=25)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--shape", default="ml-full")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04",
                                                  "ref_trajectory_c3_k64.jsonl"))
    a = ap.parse_args()
    import bench
    rs = bench.load_data(a.shape, a.k)
    U0, V0 = ref.init_factors(rs.num_users, rs.num_items, a.k, a.seed)
    ref.set_thread_count(a.threads)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    t0 = time.time()
    with open(a.out, "w") as f:
        f.write(json.dumps({"shape": a.shape, "k": a.k, "n": rs.n, "users": rs.num_users,
                            "items": rs.num_items, "threads": a.threads,
                            "start": f"RandomState({a.seed}) U0, V0 (bench.py: 0)",
                            "outer_stop": "off (min_r_decrease=-inf)"}) + "\n")
        f.flush()

        def on_iteration(it, rec):
            f.write(json.dumps(dict(iteration=it + 1, **rec,
                                    wall_s=round(time.time() - t0, 1))) + "\n")
            f.flush()

        als_replay(rs.user_ids, rs.item_ids, rs.ratings, a.k, U0, V0,
                   min_r_decrease=-np.inf, max_iteration=a.iterations, on_iteration=on_iteration)


if __name__ == "__main__":
    main()
