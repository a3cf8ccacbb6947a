"""How determined is the headline's first users solve?  (CPU, TEST INFRA)

    python tools/first_solve_sensitivity.py [--out F] [--threads 2 4 6 8 16]

The bench's workload (ML-full shape, k = 64) from the RandomState(0) start:
the first users CG solve (matrix.cpp:456-529 inside als(), iteration 1)
stops after 59 / 54 / 59 CG iterations in the compiled reference at 6 / 8 /
16 threads, and after 35 in the engine (profiles/r04/cg_count_parity_c3_k64
.jsonl).  This tool runs that one solve many ways and records every run's
count and r.r sequence:

  ref_tc<T>  the reference's own cg_least_squares on its design matrix at T
             threads (the summation order is the thread split);
  ex64       the oracle's block-Gram CG, all fp64 (the reference in block
             form);
  x32        ex64 with x0 rounded to fp32 (the engine's factor table);
  g32        G, c rounded to fp32, x0 fp64;
  g32x32     G, c and x0 in fp32 (the engine's precision contract);
  ex64_eps<s> ex64 from x0 (1 + 1e-13 xi), xi ~ N(0, 1) seed s: a relative
             perturbation 10^5 times below fp32 rounding.

If counts scatter between ~35 and ~60 over perturbations far below any
arithmetic difference between the engine and the reference, the 35-vs-59
split is the solve's own sensitivity, not a defect of either side.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import als_oracle as O  # noqa: E402
from oracle import ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--threads", type=int, nargs="*", default=[2, 4, 6, 8, 16])
    ap.add_argument("--eps-seeds", type=int, default=6)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05",
                                                  "first_solve_sensitivity_c3_k64.jsonl"))
    a = ap.parse_args()
    import bench
    k = a.k
    K = k + 1
    rs = bench.load_data("ml-full", k, scale=a.scale)
    U0, V0 = ref.init_factors(rs.num_users, rs.num_items, k, 0)
    uid = np.ascontiguousarray(rs.user_ids, np.int32)
    iid = np.ascontiguousarray(rs.item_ids, np.int32)
    r = np.ascontiguousarray(rs.ratings, np.float64)
    n = len(r)
    f = open(a.out, "a")
    t0 = time.time()

    def emit(name, its, rr, tr=None):
        rec = {"variant": name, "cg_iterations": int(its), "final_rr": rr,
               "wall_s": round(time.time() - t0, 1)}
        if tr is not None:
            rec["rr"] = tr
        print(json.dumps({x: rec[x] for x in rec if x != "rr"}), flush=True)
        f.write(json.dumps(rec) + "\n")
        f.flush()

    # the reference's own solve on its design matrix (fill_user_A, :898-952)
    rp = (np.arange(n + 1, dtype=np.int64) * K).astype(np.int32)
    ci = (uid.astype(np.int64)[:, None] * K + np.arange(K)).astype(np.int32).reshape(-1)
    va = np.empty((n, K))
    va[:, :k] = V0.reshape(-1, k)[iid]
    va[:, k] = 1.0
    va = va.reshape(-1)
    for tc in a.threads:
        ref.set_thread_count(tc)
        _, its, rr = ref.cg_least_squares(rp, ci, va, len(U0), r, U0)
        emit(f"ref_tc{tc}", its, rr)
    ref.set_thread_count(1)
    del va, ci, rp

    G, c = O.gram_user(uid, iid, r, V0, k, rs.num_users)
    runs = [("ex64", G, c, U0.copy()),
            ("x32", G, c, U0.astype(np.float32).astype(np.float64))]
    for s in range(a.eps_seeds):
        xi = np.random.default_rng(s).standard_normal(len(U0))
        runs.append((f"ex64_eps{s}", G, c, U0 * (1 + 1e-13 * xi)))
    for name, Gv, cv, x in runs:
        tr = []
        its, rr = O.cg_blocks(Gv, cv, x, 0.01, 200, trace=tr)
        emit(name, its, rr, tr)
    G32 = G.astype(np.float32).astype(np.float64)
    c32 = c.astype(np.float32).astype(np.float64)
    del G, runs
    for name, x in (("g32", U0.copy()), ("g32x32", U0.astype(np.float32))):
        tr = []
        its, rr = O.cg_blocks(G32, c32, x, 0.01, 200, trace=tr)
        emit(name, its, rr, tr)


if __name__ == "__main__":
    main()
