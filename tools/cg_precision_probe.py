"""Why does a CG half-step take the iteration count it takes?  (CPU, TEST INFRA)

    python tools/cg_precision_probe.py [--from-it 5] [--steps 6] [--threads 6] [--out F]

On the bench workload (ML-full shape, k = 64, RandomState(0) start) the
compiled reference's ALS is replayed (``oracle/ref_replay``: bit-identical to
``als_from_python``) to iteration ``--from-it``; then for ``--steps`` further
half-steps of each side, from the reference's own state, the same CG solve
is run five ways and the iteration counts compared:

  ref      the reference's cg_least_squares on its design matrix (fp64 SpMV /
           SpMV^T, matrix.cpp:456-529) -- the state then advances with it;
  ex64     the oracle's block-Gram CG, everything fp64 (the reference in
           block form);
  rows32   the factor rows rounded to fp32 (the engine's fp32 tables), G, c
           and x fp64;
  engine   fp32 rows, G and c rounded to fp32, fp32 x (the engine's
           precision contract, DESIGN.md "Precision");
  g32x64   as engine but fp64 x.

A systematic gap between ``ref`` / ``blk64`` and ``blk32`` would make the
engine's CG counts (and with them its rate per ALS iteration) differ from the
reference's for a reason other than the trajectory's chaos.
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
    ap.add_argument("--from-it", type=int, default=5)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04",
                                                  "cg_precision_probe.jsonl"))
    a = ap.parse_args()
    import bench
    k = a.k
    K = k + 1
    rs = bench.load_data("ml-full", k, scale=a.scale)
    U0, V0 = ref.init_factors(rs.num_users, rs.num_items, k, a.seed)
    ref.set_thread_count(a.threads)
    uid = np.ascontiguousarray(rs.user_ids, np.int32)
    iid = np.ascontiguousarray(rs.item_ids, np.int32)
    r = np.ascontiguousarray(rs.ratings, np.float64)
    n = len(r)
    U = U0.copy()
    V = V0.copy()
    rp_u = (np.arange(n + 1, dtype=np.int64) * K).astype(np.int32)
    ci_u = (uid.astype(np.int64)[:, None] * K + np.arange(K)).astype(np.int32).reshape(-1)
    va_u = np.empty((n, K))
    va_u[:, k] = 1.0
    rp_i = (np.arange(n + 1, dtype=np.int64) * k).astype(np.int32)
    ci_i = (iid.astype(np.int64)[:, None] * k + np.arange(k)).astype(np.int32).reshape(-1)
    va_i = np.empty((n, k))
    Vm = V.reshape(-1, k)
    Um = U.reshape(-1, K)
    f = open(a.out, "a")
    t0 = time.time()

    ord_u = np.argsort(uid, kind="stable")
    off_u = np.concatenate([[0], np.cumsum(np.bincount(uid, minlength=rs.num_users))])
    ord_i = np.argsort(iid, kind="stable")
    off_i = np.concatenate([[0], np.cumsum(np.bincount(iid, minlength=rs.num_items))])

    def grams(side, rows32):
        """Normal equations in fp64 (oracle gram_user / gram_item, one entity
        at a time to stay within memory) from the fp64 factor rows, or
        (rows32) from the rows rounded to fp32 as the engine's fp32 factor
        tables hold them."""
        if side == "users":
            E, KK, order, off = rs.num_users, K, ord_u, off_u
        else:
            E, KK, order, off = rs.num_items, k, ord_i, off_i
        G = np.zeros((E, KK, KK))
        c = np.zeros((E, KK))
        Vs = Vm.astype(np.float32).astype(np.float64) if rows32 else Vm
        Us = Um.astype(np.float32).astype(np.float64) if rows32 else Um
        for e in range(E):
            sel = order[off[e]:off[e + 1]]
            if len(sel) == 0:
                continue
            if side == "users":
                ae = np.empty((len(sel), K))
                ae[:, :k] = Vs[iid[sel]]
                ae[:, k] = 1.0
                w = r[sel]
            else:
                ae = Us[uid[sel], :k]
                w = r[sel] - Us[uid[sel], k]
            G[e] = ae.T @ ae
            c[e] = ae.T @ w
        return G, c

    def probe(side, it, x0):
        out = {}
        G, c = grams(side, False)
        x = x0.copy()
        out["ex64"] = list(O.cg_blocks(G, c, x, 0.01, 200))
        G, c = grams(side, True)
        x = x0.copy()
        out["rows32"] = list(O.cg_blocks(G, c, x, 0.01, 200))
        G = G.astype(np.float32).astype(np.float64)
        c = c.astype(np.float32).astype(np.float64)
        x = x0.astype(np.float32)
        out["engine"] = list(O.cg_blocks(G, c, x, 0.01, 200))
        x = x0.copy()
        out["g32x64"] = list(O.cg_blocks(G, c, x, 0.01, 200))
        return out

    for it in range(a.from_it + a.steps):
        probing = it >= a.from_it
        va_u[:, :k] = Vm[iid]
        rec_u = probe("users", it, U) if probing else None
        x, cu, rru = ref.cg_least_squares(rp_u, ci_u, va_u.reshape(-1), len(U), r, U)
        U[:] = x
        va_i[:, :] = Um[uid, :k]
        b = r - Um[uid, k]
        rec_i = probe("items", it, V) if probing else None
        x, cit, rri = ref.cg_least_squares(rp_i, ci_i, va_i.reshape(-1), len(V), b, V)
        V[:] = x
        line = {"iteration": it + 1, "ref_users": [cu, rru], "ref_items": [cit, rri],
                "wall_s": round(time.time() - t0, 1)}
        if probing:
            line["users"] = rec_u
            line["items"] = rec_i
        print(json.dumps(line), flush=True)
        if probing:
            f.write(json.dumps(line) + "\n")
            f.flush()


if __name__ == "__main__":
    main()
