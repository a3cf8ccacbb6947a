"""A/B of the CG iteration at a FIXED number of CG iterations (no stop rule:
min_r_decrease = -inf never fails, max_iteration = M), so summation-order
changes cannot confound kernel timings.  ML-full shape, warmed up by a few
ALS iterations; reports per side the solve time per CG iteration (HIP-event
span of the solve phase / M) and the per-class kernel means.

    python tools/cg_ab.py [--k 64] [--m 20] [--reps 3] [--onepass 0|1] [--tag NAME]
                          [--opt gram_rhs_mfma=0 ...] [--shard R/N]
(MR_LIB_PATH selects a variant library, tools/build_var.sh)

``--shard R/N``: one rank's share of an N-rank run on this one GPU -- a shard
context over rank R's cost-balanced users and items (distributed.shard_views)
with no transport attached, so the CG scalars stay local: the per-rank
kernel work of the sharded run without its exchanges (the collective model's
"compute per rank")."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_data  # noqa: E402
from movie_recommender_amd.engine import AlsContext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--m", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--onepass", type=int, default=1)
ap.add_argument("--tag", default="")
ap.add_argument("--opt", action="append", default=[],
                help="engine option NAME=VALUE (engine.OPTIONS), repeatable")
ap.add_argument("--shard", default=None, help="R/N: rank R's share of an N-rank run")
ap.add_argument("--wall", action="store_true",
                help="also time the CG iteration WITHOUT per-launch events: host wall "
                     "time of reps half-steps at m and at 2m fixed CG iterations, "
                     "(T(2m) - T(m)) / (reps m) -- the Gram and the per-call overheads cancel")
a = ap.parse_args()
rs = load_data("ml-full", a.k)
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (a.k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * a.k)
out = {"tag": a.tag or os.environ.get("MR_LIB_PATH", "default"), "k": a.k, "m": a.m,
       "onepass": a.onepass}
if a.shard:
    from movie_recommender_amd.distributed import shard_views
    R, N = (int(x) for x in a.shard.split("/"))
    ur, ir, uv, iv, _, _ = shard_views(rs.user_ids, rs.item_ids, rs.ratings, rs.num_users,
                                       rs.num_items, R, N, k=a.k)
    out["shard"] = {"rank": R, "world": N, "users": list(ur), "items": list(ir),
                    "user_ratings": int(len(uv[0])), "item_ratings": int(len(iv[0]))}
    make = lambda: AlsContext(uv[0], uv[1], uv[2], a.k, rs.num_users, rs.num_items,  # noqa
                              user_range=ur, item_range=ir, item_view=iv)
else:
    make = lambda: AlsContext(rs.user_ids, rs.item_ids, rs.ratings, a.k, rs.num_users,  # noqa
                              rs.num_items)
with make() as ctx:
    ctx.set_option("cg_onepass", a.onepass)
    for o in a.opt:
        name, val = o.split("=")
        ctx.set_option(name, float(val))
    out["grid"] = {side: {"onepass": [ctx.cg_grid(side, False, nt) for nt in (0, 1)],
                          "resident": [ctx.cg_grid(side, True, nt) for nt in (0, 1)]}
                   for side in ("users", "items")}
    ctx.set_factors(U0, V0)
    ctx.iterate(3)
    ctx.sync()
    for side in ("users", "items"):
        ctx.reset_stats()
        ctx.set_timing(True)
        its = []
        for _ in range(a.reps):
            it, _ = ctx.half_step(side, -1e300, a.m)
            its.append(it)
        st = ctx.stats()
        ctx.set_timing(False)
        ph = st["phase_ms"]["solve_" + side]
        n_it = sum(its)
        out[side] = {"cg_iterations": its, "ms_per_cg_iteration": round(ph / n_it, 4),
                     "gram_ms": round(st["phase_ms"]["gram_" + side] / a.reps, 4),
                     "kernels": {c: round(st["kernel_ms"][c] / max(1, st["kernel_launches"][c]) * 1e3, 2)
                                 for c in st["kernel_ms"] if st["kernel_launches"][c]}}
    if a.wall:
        import time
        for side in ("users", "items"):
            T = {}
            for m in (a.m, 2 * a.m):
                ctx.half_step(side, -1e300, m)   # warm
                ctx.sync()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    ctx.half_step(side, -1e300, m)
                ctx.sync()
                T[m] = time.perf_counter() - t0
            out[side]["wall_ms_per_cg_iteration"] = round((T[2 * a.m] - T[a.m]) * 1e3
                                                          / (a.reps * a.m), 4)
print(json.dumps(out), flush=True)
