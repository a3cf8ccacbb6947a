"""Diagnostic: per-half-step CG iteration counts and final rr on the bench
workload (ML-full shape), for comparing kernel variants / library builds.
    python tools/cg_trace.py [--k 64] [--steps 8] [--model lowrank|uniform]"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--model", default="lowrank")
ap.add_argument("--shape", default="ml-full")
a = ap.parse_args()
rs = synth.movielens_like(a.shape, a.k, model=a.model)
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (a.k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * a.k)
out = []
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, a.k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    for s in range(a.steps):
        t0 = time.perf_counter()
        cu, rru = ctx.half_step("users")
        ci, rri = ctx.half_step("items")
        ctx.sync()
        out.append(dict(step=s, cg_users=cu, rr_users=rru, cg_items=ci, rr_items=rri,
                        ms=round((time.perf_counter() - t0) * 1e3, 2)))
        print(json.dumps(out[-1]), flush=True)
