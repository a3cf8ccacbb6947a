"""Determinism check: the same ALS steps replayed from one factor snapshot
must give bit-identical factors and CG counts (with and without kernel-event
timing).  python tools/replay_check.py [--k 128] [--steps 5]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--shape", default="ml-full")
a = ap.parse_args()
rs = synth.movielens_like(a.shape, a.k)
k = a.k
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * k)
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    ctx.iterate(3)
    snap = ctx.get_factors()
    res = []
    for timing in (True, False, False, True):
        ctx.set_factors(*snap)
        ctx.reset_stats()
        ctx.set_timing(timing)
        ctx.iterate(a.steps)
        st = ctx.stats()
        U, V = ctx.get_factors()
        res.append((U, V, st["cg_users_total"], st["cg_items_total"]))
        print(f"timing={timing} cg users {st['cg_users_total']} items {st['cg_items_total']}")
    for i, j in ((0, 3), (1, 2), (0, 1)):
        same = np.array_equal(res[i][0], res[j][0]) and np.array_equal(res[i][1], res[j][1])
        print(f"run {i} vs {j}: bitwise equal = {same}; max |dU| = {np.max(np.abs(res[i][0]-res[j][0])):.3e}")
