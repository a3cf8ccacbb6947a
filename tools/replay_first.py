"""Isolate run-to-run state leaks: set/get round trip, then the first user
half-step (and the following item half-step) repeated from one snapshot.
Usage: python tools/replay_first.py [k]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

k = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rs = synth.movielens_like("ml-full", k)
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * k)
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    ctx.iterate(3)
    snap = tuple(a.copy() for a in ctx.get_factors())
    for r in range(3):
        ctx.set_factors(*snap)
        U, V = ctx.get_factors()
        print("roundtrip", r, np.array_equal(U, snap[0]), np.array_equal(V, snap[1]), flush=True)
    ref = None
    for r in range(4):
        ctx.set_factors(*snap)
        ctx.sync()
        its_u, rr_u = ctx.half_step("users")
        ctx.sync()
        U1, _ = ctx.get_factors()
        its_i, rr_i = ctx.half_step("items")
        ctx.sync()
        U2, V2 = ctx.get_factors()
        print(f"run {r}: users its {its_u} rr {rr_u:.17g} |U| {np.abs(U1).sum():.12e}; "
              f"items its {its_i} rr {rr_i:.17g} |U| {np.abs(U2).sum():.12e} "
              f"|V| {np.abs(V2).sum():.12e}", flush=True)
        if ref is None:
            ref = (U1, U2, V2)
        else:
            print("   same as run 0:", np.array_equal(U1, ref[0]), np.array_equal(U2, ref[1]),
                  np.array_equal(V2, ref[2]), " U1==U2:", np.array_equal(U1, U2), flush=True)
