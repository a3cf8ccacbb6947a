"""Find the first half-step whose result depends on kernel-event timing:
replay from one snapshot with timing on / off, compare factors after each
half-step.  python tools/replay_bisect.py [--k 64]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--halves", type=int, default=6)
a = ap.parse_args()
rs = synth.movielens_like("ml-full", a.k)
k = a.k
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * k)
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    ctx.iterate(3)
    snap = ctx.get_factors()
    traj = {}
    for timing in (True, False, True, False):
        ctx.set_factors(*snap)
        ctx.set_timing(timing)
        out = []
        for h in range(a.halves):
            its = ctx.half_step("users" if h % 2 == 0 else "items")
            U, V = ctx.get_factors()
            out.append((its, U.copy(), V.copy()))
        traj.setdefault(timing, []).append(out)
    for h in range(a.halves):
        t0, f0 = traj[True][0][h], traj[False][0][h]
        t1, f1 = traj[True][1][h], traj[False][1][h]
        eq = lambda x, y: np.array_equal(x[1], y[1]) and np.array_equal(x[2], y[2])
        print(f"half {h}: its T={t0[0]},{t1[0]} F={f0[0]},{f1[0]}  T==T {eq(t0, t1)}  F==F {eq(f0, f1)}  T==F {eq(t0, f0)}"
              f"  max|dU| {np.max(np.abs(t0[1]-f0[1])):.2e} max|dV| {np.max(np.abs(t0[2]-f0[2])):.2e}")
