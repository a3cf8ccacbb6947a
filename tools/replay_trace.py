"""Per-half-step CG iteration counts of a replay from one snapshot, timed (T)
vs untimed (F) launches: shows the first half-step where the two diverge.
Usage: python tools/replay_trace.py [k] [half_steps]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

k = int(sys.argv[1]) if len(sys.argv) > 1 else 64
nh = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rs = synth.movielens_like("ml-full", k)
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * k)
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    ctx.iterate(3)
    snap = ctx.get_factors()
    out = {}
    for name in ("T", "F", "T2", "F2"):
        ctx.set_factors(*snap)
        ctx.sync()
        ctx.set_timing(name.startswith("T"))
        hs = [ctx.half_step(s) for _ in range(nh // 2) for s in ("users", "items")]
        its = [h[0] for h in hs]
        print(name, "rr", [f"{h[1]:.17g}" for h in hs], flush=True)
        U, V = ctx.get_factors()
        out[name] = (its, U, V)
        print(f"{name:3s} its {its} sum|U| {np.abs(U).sum():.9e} sum|V| {np.abs(V).sum():.9e}",
              flush=True)
    for name in ("F", "T2", "F2"):
        print(name, "== T:", np.array_equal(out[name][1], out["T"][1])
              and np.array_equal(out[name][2], out["T"][2]))
