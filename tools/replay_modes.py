"""Which host pattern changes results?  Replays 4 ALS iterations from one
snapshot under several host patterns and compares the factors bitwise."""
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
    snap = ctx.get_factors()
    modes = {
        "T_iter4": (True, lambda: ctx.iterate(4)),
        "F_iter4": (False, lambda: ctx.iterate(4)),
        "F_iter1sync": (False, lambda: [(ctx.iterate(1), ctx.sync()) for _ in range(4)]),
        "F_halfsync": (False, lambda: [(ctx.half_step(s), ctx.sync()) for _ in range(4) for s in ("users", "items")]),
        "F_half": (False, lambda: [ctx.half_step(s) for _ in range(4) for s in ("users", "items")]),
        "T_half": (True, lambda: [ctx.half_step(s) for _ in range(4) for s in ("users", "items")]),
        "F_iter4b": (False, lambda: ctx.iterate(4)),
    }
    res = {}
    for name, (timing, fn) in modes.items():
        ctx.set_factors(*snap)
        ctx.reset_stats()
        ctx.set_timing(timing)
        fn()
        st = ctx.stats()
        U, V = ctx.get_factors()
        res[name] = (U, V)
        print(f"{name:12s} cg users {st['cg_users_total']} items {st['cg_items_total']} "
              f"sum|U| {np.abs(U).sum():.9e}")
    ref = res["T_iter4"]
    for name, (U, V) in res.items():
        print(f"{name:12s} == T_iter4: {np.array_equal(U, ref[0]) and np.array_equal(V, ref[1])}")
