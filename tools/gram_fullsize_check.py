"""Full-size Gram readout per entity, bf3 vs f32 path (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext
k = 64
rs = synth.movielens_like("ml-full", k)
rng = np.random.default_rng(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1)); V0 = rng.uniform(-1, 1, rs.num_items * k)
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    for side in ("users", "items"):
        ids = rs.user_ids if side == "users" else rs.item_ids
        cnt = np.bincount(ids)
        ents = np.unique(np.concatenate([np.argsort(cnt)[-3:], np.argsort(cnt)[:3],
                                         rng.integers(0, len(cnt), 6)])).astype(np.int32)
        for bf3 in ("1", "0"):
            os.environ["MR_GRAM_BF3"] = bf3
            ctx.build_normal_equations(side)
            G, c = ctx.normal_equations(side, ents)
            print(side, "bf3", bf3, [(int(e), int(cnt[e]), float(np.abs(G[t]).max())) for t, e in enumerate(ents)], flush=True)
