"""smoke()'s case with the bf16x3 and fp32 Gram paths against the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext
from oracle import als_oracle
k = 32
u, i, r, *_ = synth.dense_fixture(60, 50, k, keep=0.8, seed=1)
rs = np.random.RandomState(0)
U0 = rs.uniform(-1, 1, 60 * (k + 1)); V0 = rs.uniform(-1, 1, 50 * k)
Uo, Vo, reto, _ = als_oracle.als_block(u, i, r, k, U0, V0, 0.01, 3)
for bf3 in ("1", "0"):
    os.environ["MR_GRAM_BF3"] = bf3
    with AlsContext(u, i, r, k, 60, 50, device=0) as ctx:
        ctx.set_factors(U0, V0); ret = ctx.run(0.01, 3); U, V = ctx.get_factors(); st = ctx.stats()
    print("bf3", bf3, ret, reto, np.max(np.abs(U - Uo)) / np.max(np.abs(Uo)),
          np.max(np.abs(V - Vo)) / np.max(np.abs(Vo)), st["cg_users_total"], st["cg_items_total"], flush=True)
