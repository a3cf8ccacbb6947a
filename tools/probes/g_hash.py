"""Hash of the normal equations and of two ALS iterations' factors for a set
of k (both sides, split and unsplit entities): run once per library build
(MR_LIB_PATH) and compare the lines -- a layout-preserving kernel change
(e.g. MR_G_WIDE) must print identical hashes."""
import hashlib
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from movie_recommender_amd import _lib  # noqa: E402
from movie_recommender_amd.engine import AlsContext  # noqa: E402


def h(*arrs):
    m = hashlib.sha256()
    for a in arrs:
        m.update(np.ascontiguousarray(a).tobytes())
    return m.hexdigest()[:16]


out = {}
for chunk in (2048, 64):
    _lib.check(_lib.lib().mr_set_gram_chunk(chunk), "chunk")
    for k in (32, 33, 48, 64, 65, 80, 96, 112, 120, 128):
        rng = np.random.default_rng(k)
        nU, nI, n = 400, 300, 30000
        u = rng.integers(0, nU, n).astype(np.int32)
        i = (rng.zipf(1.3, n) % nI).astype(np.int32)
        key = np.unique(u.astype(np.int64) * nI + i)
        u = (key // nI).astype(np.int32)
        i = (key % nI).astype(np.int32)
        r = rng.normal(0, 1, len(u))
        U0 = rng.uniform(-1, 1, nU * (k + 1))
        V0 = rng.uniform(-1, 1, nI * k)
        with AlsContext(u, i, r, k, nU, nI) as ctx:
            ctx.set_factors(U0, V0)
            hs = []
            for side, ne in (("users", nU), ("items", nI)):
                ctx.build_normal_equations(side)
                G, c = ctx.normal_equations(side, np.arange(ne))
                hs.append(h(G, c))
            ctx.set_factors(U0, V0)
            ctx.iterate(2)
            U, V = ctx.get_factors()
            hs.append(h(U, V))
        out[f"k{k}_c{chunk}"] = hs
_lib.check(_lib.lib().mr_set_gram_chunk(2048), "reset chunk")
print(json.dumps(out, sort_keys=True))
