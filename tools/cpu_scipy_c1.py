"""Time the reference's SciPy ALS path (oracle/scipy_als.py) on the C1
workload (BASELINE.json configs[0]: MovieLens-100K shape, k = 10) on this
host's CPU share, as the north star's "SciPy CPU path" baseline; prints one
JSON line.  The GPU side of the same config: ``bench.py --shape ml-100k
--k 10``."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from movie_recommender_amd import synth  # noqa: E402
from oracle import scipy_als  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rs = synth.movielens_like("ml-100k", k)
u = rs.user_ids.astype(np.int64)
i = rs.item_ids.astype(np.int64)
sec, ts = scipy_als.time_iterations(u, i, rs.ratings, rs.num_users, rs.num_items, k)
print(json.dumps({"metric": "ratings/sec per ALS iteration (SciPy lsqr path, C1 shape)",
                  "value": rs.n / sec, "unit": "ratings/s", "k": k, "n_ratings": int(rs.n),
                  "users": rs.num_users, "items": rs.num_items, "s_per_iteration": sec,
                  "iterations_s": ts, "threads": len(os.sched_getaffinity(0)),
                  "kind": "port",
                  "note": "python/100k_data/ratings_als.py:347-526 restated (vectorised design "
                          "matrices; scipy.sparse.linalg.lsqr iter_lim=100 per half-step); "
                          "not the C++ library's CG, so no parity claim"}))
