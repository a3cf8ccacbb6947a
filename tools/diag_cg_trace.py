"""Per-half-step CG counts of the GPU (fused / unfused start) against the
oracle's fp64 block form on one golden fixture (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from movie_recommender_amd.engine import AlsContext  # noqa: E402
from oracle import als_oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "als_dense_60x50_k32_it3.npz"
mi = int(sys.argv[2]) if len(sys.argv) > 2 else 3
with np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", name)) as d:
    d = {k: d[k] for k in d.files}
u, i, r = d["user_ids"].astype(np.int32), d["item_ids"].astype(np.int32), d["ratings"].astype(np.float64)
k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
Uo, Vo, reto, tr = O.als_block(u, i, r, k, d["U0"], d["V0"], max_iteration=mi)
print("oracle fp64", reto, [(a, b, f"{c:.6g}") for a, b, c in tr])
for fuse in (1, 0):
    with AlsContext(u, i, r, k, nU, nI) as ctx:
        ctx.set_option("fuse_start", fuse)
        ctx.set_factors(d["U0"], d["V0"])
        trace = []
        for it in range(mi):
            cu, _ = ctx.half_step("users")
            ci, rr = ctx.half_step("items")
            trace.append((cu, ci, f"{rr:.6g}"))
        U, V = ctx.get_factors()
    print("gpu fuse", fuse, trace, "relU", np.max(np.abs(U - Uo)) / np.max(np.abs(Uo)),
          "relU vs ref", np.max(np.abs(U - d["U"])) / np.max(np.abs(d["U"])))
