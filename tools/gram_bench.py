"""Microbenchmark of the Gram (normal-equation) kernels and one CG half-step
on the bench workload.  python tools/gram_bench.py [--k 64] [--reps 5]
(the Gram runs the bf16x3 matrix-core loop)."""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--shape", default="ml-full")
ap.add_argument("--chunk", type=int, default=None)
ap.add_argument("--cg", type=int, default=0, help="also run this many ALS iterations")
a = ap.parse_args()
cache = f"/tmp/mr_bench_{a.shape}_k{a.k}_{synth.DATA_SEED}.npz"
if os.path.exists(cache):
    d = np.load(cache)
    rs = synth.RatingSet(d["u"], d["i"], d["r"], int(d["nu"]), int(d["ni"]), a.k)
else:
    rs = synth.movielens_like(a.shape, a.k)
    np.savez(cache, u=rs.user_ids, i=rs.item_ids, r=rs.ratings, nu=rs.num_users, ni=rs.num_items)
k = a.k
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * k)
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items,
                gram_chunk=a.chunk) as ctx:
    ctx.set_factors(U0, V0)
    ctx.build_normal_equations("users"); ctx.build_normal_equations("items")
    ctx.reset_stats(); ctx.set_timing(True)
    for _ in range(a.reps):
        ctx.build_normal_equations("users")
        ctx.build_normal_equations("items")
    st = ctx.stats()
    N = rs.n
    out = {"G": os.environ.get("MR_GRAM_G", "default"), "k": k, "N": N}
    for side, nE in (("users", rs.num_users), ("items", rs.num_items)):
        ms = st["kernel_ms"]["gram_" + side] / st["kernel_launches"]["gram_" + side]
        K = k + 1 if side == "users" else k
        out[side + "_ms"] = round(ms, 4)
        out[side + "_algTF"] = round(N * (2.0 * K * K + 2 * K) / (ms * 1e-3) / 1e12, 1)
        nb = (k + 15) // 16
        out[side + "_mfmaTF"] = round(N * nb * (nb + 1) / 2 * 512 / (ms * 1e-3) / 1e12, 1)
    out["slab_ms"] = round(st["kernel_ms"]["slab_reduce"] / max(1, st["kernel_launches"]["slab_reduce"]), 4)
    if a.cg:
        ctx.reset_stats()
        ctx.iterate(a.cg)
        st = ctx.stats()
        for c in ("matvec_users", "matvec_items", "cg_update", "cg_control"):
            n = max(1, st["kernel_launches"][c])
            out[c + "_us"] = round(st["kernel_ms"][c] / n * 1e3, 2)
        out["cg_its"] = (st["cg_users_total"], st["cg_items_total"])
    print(json.dumps(out), flush=True)
