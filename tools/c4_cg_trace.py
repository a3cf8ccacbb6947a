"""Diagnostic: the engine's first users CG solve at C4 (ML-full shape, k = 128)
against the oracle's fp64 CG on the GPU's own normal equations, iteration by
iteration (engine: half_step with max_iteration m from the same start; oracle:
one run recording rr after every iteration)."""
import sys, os, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from movie_recommender_amd import synth
from movie_recommender_amd.engine import AlsContext

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
side = sys.argv[2] if len(sys.argv) > 2 else "users"
rs = synth.movielens_like("ml-full", k)
rng = np.random.default_rng(0)
U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * k)
E, K = (rs.num_users, k + 1) if side == "users" else (rs.num_items, k)
out = {"k": k, "side": side, "engine": {}, "oracle": []}
with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items) as ctx:
    ctx.set_factors(U0, V0)
    ctx.build_normal_equations(side)
    G, c = ctx.normal_equations(side, np.arange(E, dtype=np.int32))
    for m in list(range(0, 12)) + [16, 20, 24, 32, 40, 48, 64, 80, 200]:
        ctx.set_factors(U0, V0)
        its, rr = ctx.half_step(side, 0.01, m)
        out["engine"][m] = (its, rr)
c = c.reshape(-1)
x = (U0 if side == "users" else V0).astype(np.float32)
mv = lambda v: np.matmul(G, np.asarray(v, np.float64).reshape(E, K, 1)).reshape(-1)
r = mv(x) - c
p = -r
rr = float(np.dot(r, r))
out["oracle"].append((0, rr))
fails = 0
for it in range(200):
    if rr < 1e-6:
        break
    Ap = mv(p)
    alpha = rr / float(np.dot(p, Ap))
    x += alpha * p
    r += alpha * Ap
    rr2 = float(np.dot(r, r))
    beta = rr2 / rr
    fails = fails + 1 if beta > 0.99 else 0
    out["oracle"].append((it + 1, rr2, beta))
    if fails >= 2:
        break
    rr = rr2
    p = -r + beta * p
for m, (its, rre) in out["engine"].items():
    o = out["oracle"][min(m, len(out["oracle"]) - 1)]
    print(f"m={m:3d} engine its={its:3d} rr={rre:.10e}  oracle rr({o[0]})={o[1]:.10e}  rel={abs(rre - o[1]) / o[1]:.2e}")
print("oracle stop at", out["oracle"][-1])
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open(f"gpurun_out/c4_cg_trace_{side}_k{k}.json", "w"))
