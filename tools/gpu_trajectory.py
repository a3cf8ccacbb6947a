"""The engine's CG trajectory on the bench workload, several starts (GPU).

    python tools/gpu_trajectory.py [--seeds 0,1,2,3,4] [--iterations 25] [--k 64]
                                   [--opt NAME=VALUE ...] [--out F]

For each seed: the bench data (ML-full shape, cached synthetic set), start
``RandomState(seed)`` U0 then V0 (the order of ``cpp/python/cpp_ls.py:147-148``,
as ``tools/ref_trajectory.py`` uses for the compiled reference), then
``--iterations`` ALS iterations one at a time, recording each half-step's CG
iteration count and the item side's final rr.  Prints one JSON line per
seed.  Compared with the reference's trajectories (profiles/r04/
ref_trajectory_*.jsonl) it tells a systematic difference in CG counts from
the chaotic draw of one start.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_data  # noqa: E402
from movie_recommender_amd.engine import AlsContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2,3,4")
    ap.add_argument("--iterations", type=int, default=25)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rs = load_data("ml-full", a.k)
    outs = []
    with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, a.k, rs.num_users,
                    rs.num_items) as ctx:
        for o in a.opt:
            name, val = o.split("=")
            ctx.set_option(name, float(val))
        for seed in (int(s) for s in a.seeds.split(",")):
            rng = np.random.RandomState(seed)
            U0 = rng.uniform(-1, 1, rs.num_users * (a.k + 1))
            V0 = rng.uniform(-1, 1, rs.num_items * a.k)
            ctx.set_factors(U0, V0)
            tr = []
            for it in range(a.iterations):
                cu, ru = ctx.half_step("users")
                ci, ri = ctx.half_step("items")
                tr.append([cu, ci, ri])
            d = {"seed": seed, "k": a.k, "opts": a.opt, "cg_per_iteration": tr,
                 "window_6_25": [sum(x[0] for x in tr[5:25]) / max(1, len(tr[5:25])),
                                 sum(x[1] for x in tr[5:25]) / max(1, len(tr[5:25]))]}
            print(json.dumps(d), flush=True)
            outs.append(d)
    if a.out:
        with open(a.out, "w") as f:
            for d in outs:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
