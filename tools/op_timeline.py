"""Timeline of one one-pass CG launch (needs a library built with
-DMR_OP_PROF=1, tools/build_var.sh; MR_LIB_PATH selects it): where the fixed
cost of a CG iteration goes at shard sizes -- block start spread, the last
block's entities, the bin flush, the arrival, and the last block's tail
(bin collection, state, publish).  Times in microseconds from the first
block's start, s_memrealtime (100 MHz).

    python tools/op_timeline.py [--k 64] [--shard R/N] [--side users] [--m 8]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_data  # noqa: E402
from movie_recommender_amd import _lib  # noqa: E402
from movie_recommender_amd.engine import AlsContext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--shard", default=None)
ap.add_argument("--side", default="users")
ap.add_argument("--m", type=int, default=8)
ap.add_argument("--resident", action="store_true",
                help="the resident solve's iteration t0 + 2: per block start / chunks "
                     "done / arrival / broadcast seen, the last block's collect / "
                     "compute / generation store")
a = ap.parse_args()
rs = load_data("ml-full", a.k)
rng = np.random.RandomState(0)
U0 = rng.uniform(-1, 1, rs.num_users * (a.k + 1))
V0 = rng.uniform(-1, 1, rs.num_items * a.k)
if a.shard:
    from movie_recommender_amd.distributed import shard_views
    R, N = (int(x) for x in a.shard.split("/"))
    ur, ir, uv, iv, _, _ = shard_views(rs.user_ids, rs.item_ids, rs.ratings, rs.num_users,
                                       rs.num_items, R, N, k=a.k)
    ctx = AlsContext(uv[0], uv[1], uv[2], a.k, rs.num_users, rs.num_items, user_range=ur,
                     item_range=ir, item_view=iv)
else:
    ctx = AlsContext(rs.user_ids, rs.item_ids, rs.ratings, a.k, rs.num_users, rs.num_items)
L = _lib.lib()
fn = L.mr_debug_op_timeline
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
n = 8 + 4 * 4096
buf = (ctypes.c_longlong * n)()
out = {"k": a.k, "shard": a.shard, "side": a.side, "m": a.m}
with ctx:
    ctx.set_option("cg_resident", 1 if a.resident else 0)
    ctx.set_factors(U0, V0)
    for _ in range(2):
        ctx.half_step(a.side, float("-inf"), a.m)   # warm, fixed CG count
    got = fn(buf, n)
    assert got > 0, "library not built with -DMR_OP_PROF=1"
t = np.frombuffer(buf, dtype=np.int64).copy()
blk = t[8:].reshape(-1, 4)
used = blk[:, 0] > 0
blk = blk[used]
t0 = blk[:, 0].min()
us = lambda x: round(float(x - t0) / 100.0, 2)  # noqa: E731  (100 MHz ticks)
out["blocks"] = int(used.sum())
if a.resident:
    q = lambda col: {"min": us(blk[:, col].min()), "median": us(np.median(blk[:, col])),  # noqa
                     "p90": us(np.percentile(blk[:, col], 90)), "max": us(blk[:, col].max())}
    out.update({"chunks_done_us": q(1), "arrived_us": q(2), "broadcast_seen_us": q(3),
                "last_block_us": {"collect_start": us(t[0]), "collected": us(t[1]),
                                  "computed": us(t[2]), "gen_stored": us(t[3])}})
    print(json.dumps(out))
    sys.exit(0)
out["entry_us"] = {"min": 0.0, "median": us(np.median(blk[:, 0])), "max": us(blk[:, 0].max())}
out["entities_done_us"] = {"min": us(blk[:, 1].min()), "median": us(np.median(blk[:, 1])),
                           "max": us(blk[:, 1].max())}
out["flushed_us"] = {"median": us(np.median(blk[:, 2])), "max": us(blk[:, 2].max())}
out["last_block_us"] = {"tail_start": us(t[0]), "collected": us(t[1]), "state": us(t[2]),
                        "published": us(t[3])}
print(json.dumps(out))
