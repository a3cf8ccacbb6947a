"""Device-side latency of the peer all-reduce of the CG scalars
(include/mr_als.h mr_als_peer_latency), measured with N processes on ONE GPU
(IPC mapping of the same device: no xGMI hop, so a lower bound for the
8-GPU node) -- the number DESIGN.md's collective model uses.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/peer_latency.py [--iters 20000]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch.distributed as dist  # noqa: E402

from movie_recommender_amd import _lib  # noqa: E402
from movie_recommender_amd.distributed import attach_peer_scalars  # noqa: E402
from movie_recommender_amd.engine import AlsContext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20000)
a = ap.parse_args()
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
u = np.array([0, 1], np.int32)
i = np.array([0, 1], np.int32)
with AlsContext(u, i, np.array([1.0, 2.0]), 4, 2, 2, device=0) as ctx:
    if not attach_peer_scalars(ctx, rank, world):
        raise SystemExit("peer all-reduce could not be set up")
    res = []
    for rep in range(3):
        us = ctypes.c_double(0.0)
        dist.barrier()
        _lib.check(_lib.lib().mr_als_peer_latency(ctx._h, a.iters, ctypes.byref(us)),
                   "mr_als_peer_latency")
        res.append(us.value)
    out = [None] * world
    dist.all_gather_object(out, res)
if rank == 0:
    print(json.dumps({"metric": "peer all-reduce latency (device, one value)", "unit": "us",
                      "world": world, "iters": a.iters,
                      "us_per_reduction_by_rank": out,
                      "value": min(max(r[j] for r in out) for j in range(3)),
                      "note": "all ranks on one GPU (IPC-mapped uncached exchange buffers); "
                              "over xGMI each remote record store adds the link latency"}))
dist.destroy_process_group()
