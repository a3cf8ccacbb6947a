"""Worker for the multi-process tests (launched by torch.distributed.run).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/dist_worker.py --mode oracle --fixture NAME --out F

Modes
  oracle       CPU only: the sharded ALS algorithm (rank-local normal
               equations, all-reduced CG scalars, all-gathered factor shards)
               restated with the NumPy oracle over gloo; rank 0 saves U, V, ret.
  engine_gloo  the HIP engine, one shard context per rank (all on cuda:0 when
               the box has one GPU), collectives through TorchComm callbacks
               (the same padded device exchange buffers as RCCL: pack_rows
               -> all-gather -> unstage_rows); --skew imposes uneven shards.
  engine_rccl  the HIP engine with its native RCCL communicator.
  engine_peer  engine_gloo with the CG scalars through the peer all-reduce
               (IPC-mapped exchange buffers, include/mr_als.h mr_als_set_peer).
  peer_fail_setup   engine_peer whose last rank's mr_als_set_peer fails: every
               rank must fall back to the collective scalars (peer_scalars
               False, the self-test refused as "not set up") and the run must
               still complete on them.
  peer_missing_rank engine_peer with MR_OPT_PEER_TIMEOUT_S = 3; the last rank
               never starts its solve: rank 0's run must fail (RuntimeError,
               ret -1 from the engine) within the bound instead of hanging;
               rank 0 saves the elapsed seconds and the message.
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def load(name):
    with np.load(os.path.join(HERE, "golden", name), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def oracle_sharded(d, max_iteration, rank, world):
    """Restatement of the sharded algorithm with the oracle's pieces."""
    import torch
    import torch.distributed as dist
    from oracle import als_oracle as O
    from movie_recommender_amd.distributed import shard_views

    k = int(d["k"])
    nU, nI = int(d["num_users"]), int(d["num_items"])
    u, i, r = d["user_ids"], d["item_ids"], d["ratings"]
    (u0, u1), (i0, i1), uv, iv, ub, ib = shard_views(u, i, r, nU, nI, rank, world)

    def gdot(a, b):
        t = torch.tensor([float(np.dot(a, b))], dtype=torch.float64)
        dist.all_reduce(t)
        return float(t.item())

    def allgather_rows(table, bounds, width):
        mine = torch.from_numpy(table[bounds[rank] * width: bounds[rank + 1] * width].copy())
        sizes = [int(bounds[q + 1] - bounds[q]) * width for q in range(world)]
        m = max(sizes)
        send = torch.zeros(m, dtype=torch.float64)
        send[:len(mine)] = mine
        outs = [torch.zeros(m, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(outs, send)
        for q in range(world):
            table[bounds[q] * width: bounds[q] * width + sizes[q]] = outs[q][:sizes[q]].numpy()

    U = np.array(d["U0"], np.float64)
    V = np.array(d["V0"], np.float64)
    it, old_rr = 0, 0.0
    while it < max_iteration:
        # user half-step on local users [u0, u1)
        G, c = O.gram_user(uv[0] - u0, uv[1], uv[2], V, k, u1 - u0)
        x = U[u0 * (k + 1): u1 * (k + 1)].copy()
        O.cg_normal(O.block_matvec(G), c.reshape(-1), x, 0.01, 200, dot=gdot)
        U[u0 * (k + 1): u1 * (k + 1)] = x
        allgather_rows(U, ub, k + 1)
        # item half-step on local items [i0, i1)
        G, c = O.gram_item(iv[0], iv[1] - i0, iv[2], U, k, i1 - i0)
        x = V[i0 * k: i1 * k].copy()
        _, rr = O.cg_normal(O.block_matvec(G), c.reshape(-1), x, 0.01, 200, dot=gdot)
        V[i0 * k: i1 * k] = x
        allgather_rows(V, ib, k)
        if it >= 3 and (old_rr - rr) / old_rr < 0.01:
            return U, V, it
        old_rr = rr
        it += 1
    return U, V, it


def skewed_bounds(n, world, align=1):
    """Deliberately uneven shards (rank r's share grows as 2^r): the padded
    exchange then carries mostly padding for the small ranks.  ``align``
    rounds the interior boundaries down to its multiples."""
    w = 2.0 ** np.arange(world)
    b = np.concatenate([[0], np.floor(np.cumsum(w) / w.sum() * n / align) * align])
    b = b.astype(np.int64)
    b[-1] = n
    return b


def engine_sharded(d, max_iteration, rank, world, mode, skew=False, onepass=1):
    import torch.distributed as dist
    from movie_recommender_amd.distributed import TorchComm, sharded_context
    from movie_recommender_amd.engine import device_count
    k = int(d["k"])
    dev = rank % max(1, device_count())
    comm = "rccl" if mode == "engine_rccl" else TorchComm()
    nU, nI = int(d["num_users"]), int(d["num_items"])
    # peer runs: boundaries at the sums' chunk size (distributed.SUM_CHUNK),
    # which the bitwise sharded == single-GPU test needs; gloo runs keep
    # arbitrary ones
    al = 4 if mode == "engine_peer" else 1
    bounds = (skewed_bounds(nU, world, al), skewed_bounds(nI, world, al)) if skew else None
    ctx = sharded_context(d["user_ids"], d["item_ids"], d["ratings"], k, nU, nI, dev, comm,
                          bounds=bounds, scalars="peer" if mode == "engine_peer" else "collective")
    if mode == "engine_peer" and not ctx.peer_scalars:
        raise RuntimeError("peer scalar all-reduce was not set up (self-test failed)")
    ctx.set_option("cg_onepass", onepass)
    ctx.set_factors(d["U0"], d["V0"])
    ret = ctx.run(0.01, max_iteration)
    U, V = ctx.get_factors()
    ctx.close()
    dist.barrier()
    return U, V, ret


def peer_fail_setup(d, max_iteration, rank, world):
    import torch.distributed as dist
    from movie_recommender_amd import _lib
    from movie_recommender_amd.distributed import TorchComm, sharded_context
    from movie_recommender_amd.engine import device_count
    k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
    dev = rank % max(1, device_count())
    ctx = sharded_context(d["user_ids"], d["item_ids"], d["ratings"], k, nU, nI, dev,
                          TorchComm(), scalars="peer", _fail_set_peer=(rank == world - 1))
    assert not ctx.peer_scalars, "a rank kept the peer scalars after another rank failed"
    assert _lib.lib().mr_als_peer_selftest(ctx._h) < 0, "peer_on still set after the fallback"
    assert "not set up" in _lib.last_error(), _lib.last_error()
    ctx.set_factors(d["U0"], d["V0"])
    ret = ctx.run(0.01, max_iteration)
    U, V = ctx.get_factors()
    ctx.close()
    dist.barrier()
    return U, V, ret


def peer_missing_rank(d, rank, world, out):
    import time
    import torch.distributed as dist
    from movie_recommender_amd.distributed import TorchComm, sharded_context
    from movie_recommender_amd.engine import device_count
    k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
    dev = rank % max(1, device_count())
    ctx = sharded_context(d["user_ids"], d["item_ids"], d["ratings"], k, nU, nI, dev,
                          TorchComm(), scalars="peer")
    assert ctx.peer_scalars, "peer all-reduce was not set up"
    ctx.set_option("peer_timeout_s", 3.0)
    ctx.set_factors(d["U0"], d["V0"])
    dist.barrier()
    if rank == world - 1:
        # the missing rank: never enters the solve; waits for rank 0's verdict
        dist.barrier()
        ctx.close()
        return
    t0 = time.perf_counter()
    msg = ""
    try:
        ctx.run(0.01, 3)
    except RuntimeError as e:
        msg = str(e)
    el = time.perf_counter() - t0
    if rank == 0:
        np.savez(out, elapsed=el, msg=np.array(msg))
    dist.barrier()
    ctx.close()


def comm_padded(rank, world):
    """The callback transport's host side on generic row tables: a table of
    world x maxrows rows of ldk floats (this rank's rows at rank x maxrows)
    and a 1-float-per-row column, through TorchComm's allgather_rows with
    row boundaries r x maxrows; returns the gathered tables for rank 0 to
    compare with the expected blocks.  (The engine itself passes ONE row per
    rank, ag_block_floats(maxrows, ldk, with_bias) floats wide, row_begin[r]
    = r -- the world 2 / 3 engine tests drive that layout.)"""
    import ctypes
    from movie_recommender_amd.distributed import TorchComm
    comm = TorchComm()
    maxrows, ldk = 5, 8
    tab = np.full(world * maxrows * ldk, -1.0, np.float32)
    tab_b = np.full(world * maxrows, -1.0, np.float32)
    mine = slice(rank * maxrows * ldk, (rank + 1) * maxrows * ldk)
    tab[mine] = 1000 * rank + np.arange(maxrows * ldk)
    tab_b[rank * maxrows:(rank + 1) * maxrows] = 1000 * rank + np.arange(maxrows) + 0.5
    prb = np.arange(world + 1, dtype=np.int64) * maxrows
    fp = ctypes.POINTER(ctypes.c_float)
    llp = ctypes.POINTER(ctypes.c_longlong)
    rc1 = comm.struct.allgather_rows(None, tab.ctypes.data_as(fp), ldk,
                                     prb.ctypes.data_as(llp), world)
    rc2 = comm.struct.allgather_rows(None, tab_b.ctypes.data_as(fp), 1,
                                     prb.ctypes.data_as(llp), world)
    assert rc1 == 0 and rc2 == 0, comm.errors
    return tab, tab_b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", required=True)
    ap.add_argument("--fixture", required=True)
    ap.add_argument("--max-iteration", type=int, default=200)
    ap.add_argument("--out", required=True)
    ap.add_argument("--skew", action="store_true", help="uneven shard boundaries")
    ap.add_argument("--onepass", type=int, default=1, help="engine option cg_onepass")
    a = ap.parse_args()
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    d = load(a.fixture)
    if a.mode == "peer_missing_rank":
        peer_missing_rank(d, rank, world, a.out)
        dist.barrier()
        dist.destroy_process_group()
        return
    if a.mode == "comm_padded":
        U, V = comm_padded(rank, world)
        ret = world
    elif a.mode == "peer_fail_setup":
        U, V, ret = peer_fail_setup(d, a.max_iteration, rank, world)
    elif a.mode == "oracle":
        U, V, ret = oracle_sharded(d, a.max_iteration, rank, world)
    else:
        U, V, ret = engine_sharded(d, a.max_iteration, rank, world, a.mode, a.skew, a.onepass)
    if rank == 0:
        np.savez(a.out, U=U, V=V, ret=ret)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
