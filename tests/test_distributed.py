"""Sharded (multi-process) ALS: partitioning, the distributed algorithm on CPU
(gloo, world size 2) against the single-process oracle, and on the GPU the
real engine across 2 ranks (gloo callbacks) and with its RCCL communicator."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, load_golden, rel_err

WORKER = os.path.join(ROOT, "tests", "dist_worker.py")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_workers(mode, fixture, nproc, tmp_path, max_iteration=200, timeout=600):
    out = str(tmp_path / f"{mode}_{nproc}.npz")
    env = dict(os.environ, OMP_NUM_THREADS="2", MR_QUIET="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", WORKER, "--mode", mode, "--fixture", fixture,
           "--max-iteration", str(max_iteration), "--out", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    with np.load(out) as d:
        return d["U"], d["V"], int(d["ret"])


def test_shard_bounds_balanced_and_complete():
    from movie_recommender_amd.distributed import shard_bounds
    rng = np.random.default_rng(0)
    counts = rng.zipf(1.5, 10_000) % 1000
    for world in (1, 2, 3, 8):
        b = shard_bounds(counts, world)
        assert b[0] == 0 and b[-1] == len(counts) and np.all(np.diff(b) >= 0)
        load = [counts[b[r]:b[r + 1]].sum() for r in range(world)]
        assert sum(load) == counts.sum()
        assert max(load) <= counts.sum() / world + counts.max()


def test_entity_cost_balances_gram_and_cg_work():
    """Light entities cost a CG pass each: with the per-entity term the
    rank holding many light users gets fewer of them than a pure rating
    balance would give it."""
    from movie_recommender_amd.distributed import entity_cost, shard_bounds
    counts = np.concatenate([np.full(1000, 500), np.full(20000, 25)])   # heavy then light
    plain = shard_bounds(counts, 2)
    cost = entity_cost(counts, 64)
    assert np.all(cost - counts == cost[0] - counts[0]) and cost[0] - counts[0] > 100
    b = shard_bounds(cost, 2)
    assert b[1] > plain[1]                 # the heavy rank takes some light users
    load = [cost[b[r]:b[r + 1]].sum() for r in range(2)]
    assert abs(load[0] - load[1]) <= cost.max()


def test_shard_views_partition_every_rating():
    from movie_recommender_amd.distributed import shard_views
    d = load_golden("als_mlshape_k10_it2.npz")
    u, i, r = d["user_ids"], d["item_ids"], d["ratings"]
    nU, nI = int(d["num_users"]), int(d["num_items"])
    world = 3
    nu = ni = 0
    for rank in range(world):
        (u0, u1), (i0, i1), uv, iv, ub, ib = shard_views(u, i, r, nU, nI, rank, world)
        assert np.all((uv[0] >= u0) & (uv[0] < u1)) and np.all((iv[1] >= i0) & (iv[1] < i1))
        nu += len(uv[0])
        ni += len(iv[0])
    assert nu == len(r) and ni == len(r)


@pytest.mark.parametrize("fixture,max_it", [("als_dense_300x200_k10.npz", 200),
                                            ("als_mlshape_k10_it4.npz", 4),
                                            ("als_mlshape_k64_it2.npz", 2)])
def test_sharded_algorithm_gloo_cpu(tmp_path, fixture, max_it):
    """World size 2 on CPU: sharded normal equations + all-reduced CG scalars +
    all-gathered shards reproduce the single-process algorithm (and the
    reference golden output)."""
    from oracle import als_oracle as O
    d = load_golden(fixture)
    k = int(d["k"])
    U, V, ret = run_workers("oracle", fixture, 2, tmp_path, max_it)
    Uo, Vo, reto, _ = O.als_block(d["user_ids"], d["item_ids"], d["ratings"], k, d["U0"],
                                  d["V0"], max_iteration=max_it)
    assert ret == reto == int(d["ret"])
    # only the summation grouping of the global dot products differs; the
    # tolerance follows the reference's own thread-count spread on the fixture
    tol = max(1e-9, 20 * float(d["tc_spread"]))
    assert rel_err(U, Uo) < tol and rel_err(V, Vo) < tol
    assert rel_err(U, d["U"]) < max(1e-6, tol) and rel_err(V, d["V"]) < max(1e-6, tol)


def test_sharded_algorithm_gloo_cpu_world3(tmp_path):
    """World size 3 (uneven, cost-balanced shards; 3 all-gather pieces and a
    3-way scalar all-reduce) on CPU against the single-process algorithm."""
    from oracle import als_oracle as O
    fixture = "als_dense_300x200_k10.npz"
    d = load_golden(fixture)
    k = int(d["k"])
    U, V, ret = run_workers("oracle", fixture, 3, tmp_path, 200)
    Uo, Vo, reto, _ = O.als_block(d["user_ids"], d["item_ids"], d["ratings"], k, d["U0"],
                                  d["V0"], max_iteration=200)
    assert ret == reto == int(d["ret"])
    tol = max(1e-9, 20 * float(d["tc_spread"]))
    assert rel_err(U, Uo) < tol and rel_err(V, Vo) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("fixture,max_it", [("als_dense_300x200_k10.npz", 200),
                                            ("als_dense_300x260_k64.npz", 200),
                                            ("als_mlshape_k64_it4.npz", 4),
                                            ("als_dense_340x300_k144.npz", 3)])
def test_engine_two_ranks_gloo_matches_single(gpu, tmp_path, fixture, max_it):
    """The real engine sharded over 2 ranks (both on cuda:0 on a one-GPU box;
    cost-balanced shards, all-reduced CG scalars, all-gathered factor shards)
    against the single-context run and the compiled reference's golden."""
    from movie_recommender_amd.engine import AlsContext
    d = load_golden(fixture)
    k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
    U, V, ret = run_workers("engine_gloo", fixture, 2, tmp_path, max_it)
    with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], k, nU, nI) as ctx:
        ctx.set_factors(d["U0"], d["V0"])
        ret1 = ctx.run(0.01, max_it)
        U1, V1 = ctx.get_factors()
    assert ret == ret1 == int(d["ret"])
    assert rel_err(U, U1) < 1e-5 and rel_err(V, V1) < 1e-5
    assert rel_err(U, d["U"]) < 1e-5 and rel_err(V, d["V"]) < 1e-5


@pytest.mark.gpu
def test_engine_rccl_path_matches_single(gpu, tmp_path):
    """The native RCCL communicator (one rank per available GPU; on a one-GPU
    box a single rank still runs every RCCL all-reduce / broadcast)."""
    from movie_recommender_amd.engine import AlsContext
    fixture = "als_dense_200x150_k32.npz"
    d = load_golden(fixture)
    nproc = max(1, min(2, gpu.mr_device_count()))
    U, V, ret = run_workers("engine_rccl", fixture, nproc, tmp_path)
    with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], 32, 200, 150) as ctx:
        ctx.set_factors(d["U0"], d["V0"])
        ret1 = ctx.run()
        U1, V1 = ctx.get_factors()
    assert ret == ret1
    if nproc == 1:
        assert np.array_equal(U, U1) and np.array_equal(V, V1)
    assert rel_err(U, d["U"]) < 1e-5 and rel_err(V, d["V"]) < 1e-5
