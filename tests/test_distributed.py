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


def run_workers(mode, fixture, nproc, tmp_path, max_iteration=200, timeout=600, skew=False,
                onepass=1):
    out = str(tmp_path / f"{mode}_{nproc}{'_skew' if skew else ''}_op{onepass}.npz")
    env = dict(os.environ, OMP_NUM_THREADS="2", MR_QUIET="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", WORKER, "--mode", mode, "--fixture", fixture,
           "--max-iteration", str(max_iteration), "--out", out, "--onepass", str(onepass)] + \
        (["--skew"] if skew else [])
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
    from movie_recommender_amd.distributed import SUM_CHUNK, entity_cost, shard_bounds
    counts = np.concatenate([np.full(1000, 500), np.full(20000, 25)])   # heavy then light
    plain = shard_bounds(counts, 2)
    cost = entity_cost(counts, 64)
    assert np.all(cost - counts == cost[0] - counts[0]) and cost[0] - counts[0] > 100
    b = shard_bounds(cost, 2)
    assert b[1] > plain[1]                 # the heavy rank takes some light users
    load = [cost[b[r]:b[r + 1]].sum() for r in range(2)]
    # one entity of imbalance, plus the rounding to a multiple of SUM_CHUNK
    # (up to SUM_CHUNK / 2 entities moved, each load by as many)
    assert abs(load[0] - load[1]) <= (SUM_CHUNK + 1) * cost.max()


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


def test_callback_transport_padded_exchange_gloo_cpu(tmp_path):
    """World size 3 on CPU: the host side of the callback transport exactly as
    the engine drives it (Engine::allgather_side) -- each rank's packed block
    at rank x maxrows of the padded table, TorchComm.allgather_rows with
    padded row boundaries, factor rows and then the bias column -- gives
    every rank every block."""
    world, maxrows, ldk = 3, 5, 8
    tab, tab_b, ret = run_workers("comm_padded", "als_dense_38x45_k5.npz", world, tmp_path)
    assert ret == world
    for r in range(world):
        blk = tab[r * maxrows * ldk:(r + 1) * maxrows * ldk]
        assert np.array_equal(blk, 1000 * r + np.arange(maxrows * ldk, dtype=np.float32))
        assert np.array_equal(tab_b[r * maxrows:(r + 1) * maxrows],
                              1000 * r + np.arange(maxrows, dtype=np.float32) + 0.5)


def test_shard_bounds_aligned_to_sum_chunk():
    """Interior boundaries at multiples of the one-pass CG's sum chunk (the
    condition for sharded == single-GPU bit for bit)."""
    from movie_recommender_amd.distributed import SUM_CHUNK, shard_bounds
    rng = np.random.default_rng(3)
    for n, world in ((103, 2), (1000, 3), (50367, 8), (9, 4)):
        b = shard_bounds(rng.integers(1, 500, n), world)
        assert b[0] == 0 and b[-1] == n and np.all(np.diff(b) >= 0)
        assert all(int(x) % SUM_CHUNK == 0 or int(x) == n for x in b[1:-1])


def test_skewed_bounds_cover_and_grow():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dist_worker import skewed_bounds
    for n, world in ((300, 3), (260, 2), (50, 8)):
        b = skewed_bounds(n, world)
        assert b[0] == 0 and b[-1] == n and np.all(np.diff(b) >= 0)
        assert np.diff(b)[-1] > np.diff(b)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("fixture,max_it,nproc,skew", [
    ("als_dense_300x200_k10.npz", 200, 2, False),
    ("als_dense_300x260_k64.npz", 200, 2, False),
    ("als_mlshape_k64_it4.npz", 4, 2, False),
    ("als_dense_340x300_k144.npz", 3, 2, False),
    # round 3: world 3, uneven (2^r) shards, k = 64 and 128 -- the padded
    # pack_rows -> all-gather -> unstage_rows exchange the RCCL path runs
    ("als_dense_300x260_k64.npz", 200, 3, True),
    ("als_mlshape_k64_it4.npz", 4, 3, False),
    ("als_dense_400x300_k128.npz", 200, 2, False),
    ("als_dense_400x300_k128.npz", 200, 3, True)])
def test_engine_sharded_gloo_matches_single(gpu, tmp_path, fixture, max_it, nproc, skew):
    """The real engine sharded over 2 or 3 ranks (all on cuda:0 on a one-GPU
    box; cost-balanced or deliberately uneven shards, all-reduced CG scalars,
    factor shards exchanged through the padded device buffers of the RCCL
    path) against the single-context run and the compiled reference's
    golden."""
    from movie_recommender_amd.engine import AlsContext
    d = load_golden(fixture)
    k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
    U, V, ret = run_workers("engine_gloo", fixture, nproc, tmp_path, max_it, skew=skew)
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
        ctx.set_option("cg_onepass", 0)   # the RCCL collectives run the two-kernel CG
        ctx.set_factors(d["U0"], d["V0"])
        ret1 = ctx.run()
        U1, V1 = ctx.get_factors()
    assert ret == ret1
    if nproc == 1:
        assert np.array_equal(U, U1) and np.array_equal(V, V1)
    assert rel_err(U, d["U"]) < 1e-5 and rel_err(V, d["V"]) < 1e-5


def _unstage_expected(world, skip, rb, maxrows, ldk, recv, recv_b, fac, bias):
    fac = fac.copy()
    bias = bias.copy() if bias is not None else None
    for s in range(world):
        if s == skip:
            continue
        n = rb[s + 1] - rb[s]
        blk = recv.reshape(world, maxrows, ldk)[s, :n]
        fac.reshape(-1, ldk)[rb[s]:rb[s] + n] = blk
        if bias is not None:
            bias[rb[s]:rb[s] + n] = recv_b.reshape(world, maxrows)[s, :n]
    return fac, bias


@pytest.mark.gpu
@pytest.mark.parametrize("ldk,with_bias", [(64, True), (128, False), (16, True)])
def test_unstage_rows_fabricated_world8(gpu, ldk, with_bias):
    """unstage_rows_kernel (the RCCL path's receive side) on a fabricated
    world = 8 receive buffer: uneven shards, two empty ones, the largest
    defining maxrows, each rank in turn the skipped (own) one -- against a
    NumPy restatement, bit for bit (a pure copy)."""
    import ctypes
    from movie_recommender_amd import _lib
    L = _lib.lib()
    world = 8
    sizes = np.array([37, 0, 5, 64, 1, 0, 23, 41])
    rb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    maxrows = int(sizes.max())
    rows = int(rb[-1])
    rng = np.random.default_rng(ldk)
    recv = rng.standard_normal(world * maxrows * ldk).astype(np.float32)
    recv_b = rng.standard_normal(world * maxrows).astype(np.float32) if with_bias else None
    fac0 = rng.standard_normal(rows * ldk).astype(np.float32)
    bias0 = rng.standard_normal(rows).astype(np.float32) if with_bias else None
    fp = lambda a: a.ctypes.data_as(_lib.FP) if a is not None else None  # noqa: E731
    for skip in range(-1, world):
        fac = fac0.copy()
        bias = bias0.copy() if with_bias else None
        _lib.check(L.mr_test_unstage_rows(0, world, skip, rb.ctypes.data_as(_lib.LLP), maxrows,
                                          ldk, fp(recv), fp(recv_b), fp(fac), fp(bias)),
                   "mr_test_unstage_rows")
        ef, eb = _unstage_expected(world, skip, rb, maxrows, ldk, recv, recv_b, fac0, bias0)
        assert np.array_equal(fac, ef)
        if with_bias:
            assert np.array_equal(bias, eb)
    # shapes the kernel cannot take are refused on the host
    bad = rb.copy()
    bad[4] = bad[3] - 1
    assert L.mr_test_unstage_rows(0, world, 0, bad.ctypes.data_as(_lib.LLP), maxrows, ldk,
                                  fp(recv), fp(recv_b), fp(fac0.copy()),
                                  fp(bias0.copy() if with_bias else None)) < 0
    assert L.mr_test_unstage_rows(0, world, 0, rb.ctypes.data_as(_lib.LLP), maxrows - 1, ldk,
                                  fp(recv), fp(recv_b), fp(fac0.copy()),
                                  fp(bias0.copy() if with_bias else None)) < 0


@pytest.mark.gpu
def test_pack_rows_matches_slice(gpu):
    """pack_rows_kernel (the send side): rows [r0, r0+n) and their bias."""
    from movie_recommender_amd import _lib
    L = _lib.lib()
    rows, ldk = 300, 64
    rng = np.random.default_rng(1)
    fac = rng.standard_normal(rows * ldk).astype(np.float32)
    bias = rng.standard_normal(rows).astype(np.float32)
    for r0, n in ((0, 300), (17, 113), (299, 1), (120, 0)):
        send = np.zeros(max(n, 1) * ldk, np.float32)
        send_b = np.zeros(max(n, 1), np.float32)
        _lib.check(L.mr_test_pack_rows(0, rows, ldk, fac.ctypes.data_as(_lib.FP),
                                       bias.ctypes.data_as(_lib.FP), r0, n,
                                       send.ctypes.data_as(_lib.FP),
                                       send_b.ctypes.data_as(_lib.FP)), "mr_test_pack_rows")
        assert np.array_equal(send[:n * ldk], fac[r0 * ldk:(r0 + n) * ldk])
        assert np.array_equal(send_b[:n], bias[r0:r0 + n])


@pytest.mark.gpu
@pytest.mark.parametrize("fixture,max_it,nproc,skew", [
    ("als_dense_300x260_k64.npz", 200, 2, False),
    ("als_mlshape_k64_it4.npz", 4, 2, False),
    ("als_dense_200x150_k32.npz", 200, 3, True),
    ("als_dense_400x300_k128.npz", 200, 3, False)])
def test_engine_peer_scalars_match_collective(gpu, tmp_path, fixture, max_it, nproc, skew):
    """The CG scalars through the peer all-reduce (exchange buffers mapped by
    hipIpcOpenMemHandle between the rank processes, here all on one GPU;
    each rank sums the records in rank order) against the same sharded run
    with the scalars through the gloo callbacks: at world 2 bit for bit (a
    sum of two terms is the same in either order), at world 3 within the
    reference tolerance; both against the compiled reference's golden."""
    d = load_golden(fixture)
    # the two-kernel CG (cg_onepass 0) with either transport of the scalars
    Up, Vp, retp = run_workers("engine_peer", fixture, nproc, tmp_path, max_it, skew=skew,
                               onepass=0)
    Ug, Vg, retg = run_workers("engine_gloo", fixture, nproc, tmp_path, max_it, skew=skew,
                               onepass=0)
    assert retp == retg == int(d["ret"])
    if nproc == 2:
        assert np.array_equal(Up, Ug) and np.array_equal(Vp, Vg)
    else:
        assert rel_err(Up, Ug) < 1e-5 and rel_err(Vp, Vg) < 1e-5
    assert rel_err(Up, d["U"]) < 1e-5 and rel_err(Vp, d["V"]) < 1e-5
    # the one-pass CG (the default with peer scalars: one reduction of three
    # sums per CG iteration) against the golden
    U1, V1, ret1 = run_workers("engine_peer", fixture, nproc, tmp_path, max_it, skew=skew,
                               onepass=1)
    assert ret1 == int(d["ret"])
    assert rel_err(U1, d["U"]) < 1e-5 and rel_err(V1, d["V"]) < 1e-5
    if int(d["k"]) <= 64:
        # one-pass CG with its fused start: every cross-entity sum is an exact
        # integer sum (kernels.hip "Order-independent CG sums"), so the
        # sharded run reproduces the single-GPU run bit for bit
        from movie_recommender_amd.engine import AlsContext
        with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], int(d["k"]),
                        int(d["num_users"]), int(d["num_items"])) as ctx:
            ctx.set_option("cg_onepass", 1)
            ctx.set_factors(d["U0"], d["V0"])
            ret_s = ctx.run(0.01, max_it)
            Us, Vs = ctx.get_factors()
        assert ret_s == ret1
        assert np.array_equal(Us, U1) and np.array_equal(Vs, V1), (rel_err(U1, Us), rel_err(V1, Vs))


@pytest.mark.gpu
@pytest.mark.parametrize("nproc", [2, 3])
def test_peer_setup_failure_falls_back_on_every_rank(gpu, tmp_path, nproc):
    """one rank's mr_als_set_peer fails -> every rank (including
    those whose own set_peer succeeded) switches back to the collective
    scalars, so all ranks issue the same launches; the run completes on the
    collective path and matches the compiled reference's golden."""
    fixture = "als_dense_300x260_k64.npz"
    d = load_golden(fixture)
    U, V, ret = run_workers("peer_fail_setup", fixture, nproc, tmp_path, 200)
    assert ret == int(d["ret"])
    assert rel_err(U, d["U"]) < 1e-5 and rel_err(V, d["V"]) < 1e-5


@pytest.mark.gpu
def test_peer_missing_rank_fails_within_timeout(gpu, tmp_path):
    """A rank that never arrives: the peer all-reduce gives up after
    MR_OPT_PEER_TIMEOUT_S (3 s here) and the solve fails with an error the
    Python layer raises -- bounded, no hang (the process exits normally)."""
    fixture = "als_dense_300x260_k64.npz"
    out = str(tmp_path / "missing.npz")
    env = dict(os.environ, OMP_NUM_THREADS="2", MR_QUIET="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", WORKER, "--mode",
           "peer_missing_rank", "--fixture", fixture, "--out", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    with np.load(out) as z:
        el, msg = float(z["elapsed"]), str(z["msg"])
    assert "timed out" in msg, msg
    assert 2.5 < el < 30.0, el
