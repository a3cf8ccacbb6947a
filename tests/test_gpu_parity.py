"""GPU parity: the HIP path (through the C ABI) against the compiled
reference's golden vectors and the CPU oracle.

Tolerances (fp32 normal equations, fp64 CG vectors r / p / q and scalars,
products G p accumulated in fp64; north_star: "within 1e-5 relative"):
  * dense golden fixtures (G2, k = 3 .. 128):  max|x - ref| / max|ref| <= 1e-5,
    same `ret`
  * MovieLens-shaped sparse fixtures (G3, k = 10, 32, 64; 40-100 CG iterations
    per half-step): <= 1e-5, same `ret`
  * general CG least squares (fp64 on the GPU): <= 1e-9, same iterations
  * Gram kernel vs fp64 NumPy Gram on sampled entities: <= 2e-5 relative to
    the block's largest entry
"""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden, rel_err

pytestmark = pytest.mark.gpu

DENSE = ["als_dense_38x45_k5.npz", "als_dense_40x45_k3.npz",
         "als_dense_300x200_k10.npz", "als_dense_200x150_k32.npz",
         "als_dense_60x50_k32_it3.npz", "als_dense_300x260_k64.npz",
         "als_dense_400x300_k128.npz", "als_dense_340x300_k144.npz",
         "als_dense_120x100_k24.npz"]
MLSHAPE = ["als_mlshape_k10_it2.npz", "als_mlshape_k10_it4.npz",
           "als_mlshape_k32_it2.npz", "als_mlshape_k32_it4.npz",
           "als_mlshape_k64_it2.npz", "als_mlshape_k64_it4.npz"]
# headline-k fixtures: NB = 4 / 8 block GEMV and the fused CG start; k = 144
# runs the streamed large-k Gram / GEMV (split work items at chunk 64)
HEADLINE = ["als_dense_60x50_k32_it3.npz", "als_dense_300x260_k64.npz",
            "als_dense_400x300_k128.npz", "als_mlshape_k64_it4.npz",
            "als_dense_340x300_k144.npz"]


def max_iteration_of(name, d):
    if "max_iteration" in d:
        return int(d["max_iteration"])
    if "_it" in name:
        return int(name.split("_it")[1].split(".")[0])
    return 200


def tolerance_of(d):
    """1e-5 (north_star), or twice the reference's own thread-count spread on
    a fixture where that is larger (the ill-conditioned 60 x 50, k = 32 case:
    6.2e-4 between 1 and 8 threads)."""
    return max(1e-5, 2 * float(d["tc_spread"]))


def abi_als(L, d, max_iteration=200, min_r_decrease=0.01):
    """Call als_from_python exactly as the reference wrapper does, but with the
    fixture's initial factors."""
    from movie_recommender_amd import _lib
    u = np.ascontiguousarray(d["user_ids"], np.int32)
    i = np.ascontiguousarray(d["item_ids"], np.int32)
    r = np.ascontiguousarray(d["ratings"], np.float64)
    U = np.array(d["U0"], np.float64)
    V = np.array(d["V0"], np.float64)
    k = int(d["k"])
    ret = L.als_from_python(u.ctypes.data_as(_lib.IP), i.ctypes.data_as(_lib.IP), len(r),
                            r.ctypes.data_as(_lib.DP), k, len(U), U.ctypes.data_as(_lib.DP),
                            len(V), V.ctypes.data_as(_lib.DP), min_r_decrease,
                            max_iteration, 1)
    assert ret >= 0, _lib.last_error()
    return U, V, ret


@pytest.mark.parametrize("name", DENSE)
def test_als_dense_golden(gpu, name):
    d = load_golden(name)
    U, V, ret = abi_als(gpu, d, max_iteration=max_iteration_of(name, d))
    assert ret == int(d["ret"])
    tol = tolerance_of(d)
    assert rel_err(U, d["U"]) <= tol, rel_err(U, d["U"])
    assert rel_err(V, d["V"]) <= tol, rel_err(V, d["V"])


@pytest.mark.parametrize("name", MLSHAPE)
def test_als_mlshape_golden(gpu, name):
    d = load_golden(name)
    U, V, ret = abi_als(gpu, d, max_iteration=max_iteration_of(name, d))
    assert ret == int(d["ret"])
    tol = tolerance_of(d)
    assert rel_err(U, d["U"]) <= tol, rel_err(U, d["U"])
    assert rel_err(V, d["V"]) <= tol, rel_err(V, d["V"])


@pytest.mark.parametrize("name", HEADLINE)
@pytest.mark.parametrize("chunk,fuse,onepass", [(2048, 1, 1), (64, 1, 1), (2048, 0, 1),
                                                (2048, 1, 0), (64, 1, 0), (2048, 0, 0)])
def test_headline_paths_golden(gpu, name, chunk, fuse, onepass):
    """Every CG start path against the compiled reference at k = 32 / 64 /
    128: the Gram-epilogue start (fuse 1), the start of split entities after
    slab_reduce (chunk 64 splits every entity), and the unfused reference
    order (fuse 0: x -> matvec -> INIT update); each with the one-pass CG
    iteration (cg_onepass 1, the default) and with matvec + update (0).
    Every launch-ahead level (MR_OPT_CG_SPECULATE 0, 1, 2) must give
    identical CG counts and bitwise-identical factors."""
    from movie_recommender_amd.engine import AlsContext
    from movie_recommender_amd import _lib
    d = load_golden(name)
    k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
    mi = max_iteration_of(name, d)
    outs = []
    try:
        for spec in (1, 0, 2):
            with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], k, nU, nI,
                            gram_chunk=chunk) as ctx:
                ctx.set_option("fuse_start", fuse)
                ctx.set_option("cg_speculate", spec)
                ctx.set_option("cg_onepass", onepass)
                ctx.set_factors(d["U0"], d["V0"])
                ret = ctx.run(0.01, mi)
                st = ctx.stats()
                outs.append((ctx.get_factors(), ret, st["cg_users_total"], st["cg_items_total"]))
    finally:
        _lib.check(_lib.lib().mr_set_gram_chunk(2048), "reset chunk")
    (U, V), ret, cu, ci = outs[0]
    assert ret == int(d["ret"])
    tol = tolerance_of(d)
    assert rel_err(U, d["U"]) <= tol, rel_err(U, d["U"])
    assert rel_err(V, d["V"]) <= tol, rel_err(V, d["V"])
    for (U2, V2), ret2, cu2, ci2 in outs[1:]:   # launch-ahead levels 0 and 2
        assert (ret2, cu2, ci2) == (ret, cu, ci)
        assert np.array_equal(U, U2) and np.array_equal(V, V2)


def test_cg_least_squares_golden(gpu):
    from movie_recommender_amd import _lib
    d = load_golden("cg_dense_200x50.npz")
    x = np.array(d["x0"], np.float64)
    rr = ctypes.c_double(0)
    rp = np.ascontiguousarray(d["row_ptr"], np.int32)
    ci = np.ascontiguousarray(d["col_idx"], np.int32)
    v = np.ascontiguousarray(d["vals"], np.float64)
    b = np.ascontiguousarray(d["b"], np.float64)
    for fn in (gpu.cg_least_squares_from_python, gpu.cg_least_squares2_from_python):
        x = np.array(d["x0"], np.float64)
        it = fn(len(rp) - 1, int(d["ncols"]), rp.ctypes.data_as(_lib.IP),
                ci.ctypes.data_as(_lib.IP), v.ctypes.data_as(_lib.DP), len(b),
                b.ctypes.data_as(_lib.DP), len(x), x.ctypes.data_as(_lib.DP), 0.01, 200,
                ctypes.byref(rr))
        assert it == int(d["iterations"])
        assert rel_err(x, d["x"]) <= 1e-9
        assert abs(rr.value - float(d["final_rr"])) <= 1e-6 * max(1.0, float(d["final_rr"]))


def test_reference_ffi_tests_port(gpu):
    """cpp/python/cpp_ls_test.py:5-147 through the drop-in module, seeded."""
    import random
    from movie_recommender_amd import cpp_ls
    numpy_state = np.random.get_state()
    try:
        np.random.seed(0)
        random.seed(0)
        assert cpp_ls.has_dll_loaded()
        # test_cg_least_squares
        A = np.random.uniform(-1, 1, (200, 50))
        x_real = np.random.uniform(-1, 1, (50, 1))
        b = A.dot(x_real) + np.random.normal(0, 0.1, (200, 1))
        rows, cols = np.nonzero(A)
        rp = np.zeros(201, np.int32)
        np.cumsum(np.bincount(rows, minlength=200), out=rp[1:])
        x, it, rr = cpp_ls.cg_least_squares(rp, cols.astype(np.int32), A[rows, cols], 50, b)
        assert np.sum(np.abs(x_real - x)) / 50 < 0.1
        # test_als (k=5, all users rate all items, 80 % train)
        from movie_recommender_amd import synth
        u, i, r, tu, ti, tr = synth.dense_fixture(38, 45, 5, 0.8, seed=0)
        U, V, its = cpp_ls.als(u, i, r, 5, 38, 45)
        from oracle.als_oracle import predict
        assert np.mean(np.abs(predict(U, V, tu, ti, 5) - tr)) < 0.15
    finally:
        np.random.set_state(numpy_state)


def test_engine_matches_abi_and_is_deterministic(gpu):
    from movie_recommender_amd.engine import AlsContext
    d = load_golden("als_dense_300x200_k10.npz")
    U1, V1, ret1 = abi_als(gpu, d)
    outs = []
    for _ in range(2):
        with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], 10, 300, 200) as ctx:
            ctx.set_factors(d["U0"], d["V0"])
            ret = ctx.run()
            outs.append((ctx.get_factors(), ret))
    (U2, V2), ret2 = outs[0]
    (U3, V3), ret3 = outs[1]
    assert ret1 == ret2 == ret3
    assert np.array_equal(U1, U2) and np.array_equal(V1, V2)
    assert np.array_equal(U2, U3) and np.array_equal(V2, V3)   # bitwise reproducible


def test_replay_from_snapshot_is_bitwise_identical(gpu):
    """A set -> get factor round trip is exact and replays of the same steps
    from one snapshot are bitwise identical, with and without per-launch
    timing events (bench.py's event-free pass relies on this).  Regression:
    pageable DMA staging once returned stale factor data (xfer.hip)."""
    from movie_recommender_amd import synth
    from movie_recommender_amd.engine import AlsContext
    k = 64
    rs = synth.movielens_like("ml-full", k, scale=0.02)
    rng = np.random.RandomState(0)
    U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
    V0 = rng.uniform(-1, 1, rs.num_items * k)
    with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users,
                    rs.num_items) as ctx:
        ctx.set_factors(U0, V0)
        ctx.iterate(2)
        snap = tuple(a.copy() for a in ctx.get_factors())
        for _ in range(3):
            ctx.set_factors(*snap)
            U, V = ctx.get_factors()
            assert np.array_equal(U, snap[0]) and np.array_equal(V, snap[1])
        outs = []
        for timing in (True, False, True, False):
            ctx.set_factors(*snap)
            ctx.reset_stats()
            ctx.set_timing(timing)
            ctx.iterate(3)
            st = ctx.stats()
            outs.append((ctx.get_factors(), st["cg_users_total"], st["cg_items_total"]))
        ctx.set_timing(False)
    (U1, V1), cu, ci = outs[0]
    for (U, V), cu2, ci2 in outs[1:]:
        assert (cu2, ci2) == (cu, ci)
        assert np.array_equal(U, U1) and np.array_equal(V, V1)


@pytest.mark.parametrize("k", [32, 64, 128])
def test_cg_sweep_direction_is_bitwise_neutral(gpu, k):
    """MR_OPT_CG_SWEEP only changes the order in which the one-pass kernel's
    waves visit the entity chunks; every chunk's partial sums are
    order-independent terms, so all three modes give identical CG counts
    and bitwise-identical factors (k = 128: items one-pass, users
    matvec + update)."""
    from movie_recommender_amd import synth
    from movie_recommender_amd.engine import AlsContext
    # k = 128 at 2 % of the shape: most users rate fewer than 129 movies and
    # the solves stop at once, so that case runs the full C4 shape
    rs = synth.movielens_like("ml-full", k, scale=0.02 if k < 128 else 1.0)
    rng = np.random.RandomState(1)
    U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
    V0 = rng.uniform(-1, 1, rs.num_items * k)
    outs = []
    with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users,
                    rs.num_items) as ctx:
        for sweep in (0, 1, 2):
            ctx.set_option("cg_sweep", sweep)
            ctx.set_factors(U0, V0)
            ctx.reset_stats()
            ctx.iterate(3)
            st = ctx.stats()
            outs.append((ctx.get_factors(), st["cg_users_total"], st["cg_items_total"]))
    (U1, V1), cu, ci = outs[0]
    assert cu + ci > 6, (cu, ci)
    for (U, V), cu2, ci2 in outs[1:]:
        assert (cu2, ci2) == (cu, ci)
        assert np.array_equal(U, U1) and np.array_equal(V, V1)


@pytest.mark.parametrize("k,fuse,chunk,scale", [(64, 1, 2048, 0.02), (64, 0, 2048, 0.02),
                                               (64, 1, 64, 0.02), (32, 1, 2048, 0.02),
                                               (10, 1, 2048, 0.02), (96, 1, 2048, 0.02),
                                               (120, 1, 64, 0.05), (128, 1, 2048, 0.2)])
def test_resident_solve_bitwise_equals_launch_per_iteration(gpu, k, fuse, chunk, scale):
    """MR_OPT_CG_RESIDENT (one launch per solve, every block resident, a
    per-iteration broadcast) against one launch per CG iteration: the same
    arithmetic term for term, so ret, the CG counts, the final rr and the
    factors are bitwise identical -- fused and unfused starts, split
    entities (chunk 64), NB = 1 ... 8 (k = 10 ... 128), every sweep mode, and
    max_iteration limits that stop a solve at its start or mid-way."""
    from movie_recommender_amd import synth
    from movie_recommender_amd.engine import AlsContext
    from movie_recommender_amd import _lib
    rs = synth.movielens_like("ml-full", k, scale=scale)
    rng = np.random.RandomState(3)
    U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
    V0 = rng.uniform(-1, 1, rs.num_items * k)
    try:
        with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items,
                        gram_chunk=chunk) as ctx:
            ctx.set_option("fuse_start", fuse)
            ctx.set_timing(True)
            for sweep in ((1,) if k != 64 or chunk != 2048 else (0, 1, 2)):
                ctx.set_option("cg_sweep", sweep)
                outs = []
                for resident in (0, 1):
                    ctx.set_option("cg_resident", resident)
                    ctx.set_factors(U0, V0)
                    ctx.reset_stats()
                    ctx.iterate(2)
                    trace = [ctx.half_step(side, 0.01, m) for side, m in
                             (("users", 0), ("items", 1), ("users", 3), ("items", 200))]
                    st = ctx.stats()
                    outs.append((ctx.get_factors(), st["cg_users_total"], st["cg_items_total"],
                                 trace, st["kernel_launches"]["resident_users"]))
                (Ua, Va), cua, cia, tra, nra = outs[0]
                (Ub, Vb), cub, cib, trb, nrb = outs[1]
                assert nra == 0 and nrb > 0, (nra, nrb)
                assert (cua, cia) == (cub, cib) and cua + cia > 4, (cua, cia, cub, cib)
                assert tra == trb, (tra, trb)
                assert np.array_equal(Ua, Ub) and np.array_equal(Va, Vb)
    finally:
        _lib.check(_lib.lib().mr_set_gram_chunk(2048), "reset chunk")


@pytest.mark.parametrize("ratings", ["normal", "halfstar"])
@pytest.mark.parametrize("k", [3, 10, 16, 20, 32, 33, 64, 65, 96, 120, 128, 144, 200, 300])
def test_gram_kernel_vs_numpy(gpu, k, ratings):
    """Normal equations of both sides against fp64 NumPy -- VALU fp32 for
    k < 32, bf16x3 split on the bf16 MFMA for 32 <= k <= 128, the streamed
    large-k kernel above -- including heavy entities split across waves
    (chunk 64 forces slabs) and empty entities.  "halfstar" ratings
    (rating - median style, exact in bf16) take the user-side rhs through
    the MFMA W block; "normal" ones keep it on the VALU (row sums on the
    MFMA either way)."""
    from movie_recommender_amd.engine import AlsContext
    from oracle import als_oracle as O
    rng = np.random.default_rng(k)
    nU, nI = 90, 70
    n = 4000
    u = rng.integers(0, nU - 2, n).astype(np.int32)       # last 2 users: no ratings
    i = (rng.zipf(1.3, n) % (nI - 1)).astype(np.int32)    # heavy items, last item empty
    key = np.unique(u.astype(np.int64) * nI + i)
    u = (key // nI).astype(np.int32)
    i = (key % nI).astype(np.int32)
    r = rng.normal(0, 1, len(u)) if ratings == "normal" else rng.integers(1, 11, len(u)) / 2.0 - 3.25
    U0 = rng.uniform(-1, 1, nU * (k + 1))
    V0 = rng.uniform(-1, 1, nI * k)
    with AlsContext(u, i, r, k, nU, nI, gram_chunk=64) as ctx:
        ctx.set_factors(U0, V0)
        for side, (Gf, cf) in (("users", O.gram_user(u, i, r, V0, k, nU)),
                               ("items", O.gram_item(u, i, r, U0, k, nI))):
            ctx.build_normal_equations(side)
            ents = np.arange(Gf.shape[0])
            G, c = ctx.normal_equations(side, ents)
            scale = np.maximum(np.abs(Gf).max(axis=(1, 2)), 1.0)
            assert np.max(np.abs(G - Gf).max(axis=(1, 2)) / scale) < 2e-5
            cs = np.maximum(np.abs(cf).max(axis=1), 1.0)
            assert np.max(np.abs(c - cf).max(axis=1) / cs) < 2e-5
            assert np.all(G[-1] == 0) and np.all(c[-1] == 0)   # empty entity
    from movie_recommender_amd import _lib
    _lib.check(_lib.lib().mr_set_gram_chunk(2048), "reset chunk")


@pytest.mark.parametrize("k", [5, 10, 32, 33, 64, 65, 96, 112, 120, 128, 144, 200, 300])
@pytest.mark.parametrize("fuse,chunk,onepass", [(1, 2048, 1), (1, 64, 1), (0, 2048, 1),
                                                (1, 2048, 0), (0, 2048, 0)])
def test_cg_iterations_vs_oracle(gpu, k, fuse, chunk, onepass):
    """The first CG iterations of both sides -- CG start (fused in the Gram
    epilogue, after slab_reduce for split entities, or the unfused matvec +
    INIT update), the NB = 1..8 block GEMV (NB = 5..8: the streamed tiles of
    tile_matvec_stream, odd NB with an unfolded last diagonal block), the
    update and the fused control
    -- against the oracle's fp64 CG (matrix.cpp:456-529 in block form) run on
    the GPU's own normal equations (fp32 values read back).  What remains is
    summation order (and, one-pass, r'.r' from r.r + 2 alpha r.q + alpha^2
    q.q): final rr within 1e-10, x within 2 fp32 ulps."""
    from movie_recommender_amd.engine import AlsContext
    from movie_recommender_amd import _lib
    from oracle import als_oracle as O
    rng = np.random.default_rng(100 + k)
    nU, nI = 90, 70
    n = 6000
    u = rng.integers(0, nU - 2, n).astype(np.int32)       # last 2 users: no ratings
    i = (rng.zipf(1.3, n) % (nI - 1)).astype(np.int32)    # heavy items, last item empty
    key = np.unique(u.astype(np.int64) * nI + i)
    u = (key // nI).astype(np.int32)
    i = (key % nI).astype(np.int32)
    r = rng.normal(0, 1, len(u))
    U0 = rng.uniform(-1, 1, nU * (k + 1)).astype(np.float32).astype(np.float64)
    V0 = rng.uniform(-1, 1, nI * k).astype(np.float32).astype(np.float64)
    try:
        with AlsContext(u, i, r, k, nU, nI, gram_chunk=chunk) as ctx:
            ctx.set_option("fuse_start", fuse)
            ctx.set_option("cg_onepass", onepass)
            for side, nE in (("users", nU), ("items", nI)):
                ctx.set_factors(U0, V0)
                ctx.build_normal_equations(side)
                G, c = ctx.normal_equations(side, np.arange(nE))
                x0 = (U0 if side == "users" else V0).astype(np.float32)
                r0 = np.einsum("eij,ej->ei", G, x0.astype(np.float64).reshape(nE, -1)).ravel() \
                    - c.ravel()
                for m in (0, 1, 2, 4):
                    ctx.set_factors(U0, V0)
                    its, rr = ctx.half_step(side, 0.01, m)
                    U, V = ctx.get_factors()
                    if m == 0:   # r0 = G x - c, p0 = -r0 (matrix.cpp:468-476)
                        rv, pv, _ = ctx.cg_vectors(side)
                        sc = np.max(np.abs(r0))
                        assert np.max(np.abs(rv - r0)) <= 1e-13 * sc, np.max(np.abs(rv - r0)) / sc
                        assert np.array_equal(pv, -rv)
                    x = x0.copy()
                    ito, rro = O.cg_blocks(G, c, x, 0.01, m)
                    got = U if side == "users" else V
                    assert its == ito, (side, m, its, ito)
                    assert abs(rr - rro) <= 1e-10 * abs(rro), (side, m, rr, rro)
                    step = np.max(np.abs(x.astype(np.float64) - x0))
                    assert np.max(np.abs(got - x)) <= 1e-9 * step + 2 * np.spacing(np.float32(1)), \
                        (side, m, np.max(np.abs(got - x)), step)
    finally:
        _lib.check(_lib.lib().mr_set_gram_chunk(2048), "reset chunk")


def test_gram_rhs_path_selection(gpu):
    """The user-side rhs goes through the MFMA W block only when every rating
    is exact in bf16, the option is on and k > 64: with half-star ratings
    the two settings give different roundings of c at k = 96 (both within
    2e-5 of fp64) and identical ones at k = 64; with arbitrary ratings the
    option changes nothing (bitwise)."""
    from movie_recommender_amd.engine import AlsContext
    from oracle import als_oracle as O
    for k in (96, 64):
        _rhs_path_case(AlsContext, O, k)


def _rhs_path_case(AlsContext, O, k):
    nU, nI = 60, 80
    rng = np.random.default_rng(11)
    key = np.unique(rng.integers(0, nU, 3000) * nI + rng.integers(0, nI, 3000))
    u = (key // nI).astype(np.int32)
    i = (key % nI).astype(np.int32)
    V0 = rng.uniform(-1, 1, nI * k)
    U0 = rng.uniform(-1, 1, nU * (k + 1))
    for kind, r in (("halfstar", rng.integers(1, 11, len(u)) / 2.0 - 3.0),
                    ("normal", rng.normal(0, 1, len(u)))):
        Gf, cf = O.gram_user(u, i, r, V0, k, nU)
        cs = {}
        for on in (1, 0):
            with AlsContext(u, i, r, k, nU, nI) as ctx:
                ctx.set_option("gram_rhs_mfma", on)
                ctx.set_factors(U0, V0)
                ctx.build_normal_equations("users")
                G, c = ctx.normal_equations("users", np.arange(nU))
            scale = np.maximum(np.abs(cf).max(axis=1), 1.0)
            assert np.max(np.abs(c - cf).max(axis=1) / scale) < 2e-5, (kind, on)
            cs[on] = c
        if kind == "halfstar" and k > 64:
            assert not np.array_equal(cs[1], cs[0])
        else:
            assert np.array_equal(cs[1], cs[0])


def test_split_vs_unsplit_same_result(gpu):
    from movie_recommender_amd.engine import AlsContext
    d = load_golden("als_dense_200x150_k32.npz")
    res = []
    for chunk in (64, 4096):
        with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], 32, 200, 150,
                        gram_chunk=chunk) as ctx:
            ctx.set_factors(d["U0"], d["V0"])
            ret = ctx.run()
            res.append((ctx.get_factors(), ret))
    from movie_recommender_amd import _lib
    _lib.check(_lib.lib().mr_set_gram_chunk(2048), "reset chunk")
    (Ua, Va), ra = res[0]
    (Ub, Vb), rb = res[1]
    assert ra == rb
    assert rel_err(Ua, Ub) < 1e-5 and rel_err(Va, Vb) < 1e-5


def test_empty_entities_keep_their_factors(gpu):
    """A user / item without ratings has G = 0, c = 0: CG leaves it unchanged,
    as in the reference (zero rows of A^T A)."""
    from movie_recommender_amd.engine import AlsContext
    from oracle import als_oracle as O
    d = load_golden("als_dense_38x45_k5.npz")
    k = 5
    u, i, r = d["user_ids"], d["item_ids"], d["ratings"]
    nU, nI = 40, 47            # users 38, 39 and items 45, 46 have no ratings
    rng = np.random.RandomState(4)
    U0 = rng.uniform(-1, 1, nU * (k + 1))
    V0 = rng.uniform(-1, 1, nI * k)
    with AlsContext(u, i, r, k, nU, nI) as ctx:
        ctx.set_factors(U0, V0)
        ret = ctx.run()
        U, V = ctx.get_factors()
    Uo, Vo, reto, _ = O.als_block(u, i, r, k, U0, V0)
    assert ret == reto
    assert rel_err(U, Uo) < 1e-5 and rel_err(V, Vo) < 1e-5
    assert np.allclose(U[38 * (k + 1):], U0[38 * (k + 1):], atol=1e-7)
    assert np.allclose(V[45 * k:], V0[45 * k:], atol=1e-7)


@pytest.mark.parametrize("k", [10, 64])
def test_cholesky_mode_vs_oracle(gpu, k):
    from movie_recommender_amd.engine import AlsContext
    from movie_recommender_amd import synth
    from oracle import als_oracle as O
    u, i, r, *_ = synth.dense_fixture(150, 120, k, 0.9, seed=k)
    rng = np.random.RandomState(2)
    U0 = rng.uniform(-1, 1, 150 * (k + 1))
    V0 = rng.uniform(-1, 1, 120 * k)
    ridge = 0.1
    with AlsContext(u, i, r, k, 150, 120, solver="cholesky", ridge=ridge) as ctx:
        ctx.set_factors(U0, V0)
        ctx.iterate(2)
        U, V = ctx.get_factors()
        st = ctx.stats()
    assert st["nonpd_users"] == 0 and st["nonpd_items"] == 0
    Uo, Vo = O.als_exact(u, i, r, k, U0, V0, 2, ridge=ridge)
    assert rel_err(U, Uo) < 1e-4 and rel_err(V, Vo) < 1e-4


@pytest.mark.parametrize("name", ["als_c2_ml100k_k32_it2.npz", "als_c2_ml100k_k32_it200.npz"])
def test_c2_ml100k_k32_through_abi(gpu, name):
    """C2 itself (BASELINE.json configs[1]: the ML-100K generator shrunk at
    k = 32, 23,350 ratings, 331 users x 296 movies) through the drop-in
    als_from_python.  Not pinnable at 1e-5: the compiled reference moves its
    own factors by 57 % (2 iterations) to 85 % (natural stop) between thread
    counts 1..8 (tc_spread; 18 % / 60 % after ONE iteration) -- every user
    block is ill-conditioned and the CG's stagnation stop amplifies summation
    order.  Pinned instead: `ret` is one the reference returns at some thread
    count, and the train RMSE lies in the reference's range over its 6 thread
    counts widened by that range (make_golden.py g11).  The CG arithmetic
    itself is pinned on this data by test_c2_cg_trace_vs_oracle."""
    from movie_recommender_amd import _lib
    d = load_golden(name)
    from oracle import als_oracle as O
    k = int(d["k"])
    assert (len(d["ratings"]), int(d["num_users"]), int(d["num_items"])) == (23350, 331, 296)
    U, V, ret = abi_als(_lib.lib(), d, max_iteration_of(name, d))
    rets = set(json.loads(str(d["rets_by_tc"])).values())
    tr = list(json.loads(str(d["train_rmse_by_tc"])).values())
    assert ret in rets, (ret, rets)
    got = O.rmse(U, V, d["user_ids"], d["item_ids"], d["ratings"], k)
    lo, hi = min(tr), max(tr)
    assert lo - (hi - lo) <= got <= hi + (hi - lo), (got, lo, hi)
    print(f"C2 {name}: GPU ret {ret} train RMSE {got:.5f}; reference rets {sorted(rets)} "
          f"train RMSE {lo:.5f} .. {hi:.5f}")


@pytest.mark.parametrize("side", ["users", "items"])
def test_c2_cg_trace_vs_oracle(gpu, side):
    """C2's first CG solves (users from U0 / V0, then items from the GPU's
    solved U) against the oracle's fp64 CG (matrix.cpp:456-529 in block form)
    on the GPU's own normal equations: the CG count and rr after m = 1, 2, 4,
    8 iterations and at the natural stop, while the two trajectories can
    agree (the reference's thread counts themselves part after ~10-20
    iterations on this data): iterations equal, rr within 1e-10 for m <= 8."""
    from movie_recommender_amd.engine import AlsContext
    from oracle import als_oracle as O
    d = load_golden("als_c2_ml100k_k32_it2.npz")
    k, nU, nI = int(d["k"]), int(d["num_users"]), int(d["num_items"])
    with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], k, nU, nI) as ctx:
        ctx.set_factors(d["U0"], d["V0"])
        if side == "items":
            ctx.half_step("users")
        U1, V1 = ctx.get_factors()
        nE = nU if side == "users" else nI
        ctx.build_normal_equations(side)
        G, c = ctx.normal_equations(side, np.arange(nE))
        x0 = (U1 if side == "users" else V1).astype(np.float32)
        for m in (1, 2, 4, 8):
            ctx.set_factors(U1, V1)
            its, rr = ctx.half_step(side, 0.01, m)
            x = x0.copy()     # fp32, as the factor table: x += alpha p rounded
            ito, rro = O.cg_blocks(G, c, x, 0.01, m)
            assert its == ito, (side, m, its, ito)
            assert abs(rr - rro) <= 1e-10 * abs(rro), (side, m, rr, rro)


def _gpu_rank_agreement(rs, U, V, k):
    """The reference's quality metric on GPU-trained factors through the GPU
    evaluation path (serving.MovieTable.evaluate = _als_eval +
    compute_ranking_agreement, bit-exact against the reference's functions in
    test_gpu_serving.py): every held-out user's raw ratings (residual +
    median) against u[:k].v + u[k] + median.  Mean over users with an
    agreement."""
    from movie_recommender_amd.serving import MovieTable
    ids = {i: i for i in range(rs.num_items)}
    med = {i: float(rs.medians[i]) for i in range(rs.num_items)}
    order = np.argsort(rs.test_user_ids, kind="stable")
    tu = rs.test_user_ids[order]
    ti = rs.test_item_ids[order]
    raw = rs.test_ratings[order] + rs.medians[ti]
    cuts = np.flatnonzero(np.diff(tu)) + 1
    users = np.split(tu, cuts)
    lists = [list(zip(a.tolist(), b.tolist())) for a, b in zip(np.split(ti, cuts),
                                                              np.split(raw, cuts))]
    table = MovieTable(k, V, ids, med)
    try:
        res = table.evaluate(U, [int(u[0]) for u in users], lists)
    finally:
        table.close()
    a = res["agreement"]
    return float(np.nanmean(a)), int(np.count_nonzero(~np.isnan(a)))


def test_distribution_headline_config(gpu):
    """Realistic-data parity at the headline config (VERDICT r05 "do this"
    2; BASELINE.json metric "... RMSE parity"): the MovieLens-full-shaped
    synthetic set at k = 64 with 20 % of each user's ratings held out.  The
    compiled reference ran 20 initial-factor seeds x thread counts {1, 2, 4}
    with its OWN outer stop (max_iteration 200, matrix.cpp:871-875;
    dist_mlfull_k64.json from tests/golden/make_golden.py g13); the GPU runs
    the same 20 seeds once each through the product path.  The reference is
    chaotic here (one seed's held-out RMSE moves by up to ~0.05 between its
    own thread counts), so parity is a two-sample statement on held-out
    RMSE, train RMSE, ``ret`` and the reference's own quality metric (mean
    per-user rank agreement, my_util.py:101-145, computed by the GPU
    evaluation path): dist_stats.failing -- the two-sided Mann-Whitney of the
    20 GPU runs against the 60 reference runs at p >= 0.05 per metric, and
    the seed-stratified permutation test with Holm's correction (family-wise
    0.05).  Sanity bound beside it: each seed's GPU RMSE inside that seed's
    reference range widened by W, the largest range at any seed."""
    import warnings
    import dist_stats as DS
    from movie_recommender_amd import synth
    from movie_recommender_amd.engine import AlsContext
    from oracle import als_oracle as O
    from oracle.ref import init_factors
    path = os.path.join(GOLDEN, "dist_mlfull_k64.json")
    if not os.path.exists(path):
        pytest.skip("dist_mlfull_k64.json not generated (make_golden.py g13)")
    with open(path) as f:
        dist = json.load(f)
    k = dist["k"]
    rs = synth.movielens_like(dist["shape"], k, seed=dist["data_seed"],
                              test_ratio=dist["test_ratio"])
    assert rs.n == dist["n_train"] and len(rs.test_ratings) == dist["n_test"]
    assert abs(float(np.sum(rs.ratings)) - dist["ratings_checksum"]) < 1e-6
    pool = DS.runs_of(dist, "ref")
    assert len(pool) >= 20 * 3 and dist["max_iteration"] == 200
    got = []
    for seed in range(dist["n_seeds"]):
        U0, V0 = init_factors(rs.num_users, rs.num_items, k, seed)
        with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users,
                        rs.num_items) as ctx:
            ctx.set_factors(U0, V0)
            ret = ctx.run(0.01, dist["max_iteration"])
            U, V = ctx.get_factors()
        got.append(dict(seed=seed, ret=ret,
                        test_rmse=O.rmse(U, V, rs.test_user_ids, rs.test_item_ids,
                                         rs.test_ratings, k),
                        train_rmse=O.rmse(U, V, rs.user_ids, rs.item_ids, rs.ratings, k),
                        rank_agreement=_gpu_rank_agreement(rs, U, V, k)[0]))
        print("headline seed", got[-1], flush=True)
    res = DS.compare(got, pool)
    msg = (f"headline config (ML-full shape, k=64, own stop), {len(got)} GPU seeds vs "
           f"{len(pool)} reference runs: " + DS.describe(res))
    print(msg, flush=True)
    warnings.warn(msg)
    assert not DS.failing(res), msg
    for m in ("test_rmse", "train_rmse"):
        rng, W = DS.seed_ranges(pool, m)
        for g in got:
            lo, hi = rng[g["seed"]]
            assert lo - W <= g[m] <= hi + W, (m, g, lo, hi, W)


def test_predict_matches_reference_formula(gpu):
    from movie_recommender_amd.engine import AlsContext
    from oracle import als_oracle as O
    d = load_golden("als_dense_40x45_k3.npz")
    with AlsContext(d["user_ids"], d["item_ids"], d["ratings"], 3, 40, 45) as ctx:
        ctx.set_factors(d["U"], d["V"])
        p = ctx.predict(d["test_user_ids"], d["test_item_ids"])
    ref = O.predict(d["U"], d["V"], d["test_user_ids"], d["test_item_ids"], 3)
    assert np.max(np.abs(p - ref)) < 1e-5


def test_bad_ids_fail_cleanly(gpu):
    from movie_recommender_amd import cpp_ls
    u = np.array([0, 1, 5], np.int32)
    i = np.array([0, 0, 0], np.int32)
    with pytest.raises(RuntimeError):
        cpp_ls.als(u, i, np.ones(3), 2, 2, 1)


@pytest.mark.slow
def test_full_size_gram_sampled(gpu):
    """BASELINE.json configs[2] size (ML-full shape, k = 64): the Gram kernel
    on sampled entities (heaviest, lightest, random) against fp64 NumPy, and
    one CG half-step that must reduce r.r."""
    from movie_recommender_amd import synth
    from movie_recommender_amd.engine import AlsContext
    rs = synth.movielens_like("ml-full", 64)
    k = 64
    rng = np.random.default_rng(0)
    U0 = rng.uniform(-1, 1, rs.num_users * (k + 1))
    V0 = rng.uniform(-1, 1, rs.num_items * k)
    with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users,
                    rs.num_items) as ctx:
        ctx.set_factors(U0, V0)
        for side in ("users", "items"):
            ids = rs.user_ids if side == "users" else rs.item_ids
            other = rs.item_ids if side == "users" else rs.user_ids
            cnt = np.bincount(ids)
            ents = np.unique(np.concatenate([np.argsort(cnt)[-3:], np.argsort(cnt)[:3],
                                             rng.integers(0, len(cnt), 6)])).astype(np.int32)
            ctx.build_normal_equations(side)
            G, c = ctx.normal_equations(side, ents)
            Vm = V0.reshape(-1, k)
            Um = U0.reshape(-1, k + 1)
            for t, e in enumerate(ents):
                sel = ids == e
                if side == "users":
                    a = np.hstack([Vm[other[sel]], np.ones((sel.sum(), 1))])
                    w = rs.ratings[sel]
                else:
                    a = Um[other[sel], :k]
                    w = rs.ratings[sel] - Um[other[sel], k]
                Gr = a.T @ a
                cr = a.T @ w
                assert np.max(np.abs(G[t] - Gr)) / np.max(np.abs(Gr)) < 2e-5
                assert np.max(np.abs(c[t] - cr)) / max(np.max(np.abs(cr)), 1.0) < 2e-5
        its, rr = ctx.half_step("users")
        assert its >= 1 and np.isfinite(rr)


def expected_layout(ids, other, ratings, E, chunk=2048, xcd_table_bytes=0, k=64, n_other=None):
    """Host restatement of the context build (engine.hip build_side /
    build_work_xcd): stable CSR by entity, then the Gram work list.  Plain:
    entities longer than `chunk` split into slabs numbered in entity order,
    stable sort by length, heavy first.  When the opposite table exceeds
    16 MiB (32 <= k <= 128) and a heavy entity exists: every heavy entity cut
    at the opposite-id boundaries x * n_other / 8 (fixed chunks labelled by
    their middle id if its list is unsorted), each range into chunks of <=
    `chunk`, range x's chunks dealt to positions p with (p // 4) % 8 == x
    (queues longest first; a dry queue yields to the fullest), followed by
    the unsplit entities heavy first."""
    order = np.argsort(ids, kind="stable")
    off = np.zeros(E + 1, np.int64)
    np.cumsum(np.bincount(ids, minlength=E), out=off[1:])
    cidx = other[order].astype(np.int32)
    lens = np.diff(off)
    xcd = (xcd_table_bytes > (16 << 20) and 32 <= k <= 128 and bool(np.any(lens > chunk)))
    work = []
    nslab = 0
    if not xcd:
        for e in range(E):
            ln = int(lens[e])
            if ln <= chunk:
                work.append((int(off[e]), ln, e, -1))
            else:
                nc = (ln + chunk - 1) // chunk
                for c in range(nc):
                    b = int(off[e]) + c * chunk
                    work.append((b, min(chunk, int(off[e + 1]) - b), e, nslab + c))
                nslab += nc
        work.sort(key=lambda w: -w[1])     # stable: equal lengths keep entity order
        return off, cidx, ratings[order].astype(np.float32), work
    queues = [[] for _ in range(8)]
    light = []
    for e in range(E):
        b0, b1 = int(off[e]), int(off[e + 1])
        if b1 - b0 <= chunk:
            light.append((b0, b1 - b0, e, -1))
            continue
        seg = cidx[b0:b1]
        if np.all(seg[1:] >= seg[:-1]):
            a = b0
            for x in range(8):
                z = b1 if x == 7 else b0 + int(np.searchsorted(seg, (x + 1) * n_other // 8,
                                                               side="left"))
                for c in range(a, z, chunk):
                    queues[x].append((c, min(chunk, z - c), e, nslab))
                    nslab += 1
                a = z
        else:
            for c in range(b0, b1, chunk):
                ln = min(chunk, b1 - c)
                x = min(7, int(cidx[c + ln // 2]) * 8 // n_other)
                queues[x].append((c, ln, e, nslab))
                nslab += 1
    for qx in queues:
        qx.sort(key=lambda w: -w[1])
    head = [0] * 8
    for p in range(sum(len(qx) for qx in queues)):
        x = (p // 4) % 8
        if head[x] == len(queues[x]):
            best = 0
            for y in range(8):
                if len(queues[y]) - head[y] > best:
                    best, x = len(queues[y]) - head[y], y
        work.append(queues[x][head[x]])
        head[x] += 1
    light.sort(key=lambda w: -w[1])
    return off, cidx, ratings[order].astype(np.float32), work + light


def test_full_size_context_build_exact(gpu):
    """BASELINE.json configs[2] size: the device CSR of both sides and the
    Gram work lists read back and compared with their host restatement, bit
    for bit (uploads go through pinned staging, Stager in xfer.hip)."""
    from movie_recommender_amd import synth
    from movie_recommender_amd.engine import AlsContext
    k = 64
    rs = synth.movielens_like("ml-full", k)
    with AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users,
                    rs.num_items) as ctx:
        for side in ("users", "items"):
            ids, other, E = ((rs.user_ids, rs.item_ids, rs.num_users) if side == "users"
                             else (rs.item_ids, rs.user_ids, rs.num_items))
            off, idx, val, (wb, wl, we, ws) = ctx.layout(side)
            n_other = rs.num_items if side == "users" else rs.num_users
            eoff, eidx, eval_, work = expected_layout(ids, other, rs.ratings, E,
                                                      xcd_table_bytes=n_other * 64 * 4, k=k,
                                                      n_other=n_other)
            assert np.array_equal(off, eoff), side
            assert np.array_equal(idx, eidx), side
            assert np.array_equal(val, eval_), side
            w = np.array(work, np.int64)
            assert len(wb) == len(w), side
            assert np.array_equal(wb, w[:, 0]) and np.array_equal(wl, w[:, 1]), side
            assert np.array_equal(we, w[:, 2]) and np.array_equal(ws, w[:, 3]), side


def test_cg_counts_from_reference_states(gpu):
    """CG-count parity on the bench workload's own trajectory (VERDICT r03
    missing 5), at 1/4 of the ML-full shape, k = 64: before each of the
    compiled reference's CG solves (oracle/ref_replay, bit-identical to
    als_from_python) the engine is put in the same state and runs the same
    half-step (defaults 0.01, 200).  Two ALS runs of this data part
    chaotically after a few iterations, so the comparison is per half-step
    from the SAME state.  Short solves -- the reference stops within 12 CG
    iterations, by its stagnation rule -- must take exactly the reference's
    count.  Long solves (20-60 iterations on ill-conditioned user blocks) are
    chaotic in the formulation itself: the oracle's all-fp64 block-Gram
    restatement of the same solve (G = sum a a^T, the form SURVEY.md 8(c)
    prescribes) already differs from the reference's design-matrix CG there
    (42 vs 43, 41 vs 23, 24 vs 21, 25 vs 43 iterations from the reference's
    states; profiles/r04/cg_precision_probe_x0.25.jsonl), so they are held
    to the side's total within 25 %.  tools/cg_count_parity.py runs the same
    check at full size (profiles/r04: items 25 / 25, users 23 / 25 equal)."""
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from cg_count_parity import run
    recs, summ = run(scale=0.25, iterations=8)
    print(json.dumps(summ))
    for side in ("users", "items"):
        rr = [r for r in recs if r["side"] == side]
        short = [r for r in rr if r["reference"][0] <= 12]
        bad = [(r["iteration"], r["engine"][0], r["reference"][0]) for r in short
               if r["engine"][0] != r["reference"][0]]
        assert not bad, (side, bad)
        s = summ[side]
        assert abs(s["engine_total"] - s["reference_total"]) <= 0.25 * s["reference_total"], s
