"""NumPy/SciPy restatement of the reference ALS hot path -- TEST INFRA ONLY.

Follows ``/root/reference/cpp/ls_lib/matrix.cpp`` (cited per function).
Two equivalent forms are provided:

* **design-matrix form** (``als_design``): builds ``user_A`` (N x U(k+1)) and
  ``item_A`` (N x Ik) exactly as ``fill_user_A``/``fill_item_A`` do and runs
  CG on ``A^T A x = A^T b`` with SpMV/SpMV^T -- the reference algorithm.
* **block-Gram form** (``als_block``): ``A^T A`` is block diagonal, one
  ``(k+1)^2`` block per user and ``k^2`` per item, so the CG matvec is a
  batched per-entity GEMV ``G_e p_e``.  Same CG scalars, same stop rules.
  This is the form the HIP path implements; ``dtype=np.float32`` emulates
  its precision: fp32 normal equations (G, c) and factor tables (x), fp64
  CG vectors r / p / q with every product G p accumulated in fp64, fp64 dot
  products and scalars.  (fp32 r / p / q drift by percents from the
  reference on ill-conditioned blocks -- the 60 x 50, k = 32 fixture -- and
  are not used.)

Plus the exact per-entity solve (``als_exact``; Cholesky mode) and the
reference's ``als_predict``.
"""
import numpy as np
import scipy.sparse as sp


def _div(a, b):
    """IEEE-754 division as in the reference's C++ (0/0 -> nan, x/0 -> +-inf)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(a) / np.float64(b))


# --------------------------------------------------------------------------
# CG on the normal equations  (matrix.cpp:456-529, cg_least_squares)
# --------------------------------------------------------------------------
def cg_normal(matvec, c, x, min_r_decrease=0.01, max_iteration=200,
              dot=None, vdtype=np.float64, trace=None):
    """CG on ``M x = c`` with ``M = A^T A`` given as ``matvec``.

    Restates ``cg_least_squares`` (``matrix.cpp:456-529``) line by line:
    r0 = Mx - c (``:468-472``), p0 = -r0 (``:475-476``), early return when
    rr < 1e-6 at the loop top (``:490``), two consecutive beta > 1-min_r_decrease
    failures end the solve *after* x and r were updated (``:512-518``),
    ``final_rr`` tracks the last rr computed (``:486, :508``).
    ``x`` is updated in place.  Returns ``(iterations, final_rr)``; a list
    passed as ``trace`` receives r0.r0 and every iteration's r'.r'.
    """
    if dot is None:
        def dot(a, b):
            return float(np.dot(a.astype(np.float64), b.astype(np.float64)))
    r = (matvec(x) - c).astype(vdtype)
    p = (-r).astype(vdtype)
    it = 0
    fails = 0
    rr = dot(r, r)
    final_rr = rr
    if trace is not None:
        trace.append(rr)
    while it < max_iteration:
        if rr < 1e-6:
            return it, final_rr
        Ap = matvec(p).astype(vdtype)
        alpha = _div(rr, dot(p, Ap))
        x += vdtype(alpha) * p if vdtype is np.float32 else alpha * p
        r += vdtype(alpha) * Ap if vdtype is np.float32 else alpha * Ap
        rr2 = dot(r, r)
        final_rr = rr2
        if trace is not None:
            trace.append(rr2)
        beta = _div(rr2, rr)
        if beta > 1 - min_r_decrease:
            fails += 1
        else:
            fails = 0
        if fails >= 2:
            return it, final_rr
        p = (-r + (vdtype(beta) if vdtype is np.float32 else beta) * p).astype(vdtype)
        rr = rr2
        it += 1
    return it, final_rr


def cg_least_squares(row_ptr, col_idx, vals, ncols, b, x0,
                     min_r_decrease=0.01, max_iteration=200):
    """Restates ``cg_least_squares`` (``matrix.cpp:456-529``) for a general CSR A.

    Returns ``(x, iterations, final_rr)``.
    """
    nrows = len(row_ptr) - 1
    A = sp.csr_matrix((np.asarray(vals, np.float64), np.asarray(col_idx),
                       np.asarray(row_ptr)), shape=(nrows, ncols))
    At = A.T.tocsr()
    b2 = At @ np.asarray(b, np.float64).reshape(-1)          # :464-465
    x = np.array(x0, np.float64).reshape(-1).copy()
    it, rr = cg_normal(lambda v: At @ (A @ v), b2, x,
                       min_r_decrease, max_iteration)
    return x, it, rr


# --------------------------------------------------------------------------
# Design-matrix form  (matrix.cpp:744-893 + fill_* :898-1031)
# --------------------------------------------------------------------------
def build_user_A(user_ids, item_ids, V, k, num_users):
    """``fill_user_A`` (``matrix.cpp:898-952``): row r = [V[item_r,:], 1] at
    columns ``user_r*(k+1) + j``."""
    N = len(user_ids)
    K = k + 1
    Vm = np.asarray(V, np.float64).reshape(-1, k)
    vals = np.empty((N, K))
    vals[:, :k] = Vm[item_ids]
    vals[:, k] = 1.0
    cols = (np.asarray(user_ids, np.int64)[:, None] * K + np.arange(K)[None, :])
    indptr = np.arange(N + 1, dtype=np.int64) * K
    return sp.csr_matrix((vals.reshape(-1), cols.reshape(-1), indptr),
                         shape=(N, num_users * K))


def build_item_A(user_ids, item_ids, U, k, num_items):
    """``fill_item_A`` (``matrix.cpp:957-1007``): row r = U[user_r, :k] at
    columns ``item_r*k + j``."""
    N = len(user_ids)
    Um = np.asarray(U, np.float64).reshape(-1, k + 1)
    vals = Um[user_ids, :k]
    cols = (np.asarray(item_ids, np.int64)[:, None] * k + np.arange(k)[None, :])
    indptr = np.arange(N + 1, dtype=np.int64) * k
    return sp.csr_matrix((vals.reshape(-1), cols.reshape(-1), indptr),
                         shape=(N, num_items * k))


def ratings_minus_bias(user_ids, ratings, U, k):
    """``fill_ratings_minus_bias`` (``matrix.cpp:1012-1031``)."""
    Um = np.asarray(U, np.float64).reshape(-1, k + 1)
    return np.asarray(ratings, np.float64) - Um[user_ids, k]


def als_design(user_ids, item_ids, ratings, k, U0, V0,
               min_r_decrease=0.01, max_iteration=200):
    """Reference ALS in design-matrix form (``matrix.cpp:744-893``).

    Returns ``(U, V, ret, trace)``; ``trace`` lists per outer iteration the
    user/item CG iteration counts and the item-side final rr.
    """
    U = np.array(U0, np.float64).reshape(-1).copy()
    V = np.array(V0, np.float64).reshape(-1).copy()
    nU = len(U) // (k + 1)
    nI = len(V) // k
    r = np.asarray(ratings, np.float64)
    it = 0
    old_rr = 0.0
    trace = []
    while it < max_iteration:                                  # :814
        A = build_user_A(user_ids, item_ids, V, k, nU)
        At = A.T.tocsr()
        cu, _ = cg_normal(lambda v: At @ (A @ v), At @ r, U)   # :818 (0.01, 200)
        B = build_item_A(user_ids, item_ids, U, k, nI)         # :831-838
        Bt = B.T.tocsr()
        rb = ratings_minus_bias(user_ids, r, U, k)             # :841-848
        ci, rr = cg_normal(lambda v: Bt @ (B @ v), Bt @ rb, V, 0.01, 200)  # :854
        trace.append((cu, ci, rr))
        if it >= 3:                                            # :871-875
            if _div(old_rr - rr, old_rr) < min_r_decrease:
                return U, V, it, trace
        old_rr = rr
        it += 1
    return U, V, it, trace


# --------------------------------------------------------------------------
# Block-Gram form (the HIP path's algorithm)
# --------------------------------------------------------------------------
def _segments(ids, n):
    order = np.argsort(ids, kind="stable")
    counts = np.bincount(ids, minlength=n)
    off = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=off[1:])
    return order, off


def gram_user(user_ids, item_ids, ratings, V, k, num_users, dtype=np.float64):
    """Per-user normal equations: ``G_u = sum a a^T``, ``c_u = sum a r`` with
    ``a = [V_i, 1]`` -- the diagonal blocks of ``user_A^T user_A`` and
    ``user_A^T ratings`` (``matrix.cpp:465, 898-952``)."""
    K = k + 1
    Vm = np.asarray(V, np.float64).reshape(-1, k)
    a = np.empty((len(user_ids), K))
    a[:, :k] = Vm[item_ids]
    a[:, k] = 1.0
    if dtype is np.float32:
        a = a.astype(np.float32).astype(np.float64)
    w = np.asarray(ratings, np.float64)
    if dtype is np.float32:
        w = w.astype(np.float32).astype(np.float64)
    G = np.zeros((num_users, K, K))
    c = np.zeros((num_users, K))
    order, off = _segments(np.asarray(user_ids), num_users)
    for u in range(num_users):
        sel = order[off[u]:off[u + 1]]
        if len(sel) == 0:
            continue
        au = a[sel]
        G[u] = au.T @ au
        c[u] = au.T @ w[sel]
    return G.astype(dtype), c.astype(dtype)


def gram_item(user_ids, item_ids, ratings, U, k, num_items, dtype=np.float64):
    """Per-item normal equations: ``G_i = sum u u^T``, ``c_i = sum u (r - b_u)``
    (``matrix.cpp:957-1031``)."""
    Um = np.asarray(U, np.float64).reshape(-1, k + 1)
    if dtype is np.float32:
        Um = Um.astype(np.float32).astype(np.float64)
    a = Um[user_ids, :k]
    w = np.asarray(ratings, np.float64)
    if dtype is np.float32:
        w = w.astype(np.float32).astype(np.float64)
        w = (w - Um[user_ids, k]).astype(np.float32).astype(np.float64)
    else:
        w = w - Um[user_ids, k]
    G = np.zeros((num_items, k, k))
    c = np.zeros((num_items, k))
    order, off = _segments(np.asarray(item_ids), num_items)
    for i in range(num_items):
        sel = order[off[i]:off[i + 1]]
        if len(sel) == 0:
            continue
        ai = a[sel]
        G[i] = ai.T @ ai
        c[i] = ai.T @ w[sel]
    return G.astype(dtype), c.astype(dtype)


def block_matvec(G):
    """``(G x)_e = G_e x_e`` on the concatenated vector."""
    E, K, _ = G.shape

    Gd = G.astype(np.float64)   # fp32 entries, fp64 products and sums

    def mv(x):
        xe = np.asarray(x, np.float64).reshape(E, K)
        return np.einsum("eij,ej->ei", Gd, xe).reshape(-1)
    return mv


def cg_blocks(G, c, x, min_r_decrease=0.01, max_iteration=200, trace=None):
    """Block-Gram CG: ``cg_normal`` with the batched block GEMV.  Vectors are
    fp64; ``x`` keeps its own dtype (fp32 factor tables: x += alpha p is
    formed in fp64 and rounded)."""
    return cg_normal(block_matvec(G), np.asarray(c, np.float64).reshape(-1), x,
                     min_r_decrease, max_iteration, trace=trace)


def als_block(user_ids, item_ids, ratings, k, U0, V0,
              min_r_decrease=0.01, max_iteration=200, dtype=np.float64):
    """ALS with block-Gram CG half-steps; control flow of ``matrix.cpp:814-893``.

    Returns ``(U, V, ret, trace)`` in float64 layout ``U: nU*(k+1)``,
    ``V: nI*k``.
    """
    U = np.array(U0, np.float64).reshape(-1).astype(dtype)
    V = np.array(V0, np.float64).reshape(-1).astype(dtype)
    nU = len(U) // (k + 1)
    nI = len(V) // k
    it = 0
    old_rr = 0.0
    trace = []
    while it < max_iteration:
        G, c = gram_user(user_ids, item_ids, ratings, V, k, nU, dtype)
        cu, _ = cg_blocks(G, c, U, 0.01, 200)
        G, c = gram_item(user_ids, item_ids, ratings, U, k, nI, dtype)
        ci, rr = cg_blocks(G, c, V, 0.01, 200)
        trace.append((cu, ci, rr))
        if it >= 3:
            if _div(old_rr - rr, old_rr) < min_r_decrease:
                return U.astype(np.float64), V.astype(np.float64), it, trace
        old_rr = rr
        it += 1
    return U.astype(np.float64), V.astype(np.float64), it, trace


# --------------------------------------------------------------------------
# Exact per-entity solve (Cholesky mode)
# --------------------------------------------------------------------------
def solve_blocks(G, c, x, ridge=0.0):
    """x_e = (G_e + ridge I)^{-1} c_e for every entity with a PD block; entities
    whose block is not positive definite keep their previous x_e.
    Returns the number of non-PD blocks."""
    E, K, _ = G.shape
    xe = x.reshape(E, K)
    bad = 0
    for e in range(E):
        M = G[e].astype(np.float64) + ridge * np.eye(K)
        try:
            L = np.linalg.cholesky(M)
        except np.linalg.LinAlgError:
            bad += 1
            continue
        y = np.linalg.solve(L, c[e].astype(np.float64))
        xe[e] = np.linalg.solve(L.T, y)
    return bad


def als_exact(user_ids, item_ids, ratings, k, U0, V0, iterations, ridge=0.0):
    """Fixed number of exact ALS iterations (no CG)."""
    U = np.array(U0, np.float64).reshape(-1).copy()
    V = np.array(V0, np.float64).reshape(-1).copy()
    nU = len(U) // (k + 1)
    nI = len(V) // k
    for _ in range(iterations):
        G, c = gram_user(user_ids, item_ids, ratings, V, k, nU)
        solve_blocks(G, c, U, ridge)
        G, c = gram_item(user_ids, item_ids, ratings, U, k, nI)
        solve_blocks(G, c, V, ridge)
    return U, V


# --------------------------------------------------------------------------
# Prediction  (matrix.cpp:1035-1053; cpp/python/cpp_ls_test.py:151-163)
# --------------------------------------------------------------------------
def predict(U, V, user_ids, item_ids, k):
    Um = np.asarray(U, np.float64).reshape(-1, k + 1)
    Vm = np.asarray(V, np.float64).reshape(-1, k)
    return np.einsum("nj,nj->n", Um[user_ids, :k], Vm[item_ids]) + Um[user_ids, k]


def rmse(U, V, user_ids, item_ids, ratings, k):
    d = predict(U, V, user_ids, item_ids, k) - np.asarray(ratings, np.float64)
    return float(np.sqrt(np.mean(d * d)))


def rank_agreement_mean(U, V, k, user_ids, item_ids, ratings, medians):
    """Mean per-user ranking agreement on held-out ratings, the reference's
    quality metric (``_als_eval``, ``python/full_data/worker_process.py:262-306``
    with ``compute_ranking_agreement``, ``my_util.py:101-145``): each test
    user's movies are scored ``u[:k].v + u[k] + median`` (``als_predictor.py:
    35-60``) and compared with the raw ratings (residual + median); over
    every pair with actual(m1) > actual(m2), agreement when predicted(m1) >
    predicted(m2).  Users with one rating or all-equal ratings have no
    agreement (None in the reference) and are skipped.  Returns (mean over
    users with an agreement, number of such users)."""
    med = np.asarray(medians, np.float64)
    pred = predict(U, V, user_ids, item_ids, k) + med[item_ids]
    act = np.asarray(ratings, np.float64) + med[item_ids]
    order = np.argsort(user_ids, kind="stable")
    u_s, p_s, a_s = np.asarray(user_ids)[order], pred[order], act[order]
    bounds = np.flatnonzero(np.diff(u_s)) + 1
    starts = np.concatenate([[0], bounds])
    ends = np.concatenate([bounds, [len(u_s)]])
    vals = []
    for s, e in zip(starts, ends):
        if e - s < 2:
            continue
        a, p = a_s[s:e], p_s[s:e]
        gt = a[:, None] > a[None, :]
        n = int(np.count_nonzero(gt))
        if n == 0:
            continue
        vals.append(np.count_nonzero(gt & (p[:, None] > p[None, :])) / n)
    return (float(np.mean(vals)) if vals else float("nan")), len(vals)
