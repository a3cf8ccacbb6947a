"""The reference's ``als()`` replayed around its own CG -- TEST INFRA ONLY.

``als()`` (``cpp/ls_lib/matrix.cpp:744-893``) returns only its outer
iteration index; the CG iteration counts of its half-steps, which decide its
cost, stay inside.  This module restates the outer loop in Python and calls
the compiled reference's ``cg_least_squares_from_python``
(``ls_linux_dll.cpp:28-50`` -> ``cg_least_squares``, ``matrix.cpp:456-529``)
on design matrices built exactly as ``fill_user_A`` / ``fill_item_A`` /
``fill_ratings_minus_bias`` build them (``matrix.cpp:898-1031``: row r of
user_A = [V[item_r, 0..k-1], 1] at columns user_r (k+1) + j; row r of item_A
= U[user_r, 0..k-1] at columns item_r k + j; b = r - U[user_r][k]).  Both
entry points wrap the matrix with ``SparseMatrix::load`` (the same thread
spread, ``matrix.cpp:163-184``), so the replay runs the identical arithmetic:
its factors and ``ret`` equal ``als_from_python``'s bit for bit
(``tests/test_oracle.py::test_ref_replay_bitwise_equals_reference_als``), and
it reports each half-step's CG iteration count and wall time.

Used by ``bench.py``'s ``cpu_baseline`` leg to report the reference's CG
iterations per ALS iteration and its time per CG iteration on the timed
sample.
"""
import time

import numpy as np

from . import ref


def _alt(threads, rp, ci, va, ncols, b, x0):
    keep = ref.lib().get_thread_count()
    ref.set_thread_count(threads)
    try:
        _, its, rr = ref.cg_least_squares(rp, ci, va.reshape(-1), ncols, b, x0)
    finally:
        ref.set_thread_count(keep)
    return its, rr


def als_replay(user_ids, item_ids, ratings, k, U0, V0, min_r_decrease=0.01,
               max_iteration=200, on_iteration=None, on_half_step=None):
    """Returns ``(U, V, ret, trace)``; ``trace`` has one dict per ALS
    iteration: ``cg_users``, ``cg_items`` (iterations), ``t_users``,
    ``t_items`` (seconds inside the reference CG), ``rr``.
    ``on_iteration(it, record)`` is called after each iteration (progress);
    ``on_half_step(side, it, U, V, alt)`` before each CG solve with the state
    it starts from (fp64 tables, not to be modified) -- a caller can run
    another solver from the reference's own state; ``alt(threads)`` runs the
    reference's same solve at another thread count and returns
    ``(iterations, final_rr)`` (the reference's own summation-order spread)."""
    uid = np.ascontiguousarray(user_ids, np.int32)
    iid = np.ascontiguousarray(item_ids, np.int32)
    r = np.ascontiguousarray(ratings, np.float64)
    K = k + 1
    n = len(r)
    U = np.array(U0, np.float64).reshape(-1).copy()
    V = np.array(V0, np.float64).reshape(-1).copy()
    if n * K >= 2 ** 31:
        raise OverflowError("N (k+1) >= 2^31: the reference's int32 indices overflow here too")
    # user_A (fill_user_A, first fill): row_ptr r K, columns u K + j
    rp_u = (np.arange(n + 1, dtype=np.int64) * K).astype(np.int32)
    ci_u = (uid.astype(np.int64)[:, None] * K + np.arange(K)).astype(np.int32).reshape(-1)
    va_u = np.empty((n, K))
    va_u[:, k] = 1.0
    # item_A (fill_item_A): row_ptr r k, columns i k + j
    rp_i = (np.arange(n + 1, dtype=np.int64) * k).astype(np.int32)
    ci_i = (iid.astype(np.int64)[:, None] * k + np.arange(k)).astype(np.int32).reshape(-1)
    va_i = np.empty((n, k))
    Vm = V.reshape(-1, k)
    Um = U.reshape(-1, K)
    va_u[:, :k] = Vm[iid]
    va_i[:, :] = Um[uid, :k]
    trace = []
    it, old_rr = 0, 0.0
    while it < max_iteration:
        if on_half_step is not None:
            on_half_step("users", it, U, V, lambda tc: _alt(
                tc, rp_u, ci_u, va_u, len(U), r, U))
        t0 = time.perf_counter()
        x, cu, _ = ref.cg_least_squares(rp_u, ci_u, va_u.reshape(-1), len(U), r, U)
        t_u = time.perf_counter() - t0
        U[:] = x
        va_i[:, :] = Um[uid, :k]                       # fill_item_A (refresh)
        b = r - Um[uid, k]                             # fill_ratings_minus_bias
        if on_half_step is not None:
            on_half_step("items", it, U, V, lambda tc: _alt(
                tc, rp_i, ci_i, va_i, len(V), b, V))
        t0 = time.perf_counter()
        x, ci, rr = ref.cg_least_squares(rp_i, ci_i, va_i.reshape(-1), len(V), b, V)
        t_i = time.perf_counter() - t0
        V[:] = x
        trace.append(dict(cg_users=cu, cg_items=ci, t_users=t_u, t_items=t_i, rr=rr))
        if on_iteration is not None:
            on_iteration(it, trace[-1])
        if it >= 3 and (old_rr - rr) / old_rr < min_r_decrease:
            return U, V, it, trace
        va_u[:, :k] = Vm[iid]                          # fill_user_A (refresh)
        old_rr = rr
        it += 1
    return U, V, it, trace
