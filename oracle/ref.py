"""ctypes driver for the reference library built from source -- TEST INFRA ONLY.

``oracle/Makefile`` compiles ``/root/reference/cpp/ls_lib/{ls_linux_dll,matrix}.cpp``
into ``oracle/_ref/cpp_ls_lib.so``.  This module binds its five ``extern "C"``
symbols (``cpp/ls_lib/ls_linux_dll.cpp:8-103``) and reproduces the caller-side
conventions of the reference wrapper ``cpp/python/cpp_ls.py:111-169``
(U0 drawn before V0, both ``uniform(-1, 1)``), without importing that wrapper.

Used to (a) generate the golden fixtures in ``tests/golden/`` and (b) time the
reference CPU path in ``bench.py`` (``cpu_baseline.kind == "reference"``).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(_HERE, "_ref", "cpp_ls_lib.so")

_lib = None


def available() -> bool:
    return os.path.exists(REF_SO)


def lib():
    """Load ``oracle/_ref/cpp_ls_lib.so`` with explicit prototypes."""
    global _lib
    if _lib is not None:
        return _lib
    if not available():
        raise FileNotFoundError(
            f"{REF_SO} missing: run `make -C oracle ref` (needs /root/reference)")
    L = ctypes.CDLL(REF_SO)
    ip = ctypes.POINTER(ctypes.c_int)
    dp = ctypes.POINTER(ctypes.c_double)
    L.set_thread_count.argtypes = [ctypes.c_int]
    L.set_thread_count.restype = None
    L.get_thread_count.argtypes = []
    L.get_thread_count.restype = ctypes.c_int
    cg_args = [ctypes.c_int, ctypes.c_int, ip, ip, dp, ctypes.c_int, dp,
               ctypes.c_int, dp, ctypes.c_double, ctypes.c_int, dp]
    L.cg_least_squares_from_python.argtypes = cg_args
    L.cg_least_squares_from_python.restype = ctypes.c_int
    L.cg_least_squares2_from_python.argtypes = cg_args
    L.cg_least_squares2_from_python.restype = ctypes.c_int
    L.als_from_python.argtypes = [ip, ip, ctypes.c_int, dp, ctypes.c_int,
                                  ctypes.c_int, dp, ctypes.c_int, dp,
                                  ctypes.c_double, ctypes.c_int, ctypes.c_int]
    L.als_from_python.restype = ctypes.c_int
    _lib = L
    return L


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def set_thread_count(n: int):
    lib().set_thread_count(int(n))


def cg_least_squares(row_ptr, col_idx, vals, ncols, b, x0,
                     min_r_decrease=0.01, max_iteration=200, algorithm=1):
    """Reference CG least squares (``matrix.cpp:456-529`` / ``:536-613``).

    Returns ``(x, iterations, final_rr)``; ``x0`` is not modified.
    """
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
    col_idx = np.ascontiguousarray(col_idx, dtype=np.int32)
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    x = np.array(x0, dtype=np.float64).reshape(-1).copy()
    rr = ctypes.c_double(0.0)
    fn = lib().cg_least_squares_from_python if algorithm == 1 \
        else lib().cg_least_squares2_from_python
    it = fn(len(row_ptr) - 1, int(ncols), _ip(row_ptr), _ip(col_idx), _dp(vals),
            len(b), _dp(b), len(x), _dp(x), float(min_r_decrease),
            int(max_iteration), ctypes.byref(rr))
    return x, int(it), float(rr.value)


def als(user_ids, item_ids, ratings, k, U0, V0,
        min_r_decrease=0.01, max_iteration=200, algorithm=1):
    """Reference ALS (``matrix.cpp:744-893``) on caller-supplied initial factors.

    ``U0`` has ``num_users*(k+1)`` entries, ``V0`` has ``num_items*k``
    (the layout of ``cpp_ls.py:147-148``).  Returns ``(U, V, ret)``.
    """
    uid = np.ascontiguousarray(user_ids, dtype=np.int32)
    iid = np.ascontiguousarray(item_ids, dtype=np.int32)
    r = np.ascontiguousarray(ratings, dtype=np.float64)
    U = np.array(U0, dtype=np.float64).reshape(-1).copy()
    V = np.array(V0, dtype=np.float64).reshape(-1).copy()
    ret = lib().als_from_python(_ip(uid), _ip(iid), len(r), _dp(r), int(k),
                                len(U), _dp(U), len(V), _dp(V),
                                float(min_r_decrease), int(max_iteration),
                                int(algorithm))
    return U, V, int(ret)


def init_factors(num_users, num_items, k, seed):
    """Initial factors in the reference order: ``numpy.random.seed(seed)``,
    then U0 = uniform(-1,1,U*(k+1)), V0 = uniform(-1,1,I*k)
    (``cpp/python/cpp_ls.py:147-148``)."""
    rs = np.random.RandomState(seed)
    U0 = rs.uniform(-1, 1, num_users * (k + 1))
    V0 = rs.uniform(-1, 1, num_items * k)
    return U0, V0
