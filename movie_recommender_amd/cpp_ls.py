"""Drop-in for the reference ctypes wrapper ``cpp/python/cpp_ls.py``.

Same functions, argument meaning, return values and RNG use as the reference
(``cpp/python/cpp_ls.py:23-169``; ``get_thread_count`` from the
``python/full_data/cpp_ls.py:43-44`` copy), but the library behind it is the
MI355X HIP build ``movie_recommender_amd/lib/cpp_ls_lib.so``.  Differences:

* the library is located next to this package, not in the CWD
  (``cpp_ls.py:11``); set ``MR_CPP_LS_LIB`` to override;
* argument types are declared (the reference passes bare ints/pointers);
* ``cg_least_squares(..., algorithm=2)`` calls the existing symbol
  ``cg_least_squares2_from_python`` (the reference calls the misspelled
  ``cg_least_squares_from_python2`` and raises AttributeError, ``:103``);
* a failing native call raises RuntimeError instead of aborting the process.
"""
import ctypes
import multiprocessing
import random

import numpy

from . import _lib

_dll = None


def _load_dll():
    """``cpp_ls.py:5-14``: load the library and set the thread count to
    ``cpu_count()`` (stored only; GPU work is not sized by it)."""
    global _dll
    _dll = _lib.lib()
    _dll.set_thread_count(multiprocessing.cpu_count())


_load_dll()


def has_dll_loaded():
    """Returns true if the native library has been successfully loaded
    (``cpp_ls.py:23-36``: random set/get thread-count round trip)."""
    old_thread_count = _dll.get_thread_count()
    random_number = random.randint(1, 100000)
    _dll.set_thread_count(random_number)
    success = _dll.get_thread_count() == random_number
    _dll.set_thread_count(old_thread_count)
    return success


def set_thread_count(thread_count):
    _dll.set_thread_count(int(thread_count))


def get_thread_count():
    return _dll.get_thread_count()


def _i32(a):
    a = numpy.ascontiguousarray(a)
    if a.dtype != numpy.int32:
        raise TypeError(f"expected int32 array, got {a.dtype} (int64 ids give garbage in "
                        "the reference; refused here)")
    return a


def _f64(a):
    return numpy.ascontiguousarray(a, dtype=numpy.float64)


def cg_least_squares(A_row_indices, A_col_indices, A_values, A_num_columns, b,
                     min_r_decrease=0.01, max_iterations=200, algorithm=1):
    """Solves Ax = b in the least squares sense (``cpp_ls.py:44-108``).

    x is initialised ``numpy.random.uniform(-1, 1, (A_num_columns, 1))`` from
    NumPy's global RNG, as the reference does.  Returns
    ``(x, iterations, final_rr)``.
    """
    rp = _i32(A_row_indices)
    ci = _i32(A_col_indices)
    vals = _f64(A_values)
    b = _f64(b).reshape(-1)
    A_rows = len(rp) - 1
    x = numpy.random.uniform(-1, 1, (A_num_columns, 1))
    final_rr = ctypes.c_double(0)
    fn = _dll.cg_least_squares_from_python if algorithm == 1 \
        else _dll.cg_least_squares2_from_python
    iterations = fn(A_rows, int(A_num_columns),
                    rp.ctypes.data_as(_lib.IP), ci.ctypes.data_as(_lib.IP),
                    vals.ctypes.data_as(_lib.DP), len(b), b.ctypes.data_as(_lib.DP),
                    int(A_num_columns), x.ctypes.data_as(_lib.DP),
                    float(min_r_decrease), int(max_iterations), ctypes.byref(final_rr))
    _lib.check(iterations, "cg_least_squares")
    return x, iterations, final_rr.value


def als(user_ids, item_ids, ratings, num_item_factors, num_users, num_items,
        min_r_decrease=0.01, max_iterations=200, algorithm=1):
    """ALS factorisation (``cpp_ls.py:111-169``).

    ``user_factors = uniform(-1,1,num_users*(k+1))`` is drawn before
    ``item_factors = uniform(-1,1,num_items*k)`` from NumPy's global RNG, as
    in the reference.  Returns ``(user_factors, item_factors, iterations)``.
    """
    num_user_factors = num_item_factors + 1
    user_factors = numpy.random.uniform(-1, 1, num_users * num_user_factors)
    item_factors = numpy.random.uniform(-1, 1, num_items * num_item_factors)
    uid = _i32(user_ids)
    iid = _i32(item_ids)
    r = _f64(ratings)
    iterations = _dll.als_from_python(
        uid.ctypes.data_as(_lib.IP), iid.ctypes.data_as(_lib.IP), len(r),
        r.ctypes.data_as(_lib.DP), int(num_item_factors), len(user_factors),
        user_factors.ctypes.data_as(_lib.DP), len(item_factors),
        item_factors.ctypes.data_as(_lib.DP), float(min_r_decrease),
        int(max_iterations), int(algorithm))
    _lib.check(iterations, "als")
    return user_factors, item_factors, iterations
