"""CPU: the C-ABI library loads and exports every symbol declared in include/*.h."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("cpp_ls_lib.h", "mr_als.h", "mr_serving.h", "mr_prep.h", "mr_similar.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"typedef struct \w+ \{.*?\} \w+;", "", src, flags=re.S)
        for m in re.finditer(r"^[\w\s\*]+?\b(\w+)\s*\(", src, flags=re.M):
            name = m.group(1)
            if name not in ("if", "while", "for", "return", "sizeof"):
                names.append(name)
    return sorted(set(names))


def test_headers_declare_reference_abi():
    names = declared_functions()
    for ref in ["set_thread_count", "get_thread_count", "cg_least_squares_from_python",
                "cg_least_squares2_from_python", "als_from_python"]:
        assert ref in names


def test_library_exports_every_declared_symbol():
    from movie_recommender_amd import _lib
    L = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding table covers them all
    assert set(declared_functions()) <= set(_lib.SIGNATURES)


def test_thread_count_roundtrip_without_gpu():
    """cpp_ls.has_dll_loaded (cpp_ls.py:23-36) needs no device."""
    from movie_recommender_amd import cpp_ls
    assert cpp_ls.has_dll_loaded()
    cpp_ls.set_thread_count(77777)
    assert cpp_ls.get_thread_count() == 77777


def test_library_is_gfx950_only():
    so = os.path.join(ROOT, "movie_recommender_amd", "lib", "cpp_ls_lib.so")
    blob = open(so, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets  # code objects for MI355X only


def test_no_gpu_means_clean_error():
    from movie_recommender_amd import _lib
    L = _lib.lib()
    if L.mr_device_count() > 0:
        pytest.skip("device present")
    import numpy as np
    from movie_recommender_amd import cpp_ls
    u = np.zeros(4, np.int32)
    with pytest.raises(RuntimeError):
        cpp_ls.als(u, u, np.ones(4), 1, 1, 1)


@pytest.mark.gpu
def test_reference_wrapper_calling_convention(gpu):
    """The library called exactly as the reference wrapper does
    (cpp/python/cpp_ls.py:89-167): a fresh CDLL with NO argtypes / restype,
    bare Python ints, ``ctypes.c_double(...)`` for min_r_decrease, id arrays
    passed as POINTER(c_double), ``ctypes.byref`` for final_rr."""
    import ctypes
    from movie_recommender_amd import _lib
    from conftest import load_golden, rel_err
    dll = ctypes.CDLL(_lib.LIB_PATH)      # no prototypes declared on this handle
    dll.set_thread_count(77)
    assert dll.get_thread_count() == 77
    d = load_golden("als_dense_40x45_k3.npz")
    uid = np.ascontiguousarray(d["user_ids"], np.int32)
    iid = np.ascontiguousarray(d["item_ids"], np.int32)
    r = np.ascontiguousarray(d["ratings"], np.float64)
    U = np.array(d["U0"], np.float64)
    V = np.array(d["V0"], np.float64)
    dp = ctypes.POINTER(ctypes.c_double)
    it = dll.als_from_python(uid.ctypes.data_as(dp), iid.ctypes.data_as(dp), len(r),
                             r.ctypes.data_as(dp), 3, len(U), U.ctypes.data_as(dp), len(V),
                             V.ctypes.data_as(dp), ctypes.c_double(0.01), 200, 1)
    assert it == int(d["ret"])
    assert rel_err(U, d["U"]) <= 1e-5 and rel_err(V, d["V"]) <= 1e-5
    g = load_golden("cg_dense_200x50.npz")
    rp = np.ascontiguousarray(g["row_ptr"], np.int32)
    ci = np.ascontiguousarray(g["col_idx"], np.int32)
    v = np.ascontiguousarray(g["vals"], np.float64)
    b = np.ascontiguousarray(g["b"], np.float64)
    x = np.array(g["x0"], np.float64).reshape(-1, 1)
    ip = ctypes.POINTER(ctypes.c_int)
    final_rr = ctypes.c_double(0)
    it = dll.cg_least_squares_from_python(len(rp) - 1, int(g["ncols"]), rp.ctypes.data_as(ip),
                                          ci.ctypes.data_as(ip), v.ctypes.data_as(dp), len(b),
                                          b.ctypes.data_as(dp), int(g["ncols"]),
                                          x.ctypes.data_as(dp), ctypes.c_double(0.01), 200,
                                          ctypes.byref(final_rr))
    assert it == int(g["iterations"])
    assert rel_err(x.ravel(), g["x"]) <= 1e-9


def test_engine_option_table_matches_header():
    """engine.OPTIONS (the names set_option accepts) is exactly the
    MR_OPT_* enum of include/mr_als.h."""
    from movie_recommender_amd.engine import OPTIONS
    src = open(os.path.join(ROOT, "include", "mr_als.h")).read()
    enum = {m.group(1).lower(): int(m.group(2))
            for m in re.finditer(r"MR_OPT_(\w+)\s*=\s*(\d+)", src)}
    assert OPTIONS == enum
