"""ctypes binding of ``movie_recommender_amd/lib/cpp_ls_lib.so`` (gfx950 HIP).

The shared library exports the reference ABI (``include/cpp_ls_lib.h``), the
device-resident engine API (``include/mr_als.h``), the factor consumers
(``include/mr_serving.h``), the general sparse least squares
(``include/mr_cg.h``), the training-set preparation
(``include/mr_prep.h``) and the similar-movies database
(``include/mr_similar.h``).  There is no CPU
fallback: if the library is missing or cannot load, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MR_LIB_PATH") or os.path.join(HERE, "lib", "cpp_ls_lib.so")

K_NAMES = ["gram_users", "gram_items", "slab_reduce", "matvec_users",
           "matvec_items", "cg_update", "cg_control", "solve", "cg_start_split",
           "resident_users", "resident_items", "exchange"]


class MrStats(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int),
                ("last_cg_users", ctypes.c_int),
                ("last_cg_items", ctypes.c_int),
                ("cg_users_total", ctypes.c_longlong),
                ("cg_items_total", ctypes.c_longlong),
                ("last_final_rr", ctypes.c_double),
                ("nonpd_users", ctypes.c_longlong),
                ("nonpd_items", ctypes.c_longlong),
                ("kernel_ms", ctypes.c_double * len(K_NAMES)),
                ("kernel_launches", ctypes.c_longlong * len(K_NAMES)),
                ("phase_ms", ctypes.c_double * 4),
                ("kernel_units", ctypes.c_longlong * len(K_NAMES)),
                ("peer_wait_ms", ctypes.c_double),
                ("peer_reductions", ctypes.c_longlong)]

    def as_dict(self):
        return {
            "iterations": self.iterations,
            "last_cg_users": self.last_cg_users,
            "last_cg_items": self.last_cg_items,
            "cg_users_total": self.cg_users_total,
            "cg_items_total": self.cg_items_total,
            "last_final_rr": self.last_final_rr,
            "nonpd_users": self.nonpd_users,
            "nonpd_items": self.nonpd_items,
            "kernel_ms": {n: self.kernel_ms[i] for i, n in enumerate(K_NAMES)},
            "kernel_launches": {n: self.kernel_launches[i] for i, n in enumerate(K_NAMES)},
            "phase_ms": {"gram_users": self.phase_ms[0], "solve_users": self.phase_ms[1],
                         "gram_items": self.phase_ms[2], "solve_items": self.phase_ms[3]},
            "kernel_units": {n: self.kernel_units[i] for i, n in enumerate(K_NAMES)},
            "peer_wait_ms": self.peer_wait_ms,
            "peer_reductions": self.peer_reductions,
        }


ALLREDUCE_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_double), ctypes.c_int)
ALLGATHER_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_float), ctypes.c_longlong,
                                ctypes.POINTER(ctypes.c_longlong), ctypes.c_int)


CG_K_NAMES = ["spmv_a", "spmv_at", "update", "setup"]


class MrCgStats(ctypes.Structure):
    _fields_ = [("last_iterations", ctypes.c_int),
                ("iterations_total", ctypes.c_longlong),
                ("solve_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double * len(CG_K_NAMES)),
                ("kernel_launches", ctypes.c_longlong * len(CG_K_NAMES)),
                ("rows", ctypes.c_longlong), ("cols", ctypes.c_longlong),
                ("nnz", ctypes.c_longlong),
                ("blocks_a", ctypes.c_longlong), ("blocks_at", ctypes.c_longlong),
                ("block_max_nnz", ctypes.c_longlong), ("block_max_rows", ctypes.c_longlong)]

    def as_dict(self):
        return {"last_iterations": self.last_iterations,
                "iterations_total": self.iterations_total, "solve_ms": self.solve_ms,
                "kernel_ms": {n: self.kernel_ms[i] for i, n in enumerate(CG_K_NAMES)},
                "kernel_launches": {n: self.kernel_launches[i] for i, n in enumerate(CG_K_NAMES)},
                "rows": self.rows, "cols": self.cols, "nnz": self.nnz,
                "blocks_a": self.blocks_a, "blocks_at": self.blocks_at,
                "block_max_nnz": self.block_max_nnz, "block_max_rows": self.block_max_rows}


class MrComm(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p),
                ("rank", ctypes.c_int),
                ("world", ctypes.c_int),
                ("allreduce_f64", ALLREDUCE_CB),
                ("allgather_rows", ALLGATHER_CB)]


_lib = None

IP = ctypes.POINTER(ctypes.c_int)
DP = ctypes.POINTER(ctypes.c_double)
FP = ctypes.POINTER(ctypes.c_float)
LLP = ctypes.POINTER(ctypes.c_longlong)
VP = ctypes.c_void_p

# name -> (restype, argtypes); every symbol of include/*.h
SIGNATURES = {
    # reference ABI (include/cpp_ls_lib.h)
    "set_thread_count": (None, [ctypes.c_int]),
    "get_thread_count": (ctypes.c_int, []),
    "cg_least_squares_from_python": (
        ctypes.c_int, [ctypes.c_int, ctypes.c_int, IP, IP, DP, ctypes.c_int, DP,
                       ctypes.c_int, DP, ctypes.c_double, ctypes.c_int, DP]),
    "cg_least_squares2_from_python": (
        ctypes.c_int, [ctypes.c_int, ctypes.c_int, IP, IP, DP, ctypes.c_int, DP,
                       ctypes.c_int, DP, ctypes.c_double, ctypes.c_int, DP]),
    "als_from_python": (
        ctypes.c_int, [IP, IP, ctypes.c_int, DP, ctypes.c_int, ctypes.c_int, DP,
                       ctypes.c_int, DP, ctypes.c_double, ctypes.c_int, ctypes.c_int]),
    # engine API (include/mr_als.h)
    "mr_als_create": (VP, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_longlong, IP, IP, DP]),
    "mr_als_create_shard": (VP, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_longlong, IP, IP, DP,
                                 ctypes.c_longlong, IP, IP, DP,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "mr_als_set_comm": (ctypes.c_int, [VP, ctypes.POINTER(MrComm), LLP, LLP]),
    "mr_rccl_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "mr_als_set_rccl": (ctypes.c_int, [VP, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       LLP, LLP]),
    "mr_als_peer_handle": (ctypes.c_int, [VP, ctypes.c_void_p]),
    "mr_als_set_peer": (ctypes.c_int, [VP, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "mr_als_peer_selftest": (ctypes.c_int, [VP]),
    "mr_als_weights_bf16": (ctypes.c_int, [VP, ctypes.c_int]),
    "mr_als_peer_latency": (ctypes.c_int, [VP, ctypes.c_int, DP]),
    "mr_als_destroy": (None, [VP]),
    "mr_als_set_factors": (ctypes.c_int, [VP, DP, DP]),
    "mr_als_get_factors": (ctypes.c_int, [VP, DP, DP]),
    "mr_als_set_solver": (ctypes.c_int, [VP, ctypes.c_int, ctypes.c_double]),
    "mr_als_set_timing": (ctypes.c_int, [VP, ctypes.c_int]),
    "mr_als_set_option": (ctypes.c_int, [VP, ctypes.c_int, ctypes.c_double]),
    "mr_set_gram_chunk": (ctypes.c_int, [ctypes.c_int]),
    "mr_als_run": (ctypes.c_int, [VP, ctypes.c_double, ctypes.c_int]),
    "mr_als_iterate": (ctypes.c_int, [VP, ctypes.c_int]),
    "mr_als_half_step": (ctypes.c_int, [VP, ctypes.c_int, DP]),
    "mr_als_work_items": (ctypes.c_longlong, [VP, ctypes.c_int]),
    "mr_als_cg_grid": (ctypes.c_int, [VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "mr_als_local_size": (ctypes.c_int, [VP, ctypes.c_int, LLP, LLP, LLP]),
    "mr_als_get_layout": (ctypes.c_int, [VP, ctypes.c_int, LLP, IP, FP, LLP, IP, IP, IP]),
    "mr_als_init_factors": (ctypes.c_int, [VP, ctypes.c_ulonglong]),
    "mr_als_get_cg_vectors": (ctypes.c_int, [VP, ctypes.c_int, DP, DP, DP]),
    "mr_als_half_step_ex": (ctypes.c_int, [VP, ctypes.c_int, ctypes.c_double, ctypes.c_int, DP]),
    "mr_als_build_normal_equations": (ctypes.c_int, [VP, ctypes.c_int]),
    "mr_als_get_normal_equations": (ctypes.c_int, [VP, ctypes.c_int, ctypes.c_int, IP, DP, DP]),
    "mr_als_get_stats": (ctypes.c_int, [VP, ctypes.POINTER(MrStats)]),
    "mr_als_reset_stats": (ctypes.c_int, [VP]),
    "mr_als_sync": (ctypes.c_int, [VP]),
    "mr_als_stream": (VP, [VP]),
    "mr_als_num_ratings": (ctypes.c_longlong, [VP]),
    "mr_als_device_tables": (ctypes.c_int, [VP, ctypes.POINTER(FP), ctypes.POINTER(FP),
                                            ctypes.POINTER(FP), IP]),
    "mr_als_predict": (ctypes.c_int, [VP, ctypes.c_longlong, IP, IP, DP]),
    "mr_test_pack_rows": (ctypes.c_int, [ctypes.c_int, ctypes.c_longlong, ctypes.c_int, FP, FP,
                                         ctypes.c_longlong, ctypes.c_longlong, FP, FP]),
    "mr_test_xsum": (ctypes.c_int, [ctypes.c_int, DP, ctypes.c_longlong, ctypes.c_int, DP]),
    "mr_test_unstage_rows": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, LLP,
                                            ctypes.c_longlong, ctypes.c_int, FP, FP, FP, FP]),
    # general sparse least squares (include/mr_cg.h)
    "mr_cg_create": (VP, [ctypes.c_int, ctypes.c_int, ctypes.c_int, IP, IP, DP]),
    "mr_cg_destroy": (None, [VP]),
    "mr_cg_solve": (ctypes.c_int, [VP, DP, DP, ctypes.c_double, ctypes.c_int, DP]),
    "mr_cg_set_timing": (ctypes.c_int, [VP, ctypes.c_int]),
    "mr_cg_get_stats": (ctypes.c_int, [VP, ctypes.POINTER(MrCgStats)]),
    "mr_cg_reset_stats": (ctypes.c_int, [VP]),
    # factor consumers (include/mr_serving.h)
    "mr_rec_create": (VP, [ctypes.c_int, ctypes.c_int, ctypes.c_int, DP, ctypes.c_int, IP, IP,
                           DP]),
    "mr_rec_destroy": (None, [VP]),
    "mr_rec_num_candidates": (ctypes.c_int, [VP]),
    "mr_rec_fold_in": (ctypes.c_int, [VP, ctypes.c_int, LLP, IP, DP, DP, IP]),
    "mr_rec_scores": (ctypes.c_int, [VP, ctypes.c_int, DP, DP]),
    "mr_rec_top_n": (ctypes.c_int, [VP, ctypes.c_int, DP, LLP, IP, ctypes.c_int, IP, DP, IP]),
    "mr_rec_evaluate": (ctypes.c_int, [VP, ctypes.c_int, DP, ctypes.c_int, IP, LLP, IP, DP, DP,
                                       LLP, LLP, DP, DP, LLP]),
    "mr_rank_agreement": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, LLP, DP, DP, DP, LLP,
                                         LLP]),
    "mr_rec_last_kernel_ms": (ctypes.c_int, [VP, DP]),
    # training-set preparation (include/mr_prep.h)
    "mr_prep_create": (VP, [ctypes.c_int, ctypes.c_longlong, IP, IP, DP]),
    "mr_prep_destroy": (None, [VP]),
    "mr_prep_id_bounds": (ctypes.c_int, [VP, IP, IP]),
    "mr_prep_medians": (ctypes.c_int, [VP, DP]),
    "mr_prep_shrink": (ctypes.c_int, [VP, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_ubyte), IP, LLP, IP, IP]),
    "mr_prep_first_appearance": (ctypes.c_int, [VP, ctypes.c_int, LLP, LLP, LLP]),
    "mr_prep_convert": (ctypes.c_int, [VP, IP, IP, DP, IP, IP, DP]),
    "mr_prep_last_ms": (ctypes.c_double, [VP]),
    # similar movies (include/mr_similar.h)
    "mr_similar_create": (VP, [ctypes.c_int, ctypes.c_int, ctypes.c_int, LLP, IP,
                               ctypes.POINTER(ctypes.c_ubyte), ctypes.POINTER(ctypes.c_ulonglong),
                               ctypes.POINTER(ctypes.c_ubyte)]),
    "mr_similar_destroy": (None, [VP]),
    "mr_similar_find": (ctypes.c_int, [VP, ctypes.c_int, IP, DP, ctypes.c_int, ctypes.c_int, IP,
                                       DP, IP]),
    "mr_similar_last_ms": (ctypes.c_double, [VP]),
    "mr_last_error": (ctypes.c_char_p, []),
    "mr_device_count": (ctypes.c_int, []),
    "mr_device_pci_bus_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
}


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Load the HIP library (raises if it is not built: no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
            " or `make -C movie_recommender_amd/csrc`")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("MR_LIB_PATH") and not hasattr(L, name):
            continue  # an older A/B variant (tools/build_var.sh) lacks newer entry points
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    m = lib().mr_last_error()
    return m.decode() if m else ""


def check(rc, what):
    if rc is None or (isinstance(rc, int) and rc < 0):
        raise RuntimeError(f"{what} failed: {last_error()}")
    return rc
