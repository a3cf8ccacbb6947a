"""Device-resident ALS context (Python face of ``include/mr_als.h``).

``AlsContext`` keeps the ratings (by-user and by-item CSR), both factor
tables and all solver state in HBM on one MI355X; factors cross PCIe only in
``set_factors`` / ``get_factors``.  It is what ``bench.py`` times and what
the sharded driver (``movie_recommender_amd.distributed``) runs per rank.
"""
import ctypes

import numpy as np

from . import _lib

SOLVERS = {"cg": 0, "cholesky": 1}
OPTIONS = {"fuse_start": 0, "cg_speculate": 1, "wait_timeout_s": 2,
           "cg_onepass": 3, "gram_rhs_mfma": 4, "cg_sweep": 5,
           "peer_timeout_s": 6, "cg_tile_nt": 7, "cg_resident": 8}   # include/mr_als.h


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class AlsContext:
    """One ALS problem resident on one GPU.

    Parameters mirror ``cpp_ls.als``: zero-based int32 ids, fp64 ratings
    (rating minus movie median), ``k`` item factors (users carry k+1).
    For a shard, pass ``user_range``/``item_range`` and the two rating views
    (``item_view=(uid, iid, r)`` holding every rating of the shard's items).
    """

    def __init__(self, user_ids, item_ids, ratings, k, num_users, num_items,
                 device=0, solver="cg", ridge=0.0, timing=False,
                 user_range=None, item_range=None, item_view=None, gram_chunk=None):
        L = _lib.lib()
        self.device = int(device)
        self.k = int(k)
        self.num_users = int(num_users)
        self.num_items = int(num_items)
        self._keep = []
        uid, iid, r = _i32(user_ids), _i32(item_ids), _f64(ratings)
        if gram_chunk is not None:
            _lib.check(L.mr_set_gram_chunk(int(gram_chunk)), "mr_set_gram_chunk")
        if user_range is None and item_range is None and item_view is None:
            h = L.mr_als_create(int(device), self.k, self.num_users, self.num_items,
                                len(r), uid.ctypes.data_as(_lib.IP),
                                iid.ctypes.data_as(_lib.IP), r.ctypes.data_as(_lib.DP))
        else:
            u0, u1 = user_range if user_range is not None else (0, self.num_users)
            i0, i1 = item_range if item_range is not None else (0, self.num_items)
            if item_view is None:
                item_view = (uid, iid, r)
            vu, vi, vr = _i32(item_view[0]), _i32(item_view[1]), _f64(item_view[2])
            self._keep += [vu, vi, vr]
            h = L.mr_als_create_shard(
                int(device), self.k, self.num_users, self.num_items,
                len(r), uid.ctypes.data_as(_lib.IP), iid.ctypes.data_as(_lib.IP),
                r.ctypes.data_as(_lib.DP),
                len(vr), vu.ctypes.data_as(_lib.IP), vi.ctypes.data_as(_lib.IP),
                vr.ctypes.data_as(_lib.DP), int(u0), int(u1), int(i0), int(i1))
        if gram_chunk is not None:
            L.mr_set_gram_chunk(2048)
        if not h:
            raise RuntimeError(f"mr_als_create failed: {_lib.last_error()}")
        self._h = h
        self._comm = None
        self.set_solver(solver, ridge)
        if timing:
            self.set_timing(True)

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().mr_als_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- configuration -------------------------------------------------------
    def set_solver(self, solver="cg", ridge=0.0):
        _lib.check(_lib.lib().mr_als_set_solver(self._h, SOLVERS[solver], float(ridge)),
                   "mr_als_set_solver")

    def set_option(self, name, value):
        """Engine option (``mr_als_set_option``): ``fuse_start``,
        ``cg_speculate`` (0/1) or ``wait_timeout_s``."""
        _lib.check(_lib.lib().mr_als_set_option(self._h, OPTIONS[name], float(value)),
                   "mr_als_set_option")

    def set_timing(self, enable=True):
        _lib.check(_lib.lib().mr_als_set_timing(self._h, int(bool(enable))),
                   "mr_als_set_timing")

    def set_comm(self, comm_struct, user_begin, item_begin):
        ub = np.ascontiguousarray(user_begin, dtype=np.int64)
        ib = np.ascontiguousarray(item_begin, dtype=np.int64)
        self._comm = (comm_struct, ub, ib)
        _lib.check(_lib.lib().mr_als_set_comm(self._h, ctypes.byref(comm_struct),
                                              ub.ctypes.data_as(_lib.LLP),
                                              ib.ctypes.data_as(_lib.LLP)),
                   "mr_als_set_comm")

    # -- factors -------------------------------------------------------------
    def set_factors(self, U, V):
        U = _f64(U).reshape(-1)
        V = _f64(V).reshape(-1)
        assert U.size == self.num_users * (self.k + 1) and V.size == self.num_items * self.k
        _lib.check(_lib.lib().mr_als_set_factors(self._h, U.ctypes.data_as(_lib.DP),
                                                 V.ctypes.data_as(_lib.DP)),
                   "mr_als_set_factors")

    def init_factors(self, seed=0):
        """Seeded uniform(-1, 1) factors generated on the device."""
        _lib.check(_lib.lib().mr_als_init_factors(self._h, int(seed)), "mr_als_init_factors")

    def get_factors(self):
        U = np.empty(self.num_users * (self.k + 1))
        V = np.empty(self.num_items * self.k)
        _lib.check(_lib.lib().mr_als_get_factors(self._h, U.ctypes.data_as(_lib.DP),
                                                 V.ctypes.data_as(_lib.DP)),
                   "mr_als_get_factors")
        return U, V

    # -- solving ---------------------------------------------------------------
    def run(self, min_r_decrease=0.01, max_iterations=200):
        """The reference loop (``matrix.cpp:814-892``); returns its iteration index."""
        return _lib.check(_lib.lib().mr_als_run(self._h, float(min_r_decrease),
                                                int(max_iterations)), "mr_als_run")

    def cg_grid(self, side, resident=False, nt=False):
        """Workgroups of the side's CG iteration kernel (one-pass, or the
        resident solve: 0 when unavailable) for one tile-load policy."""
        return _lib.lib().mr_als_cg_grid(self._h, 0 if side == "users" else 1,
                                         int(bool(resident)), int(bool(nt)))

    def iterate(self, n=1):
        """Exactly ``n`` ALS iterations (user + item half-step each)."""
        _lib.check(_lib.lib().mr_als_iterate(self._h, int(n)), "mr_als_iterate")

    def half_step(self, side, min_r_decrease=None, max_iteration=None):
        """One half-step; returns (CG iterations, final rr).  Default CG
        arguments are the reference's (0.01, 200); others go through
        ``mr_als_half_step_ex``."""
        rr = ctypes.c_double(0)
        sd = 0 if side in (0, "users") else 1
        if min_r_decrease is None and max_iteration is None:
            its = _lib.check(_lib.lib().mr_als_half_step(self._h, sd, ctypes.byref(rr)),
                             "mr_als_half_step")
        else:
            its = _lib.check(_lib.lib().mr_als_half_step_ex(
                self._h, sd, 0.01 if min_r_decrease is None else float(min_r_decrease),
                200 if max_iteration is None else int(max_iteration), ctypes.byref(rr)),
                "mr_als_half_step_ex")
        return its, rr.value

    def build_normal_equations(self, side):
        _lib.check(_lib.lib().mr_als_build_normal_equations(
            self._h, 0 if side in (0, "users") else 1), "mr_als_build_normal_equations")

    def normal_equations(self, side, entities):
        """(G, c) of local entities as last built: users K=k+1, items K=k."""
        user = side in (0, "users")
        K = self.k + 1 if user else self.k
        ents = _i32(entities)
        G = np.empty((len(ents), K, K))
        c = np.empty((len(ents), K))
        _lib.check(_lib.lib().mr_als_get_normal_equations(
            self._h, 0 if user else 1, len(ents), ents.ctypes.data_as(_lib.IP),
            G.ctypes.data_as(_lib.DP), c.ctypes.data_as(_lib.DP)), "mr_als_get_normal_equations")
        return G, c

    def local_size(self, side):
        """(first global id, count, ratings held) of this context's entities
        of ``side`` (a shard owns a contiguous range)."""
        v = [ctypes.c_longlong(0) for _ in range(3)]
        _lib.check(_lib.lib().mr_als_local_size(self._h, 0 if side in (0, "users") else 1,
                                                *[ctypes.byref(x) for x in v]),
                   "mr_als_local_size")
        return tuple(int(x.value) for x in v)

    def layout(self, side):
        """The side's device CSR (off, idx, val) and Gram work list
        (begin, len, entity, slab) as built on the GPU (local entities)."""
        L = _lib.lib()
        user = side in (0, "users")
        sd = 0 if user else 1
        _, E, nnz = self.local_size(side)
        off = np.empty(E + 1, np.int64)
        _lib.check(L.mr_als_get_layout(self._h, sd, off.ctypes.data_as(_lib.LLP), None, None,
                                       None, None, None, None), "mr_als_get_layout")
        assert int(off[-1]) == nnz
        nw = int(L.mr_als_work_items(self._h, sd))
        idx = np.empty(nnz, np.int32)
        val = np.empty(nnz, np.float32)
        wb = np.empty(nw, np.int64)
        wl, we, ws = (np.empty(nw, np.int32) for _ in range(3))
        _lib.check(L.mr_als_get_layout(
            self._h, sd, None, idx.ctypes.data_as(_lib.IP), val.ctypes.data_as(_lib.FP),
            wb.ctypes.data_as(_lib.LLP), wl.ctypes.data_as(_lib.IP), we.ctypes.data_as(_lib.IP),
            ws.ctypes.data_as(_lib.IP)), "mr_als_get_layout")
        return off, idx, val, (wb, wl, we, ws)

    def cg_vectors(self, side):
        """(r, p, q) of the side's last CG solve over the local entities, fp64
        (users: k+1 per user)."""
        user = side in (0, "users")
        _, E, _ = self.local_size(side)
        n = E * (self.k + 1) if user else E * self.k
        out = [np.empty(n) for _ in range(3)]
        _lib.check(_lib.lib().mr_als_get_cg_vectors(
            self._h, 0 if user else 1, *[a.ctypes.data_as(_lib.DP) for a in out]),
            "mr_als_get_cg_vectors")
        return tuple(out)

    def sync(self):
        _lib.check(_lib.lib().mr_als_sync(self._h), "mr_als_sync")

    def stream(self):
        return _lib.lib().mr_als_stream(self._h)

    def stats(self):
        s = _lib.MrStats()
        _lib.check(_lib.lib().mr_als_get_stats(self._h, ctypes.byref(s)), "mr_als_get_stats")
        return s.as_dict()

    def reset_stats(self):
        _lib.check(_lib.lib().mr_als_reset_stats(self._h), "mr_als_reset_stats")

    @property
    def num_ratings(self):
        return int(_lib.lib().mr_als_num_ratings(self._h))

    def predict(self, user_ids, item_ids):
        uid, iid = _i32(user_ids), _i32(item_ids)
        out = np.empty(len(uid))
        _lib.check(_lib.lib().mr_als_predict(self._h, len(uid), uid.ctypes.data_as(_lib.IP),
                                             iid.ctypes.data_as(_lib.IP),
                                             out.ctypes.data_as(_lib.DP)), "mr_als_predict")
        return out


def device_count():
    return int(_lib.lib().mr_device_count())
