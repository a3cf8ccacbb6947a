"""Factor consumers on the GPU, with the reference's Python interfaces.

Mirrors:

* ``ALS_Model``           -- ``python/app_local/models.py:645-752``: fold-in of a
  user from ``[(movie_id, rating)]`` (least squares on ``[V, 1]`` with the RAW
  rating, as the reference does), ``is_valid``, ``predict``, ``get_param_list``;
* ``get_recommendations`` -- the scoring / sort / exclusion / rotation of
  ``python/app_local/recommend.py:86-115``;
* ``MovieTable``          -- the device-resident movie side those run on, with
  batched ``fold_in``, ``scores``, ``top_n`` and ``evaluate``;
* ``als_eval`` and ``compute_ranking_agreement`` (in ``evaluation.py``).

Every score is the reference's fp64 expression evaluated in the reference's
order on the GPU (``include/mr_serving.h``), so predictions, rankings and
agreement counts are bit-identical.  There is no CPU fallback: without the HIP
library every entry point raises.
"""

import numpy as np

from . import _lib

ROTATION_SIZE = 4   # app_local/user_data.py:19


def _ip(a):
    return a.ctypes.data_as(_lib.IP)


def _dp(a):
    return a.ctypes.data_as(_lib.DP)


def _llp(a):
    return a.ctypes.data_as(_lib.LLP)


class MovieTable:
    """A trained movie side on one GPU.

    ``als_movie_factors`` (f64[n_als * k]), ``als_movie_ids`` ({standard movie
    id: zero-based ALS id}) and ``movie_medians`` ({movie id: median}) are the
    reference's ``als{k}_item_factors``, ``als{k}_movie_ids`` and
    ``movie_medians_full`` objects (``recommend.py:62-70``).  The movies
    ``predict`` can score are those with a median and factors
    (``models.py:713-715``), kept in ``movie_medians`` order."""

    def __init__(self, num_factors, als_movie_factors, als_movie_ids, movie_medians, device=0):
        self.k = int(num_factors)
        V = np.ascontiguousarray(als_movie_factors, dtype=np.float64).reshape(-1)
        if V.size % self.k:
            raise ValueError("als_movie_factors length is not a multiple of num_factors")
        self.n_als = V.size // self.k
        self.als_movie_ids = als_movie_ids
        self.movie_medians = movie_medians
        cand = [(m, als_movie_ids[m], movie_medians[m]) for m in movie_medians
                if m in als_movie_ids]
        self.cand_mid = np.array([c[0] for c in cand], np.int32)
        self.cand_als = np.array([c[1] for c in cand], np.int32)
        self.cand_med = np.array([c[2] for c in cand], np.float64)
        self.cand_index = {int(m): c for c, m in enumerate(self.cand_mid)}
        # movie id -> candidate index (-1: not a candidate), for array inputs
        self._cand_lut = np.full(int(self.cand_mid.max()) + 1 if len(cand) else 1, -1, np.int32)
        self._cand_lut[self.cand_mid] = np.arange(len(cand), dtype=np.int32)
        L = _lib.lib()
        self._h = L.mr_rec_create(int(device), self.k, self.n_als, _dp(V), len(cand),
                                  _ip(self.cand_als), _ip(self.cand_mid), _dp(self.cand_med))
        if not self._h:
            raise RuntimeError("mr_rec_create failed: " + _lib.last_error())
        self._V = V

    # -- lifetime -----------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().mr_rec_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_candidates(self):
        return len(self.cand_mid)

    def kernel_ms(self):
        ms = np.zeros(6)
        _lib.check(_lib.lib().mr_rec_last_kernel_ms(self._h, _dp(ms)), "mr_rec_last_kernel_ms")
        return dict(zip(["scores", "exclude", "select", "fold_in", "fold_in_svd", "evaluate"],
                        ms.tolist()))

    # -- fold-in --------------------------------------------------------------
    def fold_in(self, rating_lists):
        """``models.py:667-697`` for a batch of users.  Each list is
        ``[(movie_id, rating)]``.  Returns ``(valid bool[B], X f64[B, k+1],
        method int[B])`` (method 1 Cholesky, 2 Jacobi SVD, 0 invalid)."""
        k, K = self.k, self.k + 1
        B = len(rating_lists)
        valid = np.zeros(B, bool)
        rows_u, rows_m, rows_r = [], [], []
        for u, lst in enumerate(rating_lists):
            if len(lst) < k + 1:                       # models.py:672
                continue
            m = [self.als_movie_ids[mid] for mid, _ in lst if mid in self.als_movie_ids]
            if len(m) < k + 1:                         # models.py:694
                continue
            valid[u] = True
            rows_u.append(u)
            rows_m.append(np.asarray(m, np.int32))
            rows_r.append(np.asarray([r for mid, r in lst if mid in self.als_movie_ids],
                                     np.float64))
        X = np.zeros((B, K))
        method = np.zeros(B, np.int32)
        if rows_u:
            n = len(rows_u)
            off = np.zeros(n + 1, np.int64)
            off[1:] = np.cumsum([len(m) for m in rows_m])
            idx = np.ascontiguousarray(np.concatenate(rows_m), np.int32)
            rat = np.ascontiguousarray(np.concatenate(rows_r), np.float64)
            Xv = np.zeros((n, K))
            mv = np.zeros(n, np.int32)
            _lib.check(_lib.lib().mr_rec_fold_in(self._h, n, _llp(off), _ip(idx), _dp(rat),
                                                 _dp(Xv), _ip(mv)), "mr_rec_fold_in")
            X[rows_u] = Xv
            method[rows_u] = mv
        return valid, X, method

    # -- scoring ------------------------------------------------------------
    def scores(self, X):
        """``predict`` of every candidate movie for each user row of ``X``
        (f64[B, k+1]); returns f64[B, num_candidates] (columns in
        ``cand_mid`` order)."""
        X = np.ascontiguousarray(np.atleast_2d(X), np.float64)
        if X.shape[1] != self.k + 1:
            raise ValueError("user factor rows must have k+1 entries")
        out = np.empty((X.shape[0], self.num_candidates))
        _lib.check(_lib.lib().mr_rec_scores(self._h, X.shape[0], _dp(X), _dp(out)),
                   "mr_rec_scores")
        return out

    def top_n(self, X, rated=None, num_results=ROTATION_SIZE * 100):
        """``recommend.py:86-106`` for a batch: per user row the first
        ``num_results`` movies by (score, movie id) descending that are not in
        ``rated[u]`` (any container of movie ids).  Returns a list of
        ``[(score, movie_id)]``."""
        mids, sc, cnt = self.top_n_arrays(X, rated, num_results)
        return [list(zip(sc[u, :cnt[u]].tolist(), mids[u, :cnt[u]].tolist()))
                for u in range(len(cnt))]

    def top_n_arrays(self, X, rated=None, num_results=ROTATION_SIZE * 100):
        """``top_n`` as arrays: movie ids int32[B, n], scores f64[B, n] and
        the count per user (row u is valid up to count[u]).  ``rated`` is a
        sequence of per-user movie-id containers, or -- without any Python
        loop over users -- a CSR pair ``(offsets int64[B + 1], movie_ids)``."""
        X = np.ascontiguousarray(np.atleast_2d(X), np.float64)
        B, N = X.shape[0], int(num_results)
        excl_off = excl = None
        if isinstance(rated, tuple) and len(rated) == 2 and isinstance(rated[0], np.ndarray):
            excl_off, excl = self._exclusions_csr(np.asarray(rated[0], np.int64),
                                                  np.asarray(rated[1], np.int64), B)
        elif rated is not None:
            lists = [[self.cand_index[m] for m in r if m in self.cand_index] for r in rated]
            excl_off = np.zeros(B + 1, np.int64)
            excl_off[1:] = np.cumsum([len(l) for l in lists])
            excl = np.ascontiguousarray(np.concatenate([np.asarray(l, np.int32) for l in lists])
                                        if excl_off[-1] else np.zeros(1, np.int32), np.int32)
        mids = np.zeros((B, N), np.int32)
        sc = np.zeros((B, N))
        cnt = np.zeros(B, np.int32)
        _lib.check(_lib.lib().mr_rec_top_n(
            self._h, B, _dp(X), _llp(excl_off) if excl_off is not None else None,
            _ip(excl) if excl is not None else None, N, _ip(mids), _dp(sc), _ip(cnt)),
            "mr_rec_top_n")
        return mids, sc, cnt

    def _exclusions_csr(self, off, mids, B):
        """Rated-movie lists given as CSR (offsets, movie ids) -> candidate
        indices per user, dropping ids that are not candidates (as the
        container path does), vectorised."""
        if off.shape != (B + 1,) or off[0] != 0 or np.any(np.diff(off) < 0) or off[-1] != len(mids):
            raise ValueError("rated offsets must be int64[B + 1], non-decreasing, from 0 to len(ids)")
        ok = (mids >= 0) & (mids < len(self._cand_lut))
        c = np.full(len(mids), -1, np.int32)
        c[ok] = self._cand_lut[mids[ok]]
        keep = c >= 0
        kept = np.concatenate([[0], np.cumsum(keep, dtype=np.int64)])
        excl_off = np.ascontiguousarray(kept[off], np.int64)
        excl = np.ascontiguousarray(c[keep] if keep.any() else np.zeros(1, np.int32), np.int32)
        return excl_off, excl

    # -- evaluation -----------------------------------------------------------
    def evaluate(self, U, user_rows, test_lists):
        """Per test user: the agreement of ``_test_model``
        (``worker_process.py:229-257``) for factor row ``U[(k+1)*user_rows[t]:]``
        on ``test_lists[t] = [(movie_id, rating)]``.  Returns a dict of arrays:
        agreement (NaN = None), n_agree, n_disagree, pred (per rating), sse,
        n_pred."""
        K = self.k + 1
        U = np.ascontiguousarray(U, np.float64).reshape(-1)
        n_rows = U.size // K
        T = len(test_lists)
        off = np.zeros(T + 1, np.int64)
        off[1:] = np.cumsum([len(l) for l in test_lists])
        cand = np.array([self.cand_index.get(m, -1) for l in test_lists for m, _ in l], np.int32)
        act = np.array([r for l in test_lists for _, r in l], np.float64)
        rows = np.ascontiguousarray(user_rows, np.int32)
        res = {n: np.zeros(T) for n in ("agreement", "sse")}
        for n in ("n_agree", "n_disagree", "n_pred"):
            res[n] = np.zeros(T, np.int64)
        res["pred"] = np.zeros(max(1, off[-1]))
        cand = cand if cand.size else np.zeros(1, np.int32)
        act = act if act.size else np.zeros(1)
        _lib.check(_lib.lib().mr_rec_evaluate(
            self._h, n_rows, _dp(U), T, _ip(rows), _llp(off), _ip(cand), _dp(act),
            _dp(res["agreement"]), _llp(res["n_agree"]), _llp(res["n_disagree"]),
            _dp(res["pred"]), _dp(res["sse"]), _llp(res["n_pred"])), "mr_rec_evaluate")
        res["pred"] = res["pred"][:off[-1]]
        return res


# --------------------------------------------------------------------------
# models.py:645-752 interface
# --------------------------------------------------------------------------
_TABLES = {}


def table_for(num_factors, als_movie_factors, als_movie_ids, movie_medians, device=0):
    """The ``MovieTable`` of these reference objects, built once per process
    (the app loads them once per process too, ``recommend.py:55-58``)."""
    key = (int(num_factors), id(als_movie_factors), id(als_movie_ids), id(movie_medians),
           int(device))
    t = _TABLES.get(key)
    if t is None:
        t = MovieTable(num_factors, als_movie_factors, als_movie_ids, movie_medians, device)
        _TABLES[key] = t
    return t


class ALS_Model:
    """ALS model of a single user (``app_local/models.py:645-752``).

    Same constructor arguments and methods as the reference; the fold-in and
    the predictions run on the GPU.  ``predict`` scores every movie once (one
    batched kernel) and then answers from that vector."""

    def __init__(self, num_factors, movie_ratings, movie_medians, als_movie_factors,
                 als_movie_ids, table=None):
        self._valid = False
        self._table = table or table_for(num_factors, als_movie_factors, als_movie_ids,
                                         movie_medians)
        valid, X, _ = self._table.fold_in([list(movie_ratings)])
        if not valid[0]:
            return
        self.user_factors = X[0]
        self._movie_medians = movie_medians
        self._als_movie_factors = als_movie_factors
        self._als_movie_ids = als_movie_ids
        self._scores = None
        self._valid = True

    def is_valid(self):
        return self._valid

    def predict(self, movie_id):
        """Predicted rating, or None (``models.py:708-733``)."""
        if not self._valid:
            return None
        c = self._table.cand_index.get(movie_id)
        if c is None:
            return None
        if self._scores is None:
            self._scores = self._table.scores(self.user_factors)[0]
        return float(self._scores[c])

    def get_param_list(self):
        """``models.py:740-752``: ("factor i", value) ..., ("user bias", value)."""
        uf = self.user_factors
        out = [("factor " + str(i), uf[i]) for i in range(len(uf) - 1)]
        out.append(("user bias", uf[-1]))
        return out


def get_recommendations(model, user_ratings_dict, num_results=ROTATION_SIZE * 100,
                        rotation=0):
    """``recommend.py:86-115`` for a model built by ``ALS_Model``: the first
    ``num_results`` unrated movies by (score, movie id) descending, and the
    ``rotation``-th slice ``[rotation::4]`` the app returns.  Returns
    ``(rotation_slice, full_list)`` of movie ids."""
    if not model.is_valid():
        raise ValueError("Unable to create model for this algorithm.")
    top = model._table.top_n(model.user_factors, [user_ratings_dict], num_results)[0]
    movie_ids = [m for _, m in top]
    return movie_ids[rotation::ROTATION_SIZE], movie_ids
