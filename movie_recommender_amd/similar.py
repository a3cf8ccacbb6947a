"""Similar-movies database on the GPU, with the reference's interface.

Mirrors ``python/full_data/build_similar_movies_db.py``:

* ``SimilarMovieFinder(movie_genres, movie_ratings, buff_limit, buff_point)``
  with ``find_similar_movie``, ``find_movie_index`` and ``tune``
  (``:19-211``);
* ``build_similar_movies(...)`` -- what ``build_locally`` /
  ``_find_similar_movies`` produce (``:255-291``,
  ``movie_lens_data_proc.py:657-700``): ``{movie_id: [similar movie ids]}``
  for every movie with at least one similar movie, in list order.

All pair statistics and the ranking run on the GPU (``include/mr_similar.h``)
and are exact; the host keeps the reference's per-parameter boost formula
(Python ``math``) and the one-pair helper ``tune`` needs.  Ratings must be
multiples of 0.5 (MovieLens).  There is no CPU fallback for the search.
"""
import ctypes
import math

import numpy

from . import _lib


def boost_table(buff_limit, buff_point, n_max):
    """``1.0 + buff(n)`` for n = 0 .. n_max, by the reference's expressions
    (``_scaled_dot_product:101-108``) in Python floats."""
    x_limit = 3 * math.exp(buff_limit)
    out = numpy.ones(n_max + 1)
    for n in range(3, n_max + 1):
        x = 3 + (x_limit - 3) * (n - 3) / (buff_point - 3)
        buff = math.log(x) - math.log(3)
        if buff > buff_limit:
            buff = buff_limit
        if buff < 0:
            buff = 0
        out[n] = 1.0 + buff
    return out


class SimilarMovieFinder:
    """GPU ``SimilarMovieFinder``: ``movie_genres`` = {movie id: set of genre
    ids}, ``movie_ratings`` = [(movie_id, {user_id: rating})]."""

    def __init__(self, movie_genres, movie_ratings, buff_limit=0.05, buff_point=100, device=0,
                 _arrays=None):
        self.movie_genres = movie_genres
        self.movie_ratings = movie_ratings
        self.buff_limit = buff_limit
        self.buff_point = buff_point
        if _arrays is not None:
            self._setup(*_arrays, device=device)
            return
        M = len(movie_ratings)
        users = {}
        off = numpy.zeros(M + 1, numpy.int64)
        uid, r2 = [], []
        for m, (_, ratings) in enumerate(movie_ratings):
            for u, r in ratings.items():
                uid.append(users.setdefault(u, len(users)))
                x = 2.0 * r
                if x != int(x) or not 0 <= x <= 255:
                    raise ValueError("ratings must be multiples of 0.5 in [0, 127.5]")
                r2.append(int(x))
            off[m + 1] = len(uid)
        genre_index = {}
        for gs in movie_genres.values():
            for g in gs:
                genre_index.setdefault(g, len(genre_index))
        if len(genre_index) > 64:
            raise ValueError("at most 64 distinct genre ids are supported")
        mask = numpy.zeros(max(M, 1), numpy.uint64)
        has = numpy.zeros(max(M, 1), numpy.uint8)
        for m, (mid, _) in enumerate(movie_ratings):
            if mid in movie_genres:
                gs = movie_genres[mid]
                if len(gs) == 0:
                    raise ValueError(f"movie {mid} has an empty genre set")
                has[m] = 1
                mask[m] = sum(1 << genre_index[g] for g in gs)
        self._setup(numpy.array([mid for mid, _ in movie_ratings], numpy.int64), off,
                    numpy.asarray(uid, numpy.int32), numpy.asarray(r2, numpy.uint8), len(users),
                    mask, has, device=device)

    @classmethod
    def from_arrays(cls, movie_ids, off, user_index, rating2, n_users, genre_mask, has_genres,
                    buff_limit=0.05, buff_point=100, device=0):
        """Build from flat arrays (the CSR of ``movie_ratings`` with dense user
        indices and 2 * rating), for data too large for Python dicts."""
        return cls(None, None, buff_limit, buff_point, device,
                   _arrays=(numpy.asarray(movie_ids, numpy.int64),
                            numpy.ascontiguousarray(off, numpy.int64),
                            numpy.ascontiguousarray(user_index, numpy.int32),
                            numpy.ascontiguousarray(rating2, numpy.uint8), int(n_users),
                            numpy.ascontiguousarray(genre_mask, numpy.uint64),
                            numpy.ascontiguousarray(has_genres, numpy.uint8)))

    def _setup(self, ids, off, uid, r2, n_users, mask, has, device=0):
        M = len(ids)
        self._uid = uid if len(uid) else numpy.zeros(1, numpy.int32)
        self._r2 = r2 if len(r2) else numpy.zeros(1, numpy.uint8)
        self._off = off
        self._max_deg = int(numpy.diff(off).max()) if M else 0
        self._ids = ids
        self._index = {int(mid): m for m, mid in enumerate(ids)}
        mask = mask if len(mask) else numpy.zeros(1, numpy.uint64)
        has = has if len(has) else numpy.zeros(1, numpy.uint8)
        self._h = _lib.lib().mr_similar_create(
            int(device), M, int(n_users), off.ctypes.data_as(_lib.LLP),
            self._uid.ctypes.data_as(_lib.IP),
            self._r2.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)),
            mask.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)),
            has.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)))
        if not self._h:
            raise RuntimeError("mr_similar_create failed: " + _lib.last_error())

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().mr_similar_destroy(self._h)
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

    def last_ms(self):
        return float(_lib.lib().mr_similar_last_ms(self._h))

    def find_movie_index(self, movie_id):
        """Index of movie_id in ``movie_ratings``, or -1 (``:127-135``)."""
        return self._index.get(movie_id, -1)

    def find_many(self, indices=None, num_results=20):
        """``find_similar_movie`` for many list indices at once (all when
        None).  Returns (index int32[Q, num_results], score f64[Q,
        num_results], count int32[Q])."""
        M = len(self._ids)
        q = None if indices is None else numpy.ascontiguousarray(indices, numpy.int32)
        Q = M if q is None else len(q)
        boost = boost_table(self.buff_limit, self.buff_point, max(self._max_deg, 3))
        oj = numpy.zeros((max(Q, 1), num_results), numpy.int32)
        os_ = numpy.zeros((max(Q, 1), num_results))
        oc = numpy.zeros(max(Q, 1), numpy.int32)
        _lib.check(_lib.lib().mr_similar_find(
            self._h, Q, q.ctypes.data_as(_lib.IP) if q is not None else None,
            boost.ctypes.data_as(_lib.DP), len(boost), int(num_results),
            oj.ctypes.data_as(_lib.IP), os_.ctypes.data_as(_lib.DP),
            oc.ctypes.data_as(_lib.IP)), "mr_similar_find")
        return oj[:Q], os_[:Q], oc[:Q]

    def find_similar_movie(self, movie_id_index, num_results=20):
        """(movie_ids, scores) of the most similar movies (``:138-163``)."""
        oj, os_, oc = self.find_many([movie_id_index], num_results)
        c = int(oc[0])
        if c == 0:
            return [], []
        return tuple(int(x) for x in self._ids[oj[0, :c]]), tuple(float(x) for x in os_[0, :c])

    def _scaled_dot_product(self, i1, i2):
        """One pair, as the reference (``:69-112``): used by ``tune`` only."""
        ratings1 = self.movie_ratings[i1][1]
        ratings2 = self.movie_ratings[i2][1]
        if len(ratings1) > len(ratings2):
            ratings1, ratings2 = ratings2, ratings1
        r1 = [ratings1[u] for u in ratings1 if u in ratings2]
        r2 = [ratings2[u] for u in ratings1 if u in ratings2]
        if len(r1) < 3:
            return 0.0, len(r1), 0.0
        r1, r2 = numpy.array(r1), numpy.array(r2)
        similarity = r1.dot(r2) / (numpy.linalg.norm(r1) * numpy.linalg.norm(r2))
        boost = boost_table(self.buff_limit, self.buff_point, len(r1))[len(r1)]
        return similarity * boost, len(r1), similarity

    def tune(self, movie_id1, movie_id2, top_n, expected_search_size):
        """``tune`` (``:166-211``): set buff_point to the pair's common
        reviewers and raise buff_limit until movie_id2 is in movie_id1's
        top_n."""
        index1 = self.find_movie_index(movie_id1)
        index2 = self.find_movie_index(movie_id2)
        _, common, _ = self._scaled_dot_product(index1, index2)
        self.buff_point = common
        self.buff_limit = 0
        while self.buff_limit < 2:
            movie_ids, scores = self.find_similar_movie(index1, expected_search_size * 2)
            if movie_id2 in movie_ids[:top_n]:
                return
            top_score = scores[0]
            score, _, _ = self._scaled_dot_product(index1, index2)
            self.buff_limit = self.buff_limit * top_score / score + 0.01


def build_similar_movies(movie_genres, movie_ratings, buff_point, buff_limit, num_results=20,
                         device=0):
    """``{movie_id: [similar movie ids]}`` for every movie of
    ``movie_ratings`` with at least one similar movie (list order)."""
    with SimilarMovieFinder(movie_genres, movie_ratings, buff_limit, buff_point, device) as f:
        oj, _, oc = f.find_many(None, num_results)
        out = {}
        for m in range(len(movie_ratings)):
            if oc[m]:
                out[int(f._ids[m])] = [int(x) for x in f._ids[oj[m, :oc[m]]]]
        return out


# --------------------------------------------------------------------------
# Movie-movie cosine similarity on the ALS factor layout (north star: "the
# movie-movie cosine-similarity pass reuses the same factor layout")
# --------------------------------------------------------------------------
def similar_by_factors(num_factors, als_movie_factors, als_movie_ids, num_results=20,
                       query=None, device=0):
    """For each query movie (standard ids; all of ``als_movie_ids`` when None)
    the ``num_results`` other movies with the highest cosine similarity of
    their ALS factor rows (``als{k}_item_factors`` / ``als{k}_movie_ids``,
    the reference's objects, ``recommend.py:62-70``).  Returns
    ``{movie_id: [(cosine, movie_id), ...]}``, ordered by (cosine, movie id)
    descending.

    Runs on the serving path's kernels: the rows are normalised on the host
    (fp64), the candidate table holds the normalised rows with zero medians and
    each query is a "user" row (normalised factors, zero bias), so the score
    kernel's fp64 expression ``s = 0; s += x_i * v_i ...`` IS the cosine, and
    the exact top-N select (self excluded) ranks it.  A zero factor row has
    cosine 0 with everything."""
    from .serving import MovieTable
    k = int(num_factors)
    V = numpy.ascontiguousarray(als_movie_factors, dtype=numpy.float64).reshape(-1, k)
    norm = numpy.sqrt(numpy.sum(V * V, axis=1))
    Vn = V / numpy.where(norm > 0, norm, 1.0)[:, None]
    zero_medians = {m: 0.0 for m in als_movie_ids}
    qids = list(als_movie_ids) if query is None else list(query)
    missing = [m for m in qids if m not in als_movie_ids]
    if missing:
        raise ValueError(f"query movies without ALS factors: {missing[:5]}")
    X = numpy.zeros((len(qids), k + 1))
    for t, m in enumerate(qids):
        X[t, :k] = Vn[als_movie_ids[m]]
    out = {}
    with MovieTable(k, Vn, als_movie_ids, zero_medians, device) as table:
        step = 4096
        for s in range(0, len(qids), step):
            chunk = qids[s:s + step]
            lists = table.top_n(X[s:s + step], [[m] for m in chunk], num_results)
            for m, lst in zip(chunk, lists):
                out[m] = lst
    return out
