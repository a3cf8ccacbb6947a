"""ALS training-set preparation on the GPU, with the reference's interface.

Mirrors:

* ``movie_medians``        -- ``refresh_training_sets_mp``'s median step
  (``movie_lens_data.py:454-465``, ``movie_lens_data_proc.py:393-471``):
  ``{movie_id: numpy.median(ratings)}`` over the training set, ascending ids;
* ``als_data_set_shrink``  -- ``als_data_set_shrink_mp``
  (``movie_lens_data.py:547-680``): per factor k, drop users with fewer than
  k+1 and movies with fewer than k training ratings until nothing changes
  (in place: each factor continues from the previous one's survivors), give
  the survivors zero-based ids in the order the reference's merged Python
  sets iterate (reproduced exactly for a given process split), and build the
  training arrays (ids, rating - median) plus the aligned test lists;
* ``write_reference_files`` -- the ``als{k}_*.bin`` files the reference saves
  (``:616-659``) for ``als_train`` / the evaluation to read.

The device does the O(N) work (``include/mr_prep.h``); the host keeps only
what is inherently Python: the dict/set objects the reference produces.
There is no CPU fallback.
"""
import ctypes
import os
import pickle

import numpy as np

from . import _lib


def _ip(a):
    return a.ctypes.data_as(_lib.IP)


def _dp(a):
    return a.ctypes.data_as(_lib.DP)


def _llp(a):
    return a.ctypes.data_as(_lib.LLP)


def flatten(user_ratings):
    """``[(user_id, [(movie_id, rating)])]`` -> (user ids int32[N], movie ids
    int32[N], ratings f64[N], ratings per list int64[n_lists]) in traversal
    order."""
    lens = np.fromiter((len(l) for _, l in user_ratings), np.int64, len(user_ratings))
    n = int(lens.sum())
    uid = np.repeat(np.fromiter((u for u, _ in user_ratings), np.int64, len(user_ratings)),
                    lens).astype(np.int32)
    mid = np.fromiter((m for _, l in user_ratings for m, _ in l), np.int32, n)
    r = np.fromiter((x for _, l in user_ratings for _, x in l), np.float64, n)
    return uid, mid, r, lens


def split_counts(length, num_splits):
    """``my_util.split`` lengths (``my_util.py:17-50``): the chunk sizes
    ``split_list_and_send`` gives each process (the caller's own process holds
    the last chunk)."""
    if length >= num_splits:
        idx = [int(length * i / num_splits) for i in range(num_splits)]
        return [idx[i + 1] - idx[i] for i in range(num_splits - 1)] + [length - idx[-1]]
    return [1 if i < length else 0 for i in range(num_splits)]


class TrainingSet:
    """Flattened training ratings resident on one GPU."""

    def __init__(self, user_ids, movie_ids, ratings, device=0):
        self.user_ids = np.ascontiguousarray(user_ids, np.int32)
        self.movie_ids = np.ascontiguousarray(movie_ids, np.int32)
        self.ratings = np.ascontiguousarray(ratings, np.float64)
        n = len(self.ratings)
        self._h = _lib.lib().mr_prep_create(int(device), n, _ip(self.user_ids),
                                           _ip(self.movie_ids), _dp(self.ratings))
        if not self._h:
            raise RuntimeError("mr_prep_create failed: " + _lib.last_error())
        ub = np.zeros(1, np.int32)
        mb = np.zeros(1, np.int32)
        _lib.check(_lib.lib().mr_prep_id_bounds(self._h, _ip(ub), _ip(mb)), "mr_prep_id_bounds")
        self.user_bound, self.movie_bound = int(ub[0]), int(mb[0])
        self.n_kept = None

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().mr_prep_destroy(self._h)
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
        return float(_lib.lib().mr_prep_last_ms(self._h))

    def medians(self):
        """f64[movie_bound]: numpy.median per movie id (NaN: no ratings)."""
        med = np.zeros(max(self.movie_bound, 1))
        _lib.check(_lib.lib().mr_prep_medians(self._h, _dp(med)), "mr_prep_medians")
        return med[:self.movie_bound]

    def shrink(self, k, restart=True):
        """Returns (keep bool[N], rounds, n_kept, n_users, n_movies)."""
        keep = np.zeros(max(len(self.ratings), 1), np.uint8)
        rounds = np.zeros(1, np.int32)
        nk = np.zeros(1, np.int64)
        nu = np.zeros(1, np.int32)
        nm = np.zeros(1, np.int32)
        _lib.check(_lib.lib().mr_prep_shrink(
            self._h, int(k), 1 if restart else 0,
            keep.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), _ip(rounds), _llp(nk),
            _ip(nu), _ip(nm)), "mr_prep_shrink")
        self.n_kept = int(nk[0])
        return keep[:len(self.ratings)].astype(bool), int(rounds[0]), int(nk[0]), int(nu[0]), \
            int(nm[0])

    def first_appearance(self, chunk_begin):
        """Per chunk of ratings: surviving user ids and movie ids in order of
        first appearance (the insertion order of ``_collect_ids``' sets)."""
        cb = np.ascontiguousarray(chunk_begin, np.int64)
        C = len(cb) - 1
        fu = np.zeros(max(C * self.user_bound, 1), np.int64)
        fm = np.zeros(max(C * self.movie_bound, 1), np.int64)
        _lib.check(_lib.lib().mr_prep_first_appearance(self._h, C, _llp(cb), _llp(fu), _llp(fm)),
                   "mr_prep_first_appearance")
        out = []
        inf = np.iinfo(np.int64).max
        for c in range(C):
            res = []
            for f, bound in ((fu, self.user_bound), (fm, self.movie_bound)):
                row = f[c * bound:(c + 1) * bound]
                ids = np.flatnonzero(row != inf)
                res.append(ids[np.argsort(row[ids], kind="stable")].tolist())
            out.append(tuple(res))
        return out

    def convert(self, user_map, movie_map, median):
        """Training arrays of the last shrink (ids through the dense maps,
        rating - median[movie])."""
        um = np.ascontiguousarray(user_map, np.int32)
        mm = np.ascontiguousarray(movie_map, np.int32)
        med = np.ascontiguousarray(median, np.float64)
        n = self.n_kept
        ou = np.zeros(max(n, 1), np.int32)
        om = np.zeros(max(n, 1), np.int32)
        orr = np.zeros(max(n, 1))
        _lib.check(_lib.lib().mr_prep_convert(self._h, _ip(um), _ip(mm), _dp(med), _ip(ou),
                                              _ip(om), _dp(orr)), "mr_prep_convert")
        return ou[:n], om[:n], orr[:n]


def movie_medians(user_ratings_train, device=0, training_set=None):
    """``{movie_id: median}`` of the training ratings, ascending movie ids
    (the dict ``refresh_training_sets_mp`` returns and saves)."""
    ts = training_set or TrainingSet(*flatten(user_ratings_train)[:3], device=device)
    try:
        med = ts.medians()
    finally:
        if training_set is None:
            ts.close()
    ids = np.flatnonzero(~np.isnan(med))
    return dict(zip(ids.tolist(), med[ids].tolist()))


def _reference_set_order(chunk_lists):
    """Iteration order of the set ``update_var_into_set`` returns
    (``movie_lens_data_proc.py:246-261``): the caller's own set (last chunk)
    copied, then updated with every other process's set as received through
    its pipe (a pickle round trip), in pipe order.  Each chunk's set was built
    by ``set.add`` in first-appearance order (``:589-608``)."""
    sets = [set(ids) for ids in chunk_lists]
    merged = sets[-1].copy()
    for s in sets[:-1]:
        merged.update(pickle.loads(pickle.dumps(s)))
    return list(merged)


class ShrinkResult:
    """One factor's output of ``als_data_set_shrink``."""

    def __init__(self, k, als_user_ids, als_movie_ids, train, test, rounds, kernel_ms):
        self.k = k
        self.als_user_ids = als_user_ids      # {standard user id: zero-based id}
        self.als_movie_ids = als_movie_ids    # {standard movie id: zero-based id}
        self.user_ids_train, self.movie_ids_train, self.ratings_train = train
        self.user_ratings_test = test         # aligned test lists of the kept users, or None
        self.rounds = rounds
        self.kernel_ms = kernel_ms


def als_data_set_shrink(user_ratings_train, user_ratings_test, movie_medians_train,
                        factors_list, cpu_count=1, process_list_counts=None, device=0,
                        out_dir=None):
    """``als_data_set_shrink_mp`` for ``factors_list`` (in order, shrinking in
    place from factor to factor).  ``user_ratings_test`` is aligned with
    ``user_ratings_train`` by index (or None).  The zero-based ids follow the
    reference's set iteration order for ``cpu_count`` processes; pass
    ``process_list_counts`` (user lists held by each process, caller's own
    last) when the lists were split unevenly, as ``refresh_training_sets_mp``
    leaves them.  Returns ``{k: ShrinkResult}``; with ``out_dir`` also writes
    the reference's ``als{k}_*.bin`` files there."""
    uid, mid, r, lens = flatten(user_ratings_train)
    counts = process_list_counts or split_counts(len(user_ratings_train), cpu_count)
    if sum(counts) != len(user_ratings_train):
        raise ValueError("process_list_counts must add up to len(user_ratings_train)")
    list_off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=list_off[1:])
    chunk_lists = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    chunk_begin = list_off[chunk_lists]
    med_dense = np.full(0, np.nan)
    results = {}
    user_alive = np.ones(len(user_ratings_train), bool)
    with TrainingSet(uid, mid, r, device) as ts:
        med_dense = np.full(ts.movie_bound, np.nan)
        for m, v in movie_medians_train.items():
            if 0 <= m < ts.movie_bound:
                med_dense[m] = v
        first = True
        for k in factors_list:
            keep, rounds, n_kept, n_users, n_movies = ts.shrink(k, restart=first)
            ms = ts.last_ms()
            first = False
            per_chunk = ts.first_appearance(chunk_begin)
            ms += ts.last_ms()
            movie_order = _reference_set_order([pc[1] for pc in per_chunk])
            user_order = _reference_set_order([pc[0] for pc in per_chunk])
            als_movie_ids = {m: i for i, m in enumerate(movie_order)}
            als_user_ids = {u: i for i, u in enumerate(user_order)}
            umap = np.full(ts.user_bound, -1, np.int32)
            mmap = np.full(ts.movie_bound, -1, np.int32)
            umap[np.asarray(user_order, np.int64)] = np.arange(len(user_order), dtype=np.int32)
            mmap[np.asarray(movie_order, np.int64)] = np.arange(len(movie_order), dtype=np.int32)
            train = ts.convert(umap, mmap, med_dense)
            ms += ts.last_ms()
            # lists that still hold ratings are the kept users (_drop_users)
            cs = np.concatenate([[0], np.cumsum(keep, dtype=np.int64)])
            user_alive &= (cs[list_off[1:]] - cs[list_off[:-1]]) > 0
            test = None
            if user_ratings_test is not None:
                test = [user_ratings_test[i] for i in np.flatnonzero(user_alive)]
            res = ShrinkResult(k, als_user_ids, als_movie_ids, train, test, rounds, ms)
            results[k] = res
            if out_dir is not None:
                write_reference_files(out_dir, res)
    return results


def write_reference_files(out_dir, res):
    """The files ``als_data_set_shrink_mp`` saves (``movie_lens_data.py:616-659``)."""
    os.makedirs(out_dir, exist_ok=True)
    k = res.k

    def dump(name, obj):
        with open(os.path.join(out_dir, f"als{k}_{name}.bin"), "wb") as f:
            pickle.dump(obj, f)

    dump("user_ids", res.als_user_ids)
    dump("movie_ids", res.als_movie_ids)
    dump("user_ratings_train", [res.user_ids_train, res.movie_ids_train, res.ratings_train])
    if res.user_ratings_test is not None:
        dump("user_ratings_test", res.user_ratings_test)
        dump("user_ratings_test_length", len(res.user_ratings_test))
