"""Golden fixtures for the similar-movies search, made
with the REFERENCE's own ``SimilarMovieFinder`` class.

Run in the build container (needs /root/reference; writes nothing there):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_similar.py

``build_similar_movies_db`` is imported with its driver-side imports
(``cluster``, ``movie_lens_data``, ``movie_lens_data_proc``: the cluster client,
the training driver that loads the native library, the process pool) replaced
by empty modules; ``SimilarMovieFinder`` itself needs only math and NumPy.

similar_main.npz: 1,400 movies / 2,500 users, half-star ratings with a
popular core (queries whose candidate lists exceed num_results * 20, so the
"most common reviewers" cut runs), duplicated movies (bit-equal scores: the
stable-sort tie rules), movies without genres.  Expected: find_similar_movie
for 60 query indices at num_results 20, 5 and 40.
similar_small.npz: 250 movies, the whole {movie_id: [ids]} database.
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True
for name in ("cluster", "movie_lens_data", "movie_lens_data_proc"):
    sys.modules[name] = types.ModuleType(name)
sys.path.insert(0, "/root/reference/python/full_data")
import build_similar_movies_db as ref  # noqa: E402  (reference)
sys.path.pop(0)


def dataset(seed, n_movies, n_users, n_dup, core):
    rs = np.random.RandomState(seed)
    mids = rs.choice(np.arange(1, 150_000), n_movies, replace=False)
    pop = 1.0 / (1 + np.arange(n_movies)) ** 0.7
    pop /= pop.sum()
    ratings = [dict() for _ in range(n_movies)]
    taste = rs.normal(0, 1, (n_users, 3))
    prof = rs.normal(0, 1, (n_movies, 3))
    for u in range(n_users):
        n = int(min(n_movies // 2, max(3, rs.lognormal(3.2, 0.8))))
        ms = set(rs.choice(n_movies, n, replace=False, p=pop).tolist())
        ms |= set(range(core)) if rs.random_sample() < 0.5 else set()
        for m in ms:
            x = 3 + taste[u] @ prof[m] + rs.normal(0, 0.7)
            ratings[m][int(1000 + 7 * u)] = float(np.clip(np.round(2 * x) / 2, 0.5, 5.0))
    for d in range(n_dup):                       # bit-identical twins
        a, b = core + 2 * d, core + 2 * d + 1
        ratings[b] = dict(ratings[a])
    genres = {}
    for m in range(n_movies):
        if rs.random_sample() < 0.05:
            continue                              # not in movie_genres
        k = rs.randint(1, 5)
        genres[int(mids[m])] = set(rs.choice([0, 1, 2, 3, 5, 8, 13, 21], k, replace=False)
                                   .tolist()) if rs.random_sample() < 0.8 else {0}
    for d in range(n_dup):
        a, b = core + 2 * d, core + 2 * d + 1
        if int(mids[a]) in genres:
            genres[int(mids[b])] = set(genres[int(mids[a])])
    movie_ratings = [(int(mids[m]), ratings[m]) for m in range(n_movies)]
    return genres, movie_ratings


def to_arrays(genres, movie_ratings):
    off = np.zeros(len(movie_ratings) + 1, np.int64)
    off[1:] = np.cumsum([len(r) for _, r in movie_ratings])
    g_keys = np.array(list(genres), np.int64)
    g_off = np.zeros(len(g_keys) + 1, np.int64)
    g_off[1:] = np.cumsum([len(genres[k]) for k in g_keys])
    return dict(
        movie_ids=np.array([m for m, _ in movie_ratings], np.int64), off=off,
        users=np.array([u for _, r in movie_ratings for u in r], np.int64),
        ratings=np.array([x for _, r in movie_ratings for x in r.values()], np.float64),
        g_keys=g_keys, g_off=g_off,
        g_vals=np.array([g for k in g_keys for g in genres[k]], np.int64))


def main():
    genres, mr = dataset(21, 1400, 2500, 6, 30)
    finder = ref.SimilarMovieFinder(genres, mr, buff_limit=0.05, buff_point=100)
    rs = np.random.RandomState(3)
    queries = sorted(set(list(range(0, 42)) + rs.choice(len(mr), 30, replace=False).tolist()))[:60]
    out = to_arrays(genres, mr)
    out["queries"] = np.array(queries, np.int64)
    for nres in (20, 5, 40):
        ids, scores, cnt = [], [], []
        for q in queries:
            a, b = finder.find_similar_movie(q, num_results=nres)
            ids += list(a)
            scores += list(b)
            cnt.append(len(a))
        out[f"n{nres}_ids"] = np.array(ids, np.int64)
        out[f"n{nres}_scores"] = np.array(scores, np.float64)
        out[f"n{nres}_count"] = np.array(cnt, np.int64)
    path = os.path.join(HERE, "similar_main.npz")
    np.savez_compressed(path, buff_limit=0.05, buff_point=100, **out)
    print(path, os.path.getsize(path), "bytes; results per query (n20):",
          out["n20_count"].min(), "-", out["n20_count"].max())

    genres, mr = dataset(5, 250, 600, 3, 10)
    finder = ref.SimilarMovieFinder(genres, mr, buff_limit=0.08, buff_point=40)
    db = {}
    for i in range(len(mr)):
        a, _ = finder.find_similar_movie(i)
        if len(a) > 0:
            db[mr[i][0]] = list(a)
    out = to_arrays(genres, mr)
    out["db_keys"] = np.array(list(db), np.int64)
    d_off = np.zeros(len(db) + 1, np.int64)
    d_off[1:] = np.cumsum([len(v) for v in db.values()])
    out["db_off"] = d_off
    out["db_vals"] = np.array([x for v in db.values() for x in v], np.int64)
    path = os.path.join(HERE, "similar_small.npz")
    np.savez_compressed(path, buff_limit=0.08, buff_point=40, **out)
    print(path, os.path.getsize(path), "bytes;", len(db), "movies with similar movies")


if __name__ == "__main__":
    main()
