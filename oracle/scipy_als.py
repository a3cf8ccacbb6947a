"""CPU baseline only (test / measurement infrastructure, never the product):
a restatement of the reference's SciPy ALS path for MovieLens-100K,
``python/100k_data/ratings_als.py`` ``ALS_Model.solve_for_users`` (:347-396),
``solve_for_movies`` (:399-448) and the ``fit_to_data`` loop (:501-526) --
one global ``scipy.sparse.linalg.lsqr`` (iter_lim 100) on the design matrix
per half-step instead of the C++ library's CG.  The design matrices are
built vectorised here (the reference fills them with Python loops, so its
wall time is longer than what this measures); the arithmetic is the same:
users' rows [V_i, 1], movies' rows U_u[:k], and the reference's user-bias
read ``users[3::4]`` (:433) -- a stride that is only the bias column at
k = 3; it is kept as written, since this times the
reference's path, it does not judge its output."""
import time

import numpy as np
from scipy import sparse
from scipy.sparse import linalg


def solve_for_users(movies, user_ids, movie_ids, ratings, num_users, k):
    """ratings_als.py:347-396."""
    n = len(ratings)
    rows = np.repeat(np.arange(n), k + 1)
    cols = (user_ids[:, None] * (k + 1) + np.arange(k + 1)[None, :]).ravel()
    data = np.concatenate([movies.reshape(-1, k)[movie_ids], np.ones((n, 1))], axis=1).ravel()
    A = sparse.coo_matrix((data, (rows, cols)), shape=(n, num_users * (k + 1))).tocsr()
    return linalg.lsqr(A, ratings, iter_lim=100)[0]


def solve_for_movies(users, user_ids, movie_ids, ratings, num_movies, k):
    """ratings_als.py:399-448 (bias read with the reference's [3::4] stride)."""
    n = len(ratings)
    rows = np.repeat(np.arange(n), k)
    cols = (movie_ids[:, None] * k + np.arange(k)[None, :]).ravel()
    data = users.reshape(-1, k + 1)[user_ids, :k].ravel()
    A = sparse.coo_matrix((data, (rows, cols)), shape=(n, num_movies * k)).tocsr()
    bias = users[3::4]
    return linalg.lsqr(A, ratings - bias[user_ids], iter_lim=100)[0]


def time_iterations(user_ids, movie_ids, ratings, num_users, num_movies, k, iterations=3,
                    seed=0):
    """Seconds per ALS iteration (users then movies half-step), median of
    ``iterations`` (fit_to_data's loop body without its training-error pass)."""
    rng = np.random.default_rng(seed)
    movies = rng.uniform(-1, 1, num_movies * k)
    ts = []
    for _ in range(iterations):
        t0 = time.perf_counter()
        users = solve_for_users(movies, user_ids, movie_ids, ratings, num_users, k)
        movies = solve_for_movies(users, user_ids, movie_ids, ratings, num_movies, k)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts
