"""Golden fixtures for the ALS training-set preparation,
produced by the REFERENCE's own ``movie_lens_data_proc`` functions.

Run in the build container (needs /root/reference; writes nothing there):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_prep.py

``movie_lens_data_proc`` is imported with ``build_similar_movies_db`` (an
import of that module used only by the similar-movies functions, whose own
imports pull in the training driver and the cluster code) replaced by an
empty module.  The process pool of ``als_data_set_shrink_mp``
(``movie_lens_data.py:547-680``) is driven by hand: every per-process function
(``_drop_users``, ``_count_movies``, ``_drop_movies``, ``_collect_ids``,
``_convert_training_data_to_numpy``, ``_extract_movie_ratings``,
``_compute_medians``) is the reference's, run once per simulated process on
its own ``_process_data``; the merges follow ``_proc``'s helpers (own process
last; sets through a pickle round trip like a pipe).

Fixture prep_p<P>.npz (P = 1, 3 simulated processes), factors (3, 5, 11):
inputs (train lists as CSR in traversal order, test lists aligned, the
per-process list counts) and per factor the id tables (keys in dict order),
the training arrays and the kept test lists; plus the medians.
"""
import copy
import os
import pickle
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True
sys.modules["build_similar_movies_db"] = types.ModuleType("build_similar_movies_db")
sys.path.insert(0, "/root/reference/python/full_data")
import movie_lens_data_proc as P  # noqa: E402  (reference)
sys.path.pop(0)

FACTORS = (3, 5, 11)


def user_ratings(seed, n_users=260, n_movies=900):
    """MovieLens-like lists: standard ids with gaps, skewed popularity and
    activity, half-star ratings."""
    rs = np.random.RandomState(seed)
    movie_ids = np.sort(rs.choice(np.arange(1, 200_000), n_movies, replace=False))
    pop = 1.0 / (1 + rs.permutation(n_movies)) ** 0.8
    pop /= pop.sum()
    users = np.sort(rs.choice(np.arange(1, 300_000), n_users, replace=False))
    out_train, out_test = [], []
    for u in users:
        n = int(min(n_movies - 1, max(2, rs.lognormal(3.0, 0.9))))
        ms = rs.choice(movie_ids, n, replace=False, p=pop)
        rt = rs.choice(np.arange(1, 11) / 2.0, n)
        lst = [(int(m), float(r)) for m, r in zip(ms, rt)]
        cut = max(1, int(0.8 * n))
        out_train.append((int(u), lst[:cut]))
        out_test.append((int(u), lst[cut:]))
    return out_train, out_test


def run(procs, fn, req):
    for d in procs:
        P._process_data = d
        getattr(P, fn)(req)


def merge_set(procs, name):
    s = procs[-1][name].copy()                      # update_var_into_set
    for d in procs[:-1]:
        s.update(pickle.loads(pickle.dumps(d[name])))
    return s


def build(n_procs, seed):
    train, test = user_ratings(seed)
    counts = P.my_util.split(0, len(train), n_procs)
    counts = [c for _, c in counts]
    # medians on the whole training set (single process)
    d0 = {"user_ratings_train": copy.deepcopy(train)}
    P._process_data = d0
    P._extract_movie_ratings({})
    P._compute_medians({})
    medians = dict(d0["movie_medians"])

    procs, o = [], 0
    for c in counts:
        procs.append({"user_ratings_train": copy.deepcopy(train[o:o + c]),
                      "user_ratings_test": copy.deepcopy(test[o:o + c])})
        o += c
    out = {}
    for k in FACTORS:
        rounds = 0
        has_changed = True
        while has_changed:
            rounds += 1
            run(procs, "_drop_users", {"min_ratings": k + 1})
            has_changed = any(d["has_changed"] for d in procs)
            run(procs, "_count_movies", {})
            mc = dict(procs[-1]["movie_counts"])          # add_merge_var_into_dict
            for d in procs[:-1]:
                for key, v in d["movie_counts"].items():
                    mc[key] = mc.get(key, 0) + v
            uncommon = {m for m in mc if mc[m] < k}
            if uncommon:
                has_changed = True
                run(procs, "_drop_movies", {"movies_to_drop": uncommon})
        run(procs, "_collect_ids", {})
        movie_ids = merge_set(procs, "movie_ids")
        user_ids = merge_set(procs, "user_ids")
        als_movie_ids = {m: i for i, m in enumerate(movie_ids)}
        als_user_ids = {u: i for i, u in enumerate(user_ids)}
        for d in procs:
            d.update(als_movie_ids=als_movie_ids, als_user_ids=als_user_ids, movie_medians=medians)
        run(procs, "_convert_training_data_to_numpy", {})
        cat = lambda name: np.concatenate([d[name] for d in procs])   # pipes, then own
        test_k = [x for d in procs for x in d["user_ratings_test"]]
        t_off = np.zeros(len(test_k) + 1, np.int64)
        t_off[1:] = np.cumsum([len(l) for _, l in test_k])
        out.update({
            f"k{k}_rounds": rounds,
            f"k{k}_user_keys": np.array(list(als_user_ids), np.int64),
            f"k{k}_movie_keys": np.array(list(als_movie_ids), np.int64),
            f"k{k}_u": cat("user_ids_train_numpy"), f"k{k}_m": cat("movie_ids_train_numpy"),
            f"k{k}_r": cat("ratings_train_numpy"),
            f"k{k}_test_uid": np.array([u for u, _ in test_k], np.int64), f"k{k}_test_off": t_off,
            f"k{k}_test_mid": np.array([m for _, l in test_k for m, _ in l], np.int64),
            f"k{k}_test_r": np.array([r for _, l in test_k for _, r in l], np.float64)})
    off = np.zeros(len(train) + 1, np.int64)
    off[1:] = np.cumsum([len(l) for _, l in train])
    toff = np.zeros(len(test) + 1, np.int64)
    toff[1:] = np.cumsum([len(l) for _, l in test])
    out.update(
        factors=np.array(FACTORS), n_procs=n_procs, proc_counts=np.array(counts, np.int64),
        train_uid=np.array([u for u, _ in train], np.int64), train_off=off,
        train_mid=np.array([m for _, l in train for m, _ in l], np.int64),
        train_r=np.array([r for _, l in train for _, r in l], np.float64),
        test_off=toff, test_mid=np.array([m for _, l in test for m, _ in l], np.int64),
        test_r=np.array([r for _, l in test for _, r in l], np.float64),
        med_keys=np.array(list(medians), np.int64),
        med_vals=np.array(list(medians.values()), np.float64),
        numpy=np.__version__, python=sys.version.split()[0], seed=seed)
    return out


def main():
    for n_procs, seed in ((1, 5), (3, 6)):
        d = build(n_procs, seed)
        path = os.path.join(HERE, f"prep_p{n_procs}.npz")
        np.savez_compressed(path, **d)
        print(path, os.path.getsize(path), "bytes;",
              {k: (len(d[f"k{k}_user_keys"]), len(d[f"k{k}_movie_keys"]), len(d[f"k{k}_r"]),
                   int(d[f"k{k}_rounds"])) for k in FACTORS})


if __name__ == "__main__":
    main()
