"""Golden fixtures for the factor consumers, generated
from the REFERENCE's own Python code.

Run in the build container (needs /root/reference; writes nothing there):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_serving.py

Imported from the reference (plain NumPy/SciPy modules, no data files read):
  * ``python/app_local/models.py``  -- ``ALS_Model``: fold-in (lstsq on
    ``[V, 1]`` with raw ratings) and ``predict``;
  * ``python/full_data/my_util.py`` -- ``compute_ranking_agreement``.
``recommend.py`` / ``worker_process.py`` unpickle data files at import, so
their control flow (sort, exclusion, rotation; per-user test loop) is taken
from ``oracle/serving_oracle.py`` while every score and agreement value comes
from the imported reference functions.

Fixtures  serving_k<k>.npz  (k = 3, 11, 64)
  movie table   V (f64[n_als*k]), als_keys (standard id of als id j),
                med_keys / med_vals (movie_medians in insertion order)
  fold-in       users as CSR (u_off, u_mid, u_r): valid, X[B, k+1]
  top-N         per valid user, the reference list [(score, movie_id)] of
                length num_results (rec_off, rec_mid, rec_score)
  evaluation    test users (t_uid, t_off, t_mid, t_r), factor table
                U (f64[nU*(k+1)]), als user ids t_als; expected agreement per
                test user (nan = None), and pair counts agree / disagree
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference/python"
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "app_local"))
import models as ref_models  # noqa: E402  (reference: app_local/models.py)
sys.path.pop(0)
sys.path.insert(0, os.path.join(REF, "full_data"))
import my_util as ref_util  # noqa: E402  (reference: full_data/my_util.py)
sys.path.pop(0)

from oracle import serving_oracle as O  # noqa: E402

HALF = np.arange(1, 11) / 2.0


def movie_table(rs, k, n_als, n_extra, n_ties):
    """Standard ids, factors and medians.  A few movies are exact copies of
    another movie's factors and median, so their scores tie bit-for-bit and
    the (score, movie_id) tuple order decides; some movies have factors but
    no median, some a median but no factors."""
    ids = rs.choice(np.arange(1, 40 * (n_als + n_extra)), n_als + n_extra, replace=False)
    als_keys = ids[:n_als].astype(np.int64)
    V = rs.normal(0, 0.6, (n_als, k))
    med = rs.choice(HALF, n_als)
    ties = []
    for _ in range(n_ties):
        a, b = rs.choice(n_als, 2, replace=False)
        V[b] = V[a]
        med[b] = med[a]
        ties.append((a, b))
    has_med = rs.random_sample(n_als) < 0.92
    has_med[[t for p in ties for t in p]] = True       # tied movies are scored
    med_keys = list(als_keys[has_med]) + list(ids[n_als:])
    med_vals = list(med[has_med]) + list(rs.choice(HALF, n_extra))
    order = rs.permutation(len(med_keys))           # dict insertion order
    med_keys = np.asarray(med_keys, np.int64)[order]
    med_vals = np.asarray(med_vals, np.float64)[order]
    return V.reshape(-1), als_keys, med_keys, med_vals, [(als_keys[a], als_keys[b]) for a, b in ties]


def user_lists(rs, k, als_keys, med_keys, n_users, ties):
    """Rating lists covering the fold-in branches: too few ratings, enough
    ratings but too few with factors, exactly k+1 (once with two movies of
    identical factors: a rank-deficient [V, 1], lstsq's minimum-norm
    solution), and larger lists."""
    pool_f = als_keys
    pool_nf = np.setdiff1d(med_keys, als_keys)
    lists = []
    sizes = [k, k + 1, k + 1, k + 3, 2 * k + 5, 60, 200, 900]
    for u in range(n_users):
        n = sizes[u % len(sizes)] if u < len(sizes) else int(rs.randint(k + 1, 400))
        if u == 2 and len(pool_nf) >= 2:       # k+1 ratings, 2 without factors
            m = list(rs.choice(pool_f, n - 2, replace=False)) + list(rs.choice(pool_nf, 2, replace=False))
        elif u == 1:                           # k+1 ratings, one tied pair: rank k
            a, b = ties[0]
            rest = [x for x in rs.choice(pool_f, n + 2, replace=False) if x not in (a, b)]
            m = [a, b] + rest[:n - 2]
        else:
            m = list(rs.choice(pool_f, min(n, len(pool_f)), replace=False))
        r = rs.choice(HALF, len(m))
        lists.append([(int(a), float(b)) for a, b in zip(m, r)])
    return lists


def ref_model(k, ratings, med, V, als_ids):
    return ref_models.ALS_Model(k, ratings, med, V, als_ids)


def build(k, n_als, n_extra, n_users, n_test_users, num_results, seed):
    rs = np.random.RandomState(seed)
    V, als_keys, med_keys, med_vals, ties = movie_table(rs, k, n_als, n_extra, n_ties=max(3, n_als // 200))
    als_ids = {int(m): j for j, m in enumerate(als_keys)}
    med = {int(m): float(v) for m, v in zip(med_keys, med_vals)}
    lists = user_lists(rs, k, als_keys, med_keys, n_users, ties)

    u_off = np.zeros(len(lists) + 1, np.int64)
    u_off[1:] = np.cumsum([len(l) for l in lists])
    u_mid = np.array([m for l in lists for m, _ in l], np.int64)
    u_r = np.array([r for l in lists for _, r in l], np.float64)

    valid = np.zeros(len(lists), np.int8)
    X = np.zeros((len(lists), k + 1))
    rec_off = [0]
    rec_mid, rec_score = [], []
    for u, l in enumerate(lists):
        model = ref_model(k, l, med, V, als_ids)
        ok = model.is_valid()
        if ok:
            valid[u] = 1
            X[u] = model.user_factors
            # every score from the reference model; sort / exclusion restated
            preds = [(model.predict(m), m) for m in med if model.predict(m) is not None]
            preds.sort(reverse=True)
            rated = dict(l)
            top = [(s, m) for s, m in preds if m not in rated][:num_results]
            assert top == O.recommend(X[u], rated, med, V, als_ids, num_results)
            rec_mid += [m for _, m in top]
            rec_score += [s for s, _ in top]
        rec_off.append(len(rec_mid))

    # evaluation: a trained-looking user table and held-out lists
    nU = n_test_users + 7
    U = rs.normal(0, 0.5, nU * (k + 1))
    t_als = rs.permutation(nU)[:n_test_users]
    t_uid = rs.choice(np.arange(100000, 200000), n_test_users, replace=False)
    pool = np.concatenate([als_keys, np.setdiff1d(med_keys, als_keys)[:5]])
    t_lists = []
    for t in range(n_test_users):
        n = [1, 2, 3, 5][t] if t < 4 else int(rs.randint(2, 150))
        m = rs.choice(pool, n, replace=False)
        if t == 4 or t == 5:                       # a pair with bit-equal predictions
            m[0], m[1] = ties[t - 4]
        r = rs.choice(HALF, n) if t != 2 else np.full(n, 3.5)   # t = 2: all equal
        if t == 4:
            r[0], r[1] = 4.5, 2.0
        t_lists.append([(int(a), float(b)) for a, b in zip(m, r)])
    t_off = np.zeros(n_test_users + 1, np.int64)
    t_off[1:] = np.cumsum([len(l) for l in t_lists])
    t_mid = np.array([m for l in t_lists for m, _ in l], np.int64)
    t_r = np.array([r for l in t_lists for _, r in l], np.float64)
    agreement = np.full(n_test_users, np.nan)
    n_agree = np.zeros(n_test_users, np.int64)
    n_dis = np.zeros(n_test_users, np.int64)
    for t, l in enumerate(t_lists):
        K = k + 1
        uf = U[K * t_als[t]: K * (t_als[t] + 1)]
        m = object.__new__(ref_models.ALS_Model)          # reference predict on a given row
        m.user_factors, m._valid = uf, True
        m._movie_medians, m._als_movie_factors, m._als_movie_ids = med, V, als_ids
        pred, kept = [], []
        for mid, a in l:
            p = m.predict(mid)
            if p is not None:
                pred.append((mid, p))
                kept.append((mid, a))
        if len(pred) > 1:
            val = ref_util.compute_ranking_agreement(kept, pred)
            if val is not None:
                agreement[t] = val
                ag, dg = O.ranking_agreement_counts([a for _, a in kept], [p for _, p in pred])
                assert ag / (ag + dg) == val
                n_agree[t], n_dis[t] = ag, dg
        o = O.test_model(lambda mm: O.predict(uf, mm, med, V, als_ids), l)
        assert (o is None and np.isnan(agreement[t])) or o == agreement[t]

    return dict(k=k, num_results=num_results, V=V, als_keys=als_keys, med_keys=med_keys,
                med_vals=med_vals, u_off=u_off, u_mid=u_mid, u_r=u_r, valid=valid, X=X,
                rec_off=np.array(rec_off, np.int64), rec_mid=np.array(rec_mid, np.int64),
                rec_score=np.array(rec_score, np.float64), U=U, t_als=t_als.astype(np.int64),
                t_uid=t_uid.astype(np.int64), t_off=t_off, t_mid=t_mid, t_r=t_r,
                agreement=agreement, n_agree=n_agree, n_disagree=n_dis,
                numpy=np.__version__, seed=seed)


def main():
    for k, n_als, n_extra, n_users, n_test, nres, seed in [
            (3, 400, 40, 12, 40, 60, 3),
            (11, 3000, 300, 24, 120, 400, 11),
            (64, 1200, 100, 12, 40, 400, 64)]:
        d = build(k, n_als, n_extra, n_users, n_test, nres, seed)
        path = os.path.join(HERE, f"serving_k{k}.npz")
        np.savez_compressed(path, **d)
        print(path, os.path.getsize(path), "bytes; valid users", int(d["valid"].sum()),
              "of", len(d["valid"]), "; agreements", int(np.isfinite(d["agreement"]).sum()))


if __name__ == "__main__":
    main()
