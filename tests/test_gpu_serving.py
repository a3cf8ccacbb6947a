"""GPU parity of the factor consumers (fold-in, scoring, top-N, evaluation)
against the reference fixtures (tests/golden/serving_k*.npz, made with the
reference's models.py / my_util.py) and the exact oracle order.

Tolerances: scores, rankings, pair counts and agreements are compared
bit-for-bit (same fp64 expression in the same order).  Fold-in solves the
normal equations (Cholesky, fp64) where the reference calls lstsq (SVD):
<= 1e-8 relative on well-conditioned lists; rank-deficient lists go through
the GPU Jacobi SVD and match lstsq's minimum-norm solution to <= 1e-8."""
import numpy as np
import pytest

from conftest import rel_err
from oracle import serving_oracle as O
from serving_cases import KS, exact_scores, exact_top_n, fixture, synthetic_table

pytestmark = pytest.mark.gpu


def table(d, k):
    from movie_recommender_amd.serving import MovieTable
    return MovieTable(k, d["V"], d["als_ids"], d["med"])


@pytest.mark.parametrize("k", KS)
def test_fold_in_matches_lstsq(gpu, k):
    d = fixture(k)
    with table(d, k) as t:
        valid, X, method = t.fold_in(d["lists"])
    assert np.array_equal(valid, d["valid"].astype(bool))
    for u in np.flatnonzero(valid):
        assert rel_err(X[u], d["X"][u]) <= 1e-8, (u, method[u])
    assert method[1] == 2            # the rank-deficient list took the SVD path
    assert set(method[valid]) <= {1, 2}


@pytest.mark.parametrize("k", KS)
def test_scores_bit_exact(gpu, k):
    d = fixture(k)
    with table(d, k) as t:
        vu = np.flatnonzero(d["valid"])
        S = t.scores(d["X"][vu])
        cand = [int(m) for m in t.cand_mid]
        for i, u in enumerate(vu):
            ref = np.array([O.predict(d["X"][u], m, d["med"], d["V"], d["als_ids"]) for m in cand])
            assert np.array_equal(S[i], ref)


@pytest.mark.parametrize("k", KS)
def test_top_n_identical_to_reference(gpu, k):
    d = fixture(k)
    vu = np.flatnonzero(d["valid"])
    with table(d, k) as t:
        got = t.top_n(d["X"][vu], [dict(d["lists"][u]) for u in vu], int(d["num_results"]))
    for i, u in enumerate(vu):
        assert got[i] == d["recs"][u]


def test_top_n_limits_and_no_exclusions(gpu):
    d = fixture(3)
    vu = np.flatnonzero(d["valid"])
    with table(d, 3) as t:
        nc = t.num_candidates
        cand = np.array(t.cand_mid)
        S = exact_scores(d["X"][vu], d["V"].reshape(-1, 3)[t.cand_als], t.cand_med)
        for n in (1, 7, 1024):
            got = t.top_n(d["X"][vu], None, n)
            for i in range(len(vu)):
                assert got[i] == exact_top_n(S[i], cand, set(), n)
                assert len(got[i]) == min(n, nc)
        # every candidate excluded -> empty list
        got = t.top_n(d["X"][vu[:1]], [set(int(m) for m in cand)], 10)
        assert got == [[]]


def test_top_n_large_synthetic(gpu):
    """20k candidates, 300 users with 0-500 rated movies, ties in the table."""
    from movie_recommender_amd.serving import MovieTable
    k = 32
    V, als_ids, med = synthetic_table(k, 20000, 500, seed=5, ties=200)
    rs = np.random.RandomState(1)
    X = rs.normal(0, 0.5, (300, k + 1))
    X[7] = 0.0                                  # every score = the median: massive ties
    keys = np.array(list(als_ids))
    rated = [set(int(m) for m in rs.choice(keys, rs.randint(0, 500), replace=False))
             for _ in range(300)]
    with MovieTable(k, V, als_ids, med) as t:
        got = t.top_n(X, rated, 400)
        S = exact_scores(X, V.reshape(-1, k)[t.cand_als], t.cand_med)
        cand = np.array(t.cand_mid)
        for u in range(300):
            assert got[u] == exact_top_n(S[u], cand, rated[u], 400), u
        # the same exclusions as a CSR pair of arrays (no per-user Python
        # loop), with non-candidate ids mixed in: identical arrays
        lists = [np.array(sorted(r) + [10 ** 7 + u], np.int64) for u, r in enumerate(rated)]
        off = np.concatenate([[0], np.cumsum([len(l) for l in lists])]).astype(np.int64)
        m1, s1, c1 = t.top_n_arrays(X, rated, 400)
        m2, s2, c2 = t.top_n_arrays(X, (off, np.concatenate(lists)), 400)
        assert np.array_equal(c1, c2) and np.array_equal(m1, m2)
        assert np.array_equal(s1.view(np.int64), s2.view(np.int64))


@pytest.mark.parametrize("k", KS)
def test_evaluation_exact(gpu, k):
    d = fixture(k)
    with table(d, k) as t:
        res = t.evaluate(d["U"], d["t_als"], d["t_lists"])
    a = res["agreement"]
    assert np.array_equal(np.isnan(a), np.isnan(d["agreement"]))
    ok = ~np.isnan(a)
    assert np.array_equal(a[ok], d["agreement"][ok])
    assert np.array_equal(res["n_agree"][ok], d["n_agree"][ok])
    assert np.array_equal(res["n_disagree"][ok], d["n_disagree"][ok])
    # per-rating predictions equal the reference predict (None -> NaN)
    K = k + 1
    p = []
    for i, l in enumerate(d["t_lists"]):
        uf = d["U"][K * d["t_als"][i]: K * (d["t_als"][i] + 1)]
        for m, _ in l:
            v = O.predict(uf, m, d["med"], d["V"], d["als_ids"])
            p.append(np.nan if v is None else v)
    assert np.array_equal(res["pred"], np.array(p), equal_nan=True)


def test_als_eval_interface(gpu):
    from movie_recommender_amd.evaluation import als_eval
    d = fixture(11)
    user_ids = {int(u): int(r) for u, r in zip(d["t_uid"], d["t_als"])}
    tests = list(zip(d["t_uid"].tolist(), d["t_lists"]))
    got, stats = als_eval(tests, d["med"], d["U"], user_ids, d["V"], d["als_ids"], 11,
                          return_stats=True)
    exp = [(int(u), float(a)) for u, a in zip(d["t_uid"], d["agreement"]) if not np.isnan(a)]
    assert got == exp
    assert np.isfinite(stats["rmse"])


def test_compute_ranking_agreement_interface(gpu):
    from movie_recommender_amd.evaluation import compute_ranking_agreement, ranking_agreements
    actual = [(1, 5.0), (2, 3.0), (3, 4.0), (4, 3.0)]
    pred = [(1, 4.1), (2, 3.9), (3, 3.9), (4, 2.0)]
    assert compute_ranking_agreement(actual, pred) == O.ranking_agreement(actual, pred)[0]
    assert compute_ranking_agreement(actual[:1], pred[:1]) is None
    assert compute_ranking_agreement([(1, 3.0), (2, 3.0)], pred[:2]) is None
    rs = np.random.RandomState(3)
    pairs = []
    for n in (0, 1, 2, 5, 300, 2500):
        a = rs.choice(np.arange(1, 11) / 2.0, n)
        p = np.round(rs.normal(3, 1, n), 1)        # rounded: many tied predictions
        pairs.append((a, p))
    agr, ag, dis = ranking_agreements(pairs)
    for i, (a, p) in enumerate(pairs):
        ea, ed = O.ranking_agreement_counts(a, p)
        assert (ag[i], dis[i]) == (ea, ed)
        if len(a) > 1 and ea + ed:
            assert agr[i] == ea / (ea + ed)


def test_als_model_interface(gpu):
    """models.ALS_Model drop-in: validity, predict, params, recommendations."""
    from movie_recommender_amd.serving import ALS_Model, get_recommendations
    d = fixture(11)
    for u in (0, 2, 3, 5, 6):
        l = d["lists"][u]
        m = ALS_Model(11, l, d["med"], d["V"], d["als_ids"])
        assert m.is_valid() == bool(d["valid"][u])
        if not m.is_valid():
            assert m.predict(int(d["med_keys"][0])) is None
            continue
        assert rel_err(m.user_factors, d["X"][u]) <= 1e-8
        params = m.get_param_list()
        assert params[-1][0] == "user bias" and params[0][0] == "factor 0" and len(params) == 12
        for mid in list(d["med"])[:50] + [999999999]:
            ref = O.predict(m.user_factors, mid, d["med"], d["V"], d["als_ids"])
            assert m.predict(mid) == ref
        rot0, full = get_recommendations(m, dict(l), 400)
        exp = [x for _, x in O.recommend(m.user_factors, dict(l), d["med"], d["V"],
                                         d["als_ids"], 400)]
        assert full == exp and rot0 == exp[0::4]


@pytest.mark.parametrize("k", [1, 15, 16, 63, 64, 100, 128])
def test_fold_in_sizes(gpu, k):
    """All fold-in LDS / register paths (one to four entry passes)."""
    from movie_recommender_amd.serving import MovieTable
    V, als_ids, med = synthetic_table(k, 3 * k + 40, 5, seed=k, ties=0)
    rs = np.random.RandomState(k)
    keys = list(als_ids)
    lists = [[(int(m), float(r)) for m, r in zip(rs.choice(keys, n, replace=False),
                                                  rs.choice(np.arange(1, 11) / 2.0, n))]
             for n in (k + 1, 2 * k + 3, 3 * k + 40)]
    with MovieTable(k, V, als_ids, med) as t:
        valid, X, method = t.fold_in(lists)
    for u, l in enumerate(lists):
        ok, x = O.fold_in(k, l, V, als_ids)
        assert ok and valid[u]
        assert rel_err(X[u], x) <= 1e-7, (u, method[u], np.linalg.cond(
            np.c_[V.reshape(-1, k)[[als_ids[m] for m, _ in l]], np.ones(len(l))]))


def test_top_n_all_scores_equal(gpu):
    """Every score identical (zero user, one median): the order is by movie id
    descending, through the radix-select path (no score range)."""
    from movie_recommender_amd.serving import MovieTable
    k = 8
    V, als_ids, med = synthetic_table(k, 5000, 0, seed=9, ties=0)
    med = {m: 3.0 for m in med}
    with MovieTable(k, V, als_ids, med) as t:
        X = np.zeros((3, k + 1))
        got = t.top_n(X, [set(), {max(als_ids)}, set(list(als_ids)[:4990])], 400)
    ids = sorted(als_ids, reverse=True)
    assert got[0] == [(3.0, m) for m in ids[:400]]
    assert got[1] == [(3.0, m) for m in ids[1:401]]
    rest = sorted(set(als_ids) - set(list(als_ids)[:4990]), reverse=True)
    assert got[2] == [(3.0, m) for m in rest]
