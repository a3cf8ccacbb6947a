"""CPU: the factor-consumer oracle (oracle/serving_oracle.py) reproduces the
golden fixtures made with the reference's own models.py / my_util.py, and the
vectorised exact scoring used by the larger GPU tests equals it bit for bit."""
import numpy as np
import pytest

from oracle import serving_oracle as O
from serving_cases import KS, exact_scores, exact_top_n, fixture


@pytest.mark.parametrize("k", KS)
def test_fold_in_matches_reference(k):
    d = fixture(k)
    for u, l in enumerate(d["lists"]):
        ok, x = O.fold_in(k, l, d["V"], d["als_ids"])
        assert ok == bool(d["valid"][u])
        if ok:
            assert np.array_equal(x, d["X"][u])      # same lstsq call


@pytest.mark.parametrize("k", KS)
def test_recommendations_match_reference(k):
    d = fixture(k)
    n = int(d["num_results"])
    vu = np.flatnonzero(d["valid"])
    for u in vu:
        got = O.recommend(d["X"][u], dict(d["lists"][u]), d["med"], d["V"], d["als_ids"], n)
        assert got == d["recs"][u]
    assert O.rotation(list(range(10)), 1) == [1, 5, 9]


@pytest.mark.parametrize("k", KS)
def test_agreement_matches_reference(k):
    d = fixture(k)
    K = k + 1
    got = O.als_eval(list(zip(d["t_uid"].tolist(), d["t_lists"])), d["med"], d["U"],
                     {int(u): int(r) for u, r in zip(d["t_uid"], d["t_als"])}, d["V"],
                     d["als_ids"], k)
    exp = [(int(u), float(a)) for u, a in zip(d["t_uid"], d["agreement"]) if not np.isnan(a)]
    assert got == exp
    assert K == k + 1


@pytest.mark.parametrize("k", KS)
def test_vectorised_exact_scores_equal_python_order(k):
    d = fixture(k)
    cand = [m for m in d["med"] if m in d["als_ids"]]
    Vc = d["V"].reshape(-1, k)[[d["als_ids"][m] for m in cand]]
    med = np.array([d["med"][m] for m in cand])
    vu = np.flatnonzero(d["valid"])
    S = exact_scores(d["X"][vu], Vc, med)
    for i, u in enumerate(vu):
        ref = [O.predict(d["X"][u], m, d["med"], d["V"], d["als_ids"]) for m in cand]
        assert np.array_equal(S[i], np.array(ref))
        top = exact_top_n(S[i], np.array(cand), set(m for m, _ in d["lists"][u]),
                          int(d["num_results"]))
        assert top == d["recs"][u]


def test_fixture_covers_edge_cases():
    d = fixture(11)
    # ties in the movie table are present in the candidate ranking
    s = d["rec_score"]
    assert len(s) != len(np.unique(s))
    # rank-deficient fold-in (user 1: two identical factor rows) is valid
    assert d["valid"][1] == 1
    # None agreements: single rating, all-equal ratings
    assert np.isnan(d["agreement"][0]) and np.isnan(d["agreement"][2])


def test_exclusion_csr_matches_container_path():
    """CPU: MovieTable's CSR exclusion input gives the candidate-index lists
    the per-user container path builds (non-candidates dropped, order kept)."""
    import numpy as np
    from movie_recommender_amd.serving import MovieTable
    t = MovieTable.__new__(MovieTable)
    rs = np.random.RandomState(3)
    t.cand_mid = np.sort(rs.choice(5000, 800, replace=False)).astype(np.int32)
    t.cand_index = {int(m): c for c, m in enumerate(t.cand_mid)}
    t._cand_lut = np.full(int(t.cand_mid.max()) + 1, -1, np.int32)
    t._cand_lut[t.cand_mid] = np.arange(len(t.cand_mid), dtype=np.int32)
    lists = [rs.choice(6000, rs.randint(0, 40), replace=False) for _ in range(50)] + [[]]
    off = np.concatenate([[0], np.cumsum([len(l) for l in lists])]).astype(np.int64)
    ids = np.concatenate([np.asarray(l, np.int64) for l in lists] + [np.array([-5], np.int64)])
    off[-1] += 1          # a negative id in the last (otherwise empty) list: dropped
    eo, ex = t._exclusions_csr(off, ids, len(lists))
    for u, l in enumerate(lists):
        want = [t.cand_index[int(m)] for m in l if int(m) in t.cand_index]
        assert ex[eo[u]:eo[u + 1]].tolist() == want
    import pytest
    with pytest.raises(ValueError):
        t._exclusions_csr(off[:-1], ids, len(lists))

