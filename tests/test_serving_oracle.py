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


def _key64(s):
    """The order-preserving 64-bit key of serving.hip score_key (-0.0 -> +0.0)."""
    s = np.where(s == 0.0, 0.0, s)
    b = s.view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1 << 63))


def _key_score(key):
    neg = (key >> np.uint64(63)) == 0
    b = np.where(neg, ~key, key & np.uint64(0x7FFFFFFFFFFFFFFF))
    return b.view(np.float64)


def _truncated_select(s, mids, excl, N, bins=2048, cap=2048):
    """The select of rec_select_kernel's fast path on truncated keys: bins of
    the decoded top-32-bit keys over the exact [min, max], the boundary bin of
    the N-th largest, the candidates at or above it re-ranked by their exact
    (score, movie id).  Returns None where the kernel takes its radix path."""
    key = _key64(s)
    t = (key >> np.uint64(32)).astype(np.uint64)
    t[excl] = 0
    live = t != 0
    kmin, kmax = key[live].min(), key[live].max()
    smin, smax = _key_score(np.array([kmin]))[0], _key_score(np.array([kmax]))[0]
    if not smax > smin:
        return None
    scale = bins / (smax - smin)
    v = np.where(live, (_key_score(t << np.uint64(32)) - smin) * scale, 0.0)  # t = 0: excluded
    b = np.minimum(bins - 1, np.floor(np.maximum(v, 0.0)).astype(np.int64))
    hist = np.bincount(b[live], minlength=bins)
    cum, bb = 0, bins - 1
    while bb > 0 and cum + hist[bb] < N:
        cum += hist[bb]
        bb -= 1
    if cum + hist[bb] > cap:
        return None
    sel = np.flatnonzero(live & (b >= bb))
    order = sorted(((s[i], int(mids[i])) for i in sel), reverse=True)
    return [m for _, m in order[:N]]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_truncated_key_select_is_exact(seed):
    """The top-N kernel keeps only 32 bits of each score key and re-scores
    the candidates at or above the boundary bin exactly: the result equals a
    full sort by (score, movie id) descending -- including scores that differ
    only below the kept bits, exact ties and exclusions."""
    rng = np.random.default_rng(seed)
    n, N = 48859, 400
    base = rng.normal(3.5, 0.6, n)
    near = base[: n // 4] + rng.integers(-3, 4, n // 4) * np.finfo(np.float64).eps * 4
    s = np.concatenate([near, base[n // 4:]])
    s[rng.integers(0, n, 500)] = s[7]                          # exact ties
    mids = rng.permutation(n).astype(np.int64) + 1
    excl = np.zeros(n, bool)
    excl[rng.integers(0, n, 300)] = True
    got = _truncated_select(s, mids, excl, N)
    assert got is not None
    keep = ~excl
    ref = sorted(zip(s[keep].tolist(), mids[keep].tolist()), reverse=True)[:N]
    assert got == [m for _, m in ref]
