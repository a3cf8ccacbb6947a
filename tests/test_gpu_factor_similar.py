"""Movie-movie cosine similarity on the ALS factor layout (north star;
movie_recommender_amd.similar.similar_by_factors) against a NumPy restatement
that evaluates the same fp64 expression in the same order (normalised rows,
sequential sum over factors, no fused multiply-add) and ranks by (cosine,
movie id) descending with the query itself excluded.  Bit-exact scores and
lists.  No reference function exists for this pass (it is a north-star
feature the reference lacks), so parity is pinned to this restatement only."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def cosine_oracle(V, ids, query, n):
    k = V.shape[1]
    norm = np.sqrt(np.sum(V * V, axis=1))
    Vn = V / np.where(norm > 0, norm, 1.0)[:, None]
    inv = {a: m for m, a in ids.items()}
    out = {}
    for m in query:
        q = Vn[ids[m]]
        s = np.zeros(len(V))
        for c in range(k):                    # s += x_c * v_c, in factor order
            s = s + q[c] * Vn[:, c]
        s = s + 0.0                           # + bias
        s = s + 0.0                           # + median
        cand = [(s[a], inv[a]) for a in range(len(V)) if inv[a] != m]
        cand.sort(reverse=True)
        out[m] = cand[:n]
    return out


@pytest.mark.parametrize("k,n_movies,n", [(11, 700, 20), (64, 1500, 40)])
def test_similar_by_factors_exact(gpu, k, n_movies, n):
    from movie_recommender_amd.similar import similar_by_factors
    rng = np.random.default_rng(k)
    V = rng.normal(0, 1, (n_movies, k))
    V[7] = 0.0                                # a zero row: cosine 0 everywhere
    V[11] = V[12] * 2.5                       # parallel rows: cosine 1 (ties broken by id)
    mids = rng.permutation(np.arange(100, 100 + 3 * n_movies, 3))[:n_movies]
    ids = {int(m): a for a, m in enumerate(mids)}
    query = [int(mids[a]) for a in (0, 7, 11, 12, 13, n_movies - 1)]
    got = similar_by_factors(k, V.reshape(-1), ids, n, query=query)
    ref = cosine_oracle(V, ids, query, n)
    for m in query:
        assert [x[1] for x in got[m]] == [x[1] for x in ref[m]], m
        assert np.array_equal(np.array([x[0] for x in got[m]]), np.array([x[0] for x in ref[m]])), m
    assert got[int(mids[11])][0][1] == int(mids[12])   # the parallel row ranks first
