"""GPU parity of the similar-movies search (include/mr_similar.h via
movie_recommender_amd/similar.py) with the reference's SimilarMovieFinder:
ids, scores (bit-for-bit), tie order and the num_results*20 cut."""
import numpy as np
import pytest

from oracle import similar_oracle as O
from similar_cases import expected, fixture

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nres", [20, 5, 40])
def test_find_similar_identical(gpu, nres):
    from movie_recommender_amd.similar import SimilarMovieFinder
    d = fixture("main")
    with SimilarMovieFinder(d["genres"], d["movie_ratings"], float(d["buff_limit"]),
                            int(d["buff_point"])) as f:
        for q, e in zip(d["queries"].tolist(), expected(d, nres)):
            ids, scores = f.find_similar_movie(q, nres)
            assert (tuple(ids), tuple(scores)) == e, q


def test_database_identical(gpu):
    from movie_recommender_amd.similar import build_similar_movies
    d = fixture("small")
    db = build_similar_movies(d["genres"], d["movie_ratings"], int(d["buff_point"]),
                              float(d["buff_limit"]))
    o = d["db_off"]
    exp = {int(k): d["db_vals"][o[i]:o[i + 1]].tolist() for i, k in enumerate(d["db_keys"])}
    assert db == exp and list(db) == list(exp)


def test_batch_equals_single_and_oracle(gpu):
    """All 1,400 movies in one launch; spot-check against the oracle."""
    from movie_recommender_amd.similar import SimilarMovieFinder
    d = fixture("main")
    with SimilarMovieFinder(d["genres"], d["movie_ratings"], 0.05, 100) as f:
        oj, os_, oc = f.find_many(None, 20)
        for q in (0, 1, 2, 700, 1399):
            ids, sc = O.find_similar_movie(d["genres"], d["movie_ratings"], q, 0.05, 100, 20)
            got = tuple(int(x) for x in f._ids[oj[q, :oc[q]]])
            assert got == tuple(ids) and tuple(os_[q, :oc[q]].tolist()) == tuple(sc)


def test_tune(gpu):
    """tune() (reference :166-211) on the GPU finder ends with the second movie
    in the first one's top list, as the reference's loop requires."""
    from movie_recommender_amd.similar import SimilarMovieFinder
    d = fixture("main")
    mr = d["movie_ratings"]
    with SimilarMovieFinder(d["genres"], mr) as f:
        a, b = mr[0][0], mr[3][0]
        f.tune(a, b, 2, 20)
        ids, _ = f.find_similar_movie(f.find_movie_index(a), 40)
        assert f.buff_limit >= 2 or b in ids[:2]
        assert f.buff_point == O.scaled_dot_product(mr, 0, 3, 0.05, 100)[1]


def test_rejects_non_half_star_ratings(gpu):
    from movie_recommender_amd.similar import SimilarMovieFinder
    with pytest.raises(ValueError):
        SimilarMovieFinder({1: {0}}, [(1, {5: 3.3})])
