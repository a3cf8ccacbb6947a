"""CPU: the streamed C5 generator (BASELINE.json configs[4]) partitions the
same rating set however it is cut, so every rank of a sharded run sees
consistent user and item views without materialising the whole set."""
import numpy as np

from movie_recommender_amd import synth


def test_c5_views_partition_the_rating_set():
    g = synth.C5Generator(scale=0.0005, block=1024)
    u, i, r = g.all_ratings()
    assert len(u) == g.n and u.dtype == np.int32 and i.dtype == np.int32
    assert np.array_equal(np.bincount(u, minlength=g.num_users), g.deg)
    assert set(np.unique(r * 2 + 6).astype(int)) <= set(range(1, 11))
    key = np.sort(u.astype(np.int64) * g.num_items + i)
    ub = [0, 1000, 3100, g.num_users]
    ib = [0, 7, 123, g.num_items]
    for a in range(3):
        uv = g.user_view(ub[a], ub[a + 1])
        assert np.all((uv[0] >= ub[a]) & (uv[0] < ub[a + 1]))
        assert len(uv[0]) == np.sum((u >= ub[a]) & (u < ub[a + 1]))
        iv = g.item_view(ib[a], ib[a + 1])
        sel = (i >= ib[a]) & (i < ib[a + 1])
        assert np.array_equal(np.sort(iv[0].astype(np.int64) * g.num_items + iv[1]),
                              np.sort(key[np.isin(key % g.num_items,
                                                  np.arange(ib[a], ib[a + 1]))]))
        assert np.isclose(iv[2].sum(), r[sel].sum())
    # regeneration is deterministic
    b1, b2 = g.gen_block(2), g.gen_block(2)
    assert all(np.array_equal(x, y) for x, y in zip(b1, b2))
