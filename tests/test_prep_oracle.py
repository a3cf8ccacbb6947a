"""CPU: the preparation oracle (oracle/prep_oracle.py) reproduces the fixtures
made with the reference's own movie_lens_data_proc functions."""
import copy

import numpy as np
import pytest

from oracle import prep_oracle as O
from prep_cases import expected_test, fixture


@pytest.mark.parametrize("p", [1, 3])
def test_medians(p):
    d = fixture(p)
    assert O.movie_medians(d["train"]) == d["medians"]
    assert list(O.movie_medians(d["train"])) == list(d["medians"])      # ascending ids


@pytest.mark.parametrize("p", [1, 3])
def test_shrink_ids_arrays_and_test_lists(p):
    d = fixture(p)
    counts = d["proc_counts"].tolist()
    assert counts == O.split_counts(len(d["train"]), p)
    tr = O.chunk(copy.deepcopy(d["train"]), counts)
    te = O.chunk(copy.deepcopy(d["test"]), counts)
    for k, uids, mids, (u, m, r), test in O.als_data_set_shrink(tr, te, d["medians"],
                                                                d["factors"].tolist()):
        assert list(uids) == d[f"k{k}_user_keys"].tolist()
        assert list(mids) == d[f"k{k}_movie_keys"].tolist()
        assert np.array_equal(u, d[f"k{k}_u"]) and np.array_equal(m, d[f"k{k}_m"])
        assert np.array_equal(r, d[f"k{k}_r"])
        assert test == expected_test(d, k)


def test_set_order_is_not_sorted():
    """The fixtures exercise CPython's set iteration order (ids beyond the
    table size), so a sorted id assignment would not pass."""
    d = fixture(3)
    keys = d["k3_movie_keys"]
    assert not np.all(np.diff(keys) > 0)
