"""CPU: the als_train driver's file contract (movie_lens_data.py:684-713)
with the device solve stubbed out."""
import pickle

import numpy as np


def test_als_train_reads_and_writes_reference_files(tmp_path, monkeypatch):
    from movie_recommender_amd import cpp_ls, train
    k = 3
    uid = np.array([0, 0, 1, 1, 2], np.int32)
    mid = np.array([0, 1, 0, 1, 1], np.int32)
    r = np.array([0.5, -1.0, 0.0, 1.5, 0.25])
    for name, obj in ((f"als{k}_user_ids", {11: 0, 12: 1, 13: 2}),
                      (f"als{k}_movie_ids", {7: 0, 9: 1}),
                      (f"als{k}_user_ratings_train", [uid, mid, r])):
        with open(tmp_path / f"{name}.bin", "wb") as f:
            pickle.dump(obj, f)
    calls = []

    def fake_als(u, i, rr, f, nu, ni, min_r_decrease=0.01, max_iterations=200, algorithm=1):
        calls.append((u, i, rr, f, nu, ni, algorithm))
        return np.arange(nu * (f + 1), dtype=np.float64), np.ones(ni * f), 4

    monkeypatch.setattr(cpp_ls, "als", fake_als)
    out = train.als_train([k], str(tmp_path), verbose=False, algorithm=2)
    (u, i, rr, f, nu, ni, alg), = calls
    assert (f, nu, ni, alg) == (k, 3, 2, 2)
    assert np.array_equal(u, uid) and np.array_equal(i, mid) and np.array_equal(rr, r)
    with open(tmp_path / f"als{k}_user_factors.bin", "rb") as fh:
        U = pickle.load(fh)
    with open(tmp_path / f"als{k}_item_factors.bin", "rb") as fh:
        V = pickle.load(fh)
    assert np.array_equal(U, np.arange(12.0)) and np.array_equal(V, np.ones(6))
    assert out[k][2] == 4
