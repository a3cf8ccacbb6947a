"""CPU: the oracle restatement against golden vectors of the compiled reference.

Golden fixtures were produced by ``oracle/_ref/cpp_ls_lib.so`` (reference
sources ``cpp/ls_lib``), see ``tests/golden/make_golden.py``.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden, rel_err
from oracle import als_oracle as O

DENSE = ["als_dense_38x45_k5.npz", "als_dense_40x45_k3.npz",
         "als_dense_300x200_k10.npz", "als_dense_200x150_k32.npz"]
MLSHAPE = ["als_mlshape_k10_it2.npz", "als_mlshape_k10_it4.npz",
           "als_mlshape_k32_it2.npz", "als_mlshape_k32_it4.npz"]


def test_cg_golden():
    d = load_golden("cg_dense_200x50.npz")
    x, it, rr = O.cg_least_squares(d["row_ptr"], d["col_idx"], d["vals"], int(d["ncols"]),
                                   d["b"], d["x0"])
    assert it == int(d["iterations"])
    assert rel_err(x, d["x"]) < 1e-12
    assert abs(rr - float(d["final_rr"])) <= 1e-9 * max(1.0, float(d["final_rr"]))
    # the reference's own statistical check (cpp_ls_test.py:30-39)
    assert np.mean(np.abs(x - d["x_real"])) < 0.1


@pytest.mark.parametrize("name", DENSE)
def test_als_design_form_golden(name):
    d = load_golden(name)
    k = int(d["k"])
    U, V, ret, _ = O.als_design(d["user_ids"], d["item_ids"], d["ratings"], k, d["U0"], d["V0"])
    assert ret == int(d["ret"])
    assert rel_err(U, d["U"]) < 1e-12 and rel_err(V, d["V"]) < 1e-12


@pytest.mark.parametrize("name", DENSE + MLSHAPE)
def test_als_block_form_golden(name):
    """The block-Gram form (what the HIP path computes) equals the reference."""
    d = load_golden(name)
    k = int(d["k"])
    max_it = 200 if name.startswith("als_dense") else int(name.split("_it")[1].split(".")[0])
    U, V, ret, _ = O.als_block(d["user_ids"], d["item_ids"], d["ratings"], k, d["U0"], d["V0"],
                               max_iteration=max_it)
    assert ret == int(d["ret"])
    tol = max(1e-10, 20 * float(d["tc_spread"]))
    assert rel_err(U, d["U"]) < tol and rel_err(V, d["V"]) < tol


@pytest.mark.parametrize("name", DENSE[:3])
def test_als_block_fp32_within_tolerance(name):
    """fp32 Gram/vectors + fp64 scalars stays within 1e-5 of the reference."""
    d = load_golden(name)
    k = int(d["k"])
    U, V, ret, _ = O.als_block(d["user_ids"], d["item_ids"], d["ratings"], k, d["U0"], d["V0"],
                               dtype=np.float32)
    assert ret == int(d["ret"])
    assert rel_err(U, d["U"]) < 1e-5 and rel_err(V, d["V"]) < 1e-5


def test_reference_statistical_check_on_golden():
    # cpp_ls_test.test_als: held-out mean abs error < 0.15
    d = load_golden("als_dense_38x45_k5.npz")
    p = O.predict(d["U"], d["V"], d["test_user_ids"], d["test_item_ids"], 5)
    assert np.mean(np.abs(p - d["test_ratings"])) < 0.15


def test_band_fixture_regenerates():
    """The G4 band's data set is regenerated bit-identically by synth."""
    from movie_recommender_amd import synth
    with open(os.path.join(GOLDEN, "band_ml100k_k10.json")) as f:
        band = json.load(f)
    rs = synth.movielens_like(band["shape"], band["k"], seed=band["data_seed"],
                              test_ratio=band["test_ratio"])
    assert rs.n == band["n_train"] and len(rs.test_ratings) == band["n_test"]
    assert abs(float(np.sum(rs.ratings)) - band["ratings_checksum"]) < 1e-6


def test_exact_solve_matches_numpy_lstsq():
    from movie_recommender_amd import synth
    u, i, r, *_ = synth.dense_fixture(30, 25, 4, 0.8, seed=3)
    rs = np.random.RandomState(1)
    V = rs.uniform(-1, 1, 25 * 4)
    G, c = O.gram_user(u, i, r, V, 4, 30)
    x = np.zeros(30 * 5)
    assert O.solve_blocks(G, c, x) == 0
    Vm = V.reshape(-1, 4)
    for uu in range(30):
        sel = u == uu
        A = np.hstack([Vm[i[sel]], np.ones((sel.sum(), 1))])
        ref = np.linalg.lstsq(A, r[sel], rcond=None)[0]
        assert np.allclose(x[uu * 5:(uu + 1) * 5], ref, atol=1e-9)
