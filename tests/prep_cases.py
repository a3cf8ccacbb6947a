"""Decoding of the preparation fixtures (tests/golden/prep_p*.npz)."""
import numpy as np

from conftest import load_golden


def fixture(p):
    d = load_golden(f"prep_p{p}.npz")
    o = d["train_off"]
    d["train"] = [(int(u), [(int(m), float(r)) for m, r in zip(d["train_mid"][o[i]:o[i + 1]],
                                                              d["train_r"][o[i]:o[i + 1]])])
                  for i, u in enumerate(d["train_uid"])]
    t = d["test_off"]
    d["test"] = [(int(u), [(int(m), float(r)) for m, r in zip(d["test_mid"][t[i]:t[i + 1]],
                                                             d["test_r"][t[i]:t[i + 1]])])
                 for i, u in enumerate(d["train_uid"])]
    d["medians"] = dict(zip(d["med_keys"].tolist(), d["med_vals"].tolist()))
    return d


def expected_test(d, k):
    o = d[f"k{k}_test_off"]
    return [(int(u), [(int(m), float(r)) for m, r in zip(d[f"k{k}_test_mid"][o[i]:o[i + 1]],
                                                        d[f"k{k}_test_r"][o[i]:o[i + 1]])])
            for i, u in enumerate(d[f"k{k}_test_uid"])]
