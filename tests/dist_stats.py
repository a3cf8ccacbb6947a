"""Two-sample comparison of a per-seed sample against the reference's pool
(realistic-data parity, VERDICT r04 "do this" 1).

On ill-conditioned realistic data the reference is chaotic: its factors, its
`ret` and its held-out RMSE move with the thread count at a fixed seed
(`matrix.cpp:7-16, 765-771`: the spread sets the summation order of every
CG scalar; the outer stop `:871-875` then amplifies it).  Parity there is a
statement about distributions: the GPU's per-seed results must be a sample
of the same distribution as the reference's runs over seeds x thread counts.
"""
import json
import os

import numpy as np

METRICS = ("test_rmse", "train_rmse", "ret", "rank_agreement")
P_MIN = 0.05          # two-sided, per metric ("at p >= 0.05")


def load_dist(golden_dir, k):
    with open(os.path.join(golden_dir, f"dist_ml100k_k{k}.json")) as f:
        return json.load(f)


def runs_of(dist, kind):
    return [r for r in dist["runs"] if r["kind"] == kind]


def compare(sample, pool, metrics=METRICS):
    """{metric: (mean sample, mean pool, Mann-Whitney p, KS p)} -- two-sided
    tests of ``sample`` (list of dicts) against ``pool`` (list of dicts)."""
    from scipy.stats import ks_2samp, mannwhitneyu
    out = {}
    for m in metrics:
        x = np.array([r[m] for r in sample], np.float64)
        y = np.array([r[m] for r in pool], np.float64)
        out[m] = (float(x.mean()), float(y.mean()),
                  float(mannwhitneyu(x, y, alternative="two-sided").pvalue),
                  float(ks_2samp(x, y).pvalue))
    return out


def describe(res):
    return "; ".join(f"{m} {a:.4f} vs {b:.4f} (MW p={p:.3f}, KS p={q:.3f})"
                     for m, (a, b, p, q) in res.items())


def failing(res, p_min=P_MIN):
    return {m: v for m, v in res.items() if v[2] < p_min}


def seed_ranges(pool, metric):
    """Per-seed (min, max) over the reference's thread counts, and W, the
    largest such range (the reference's within-seed chaos)."""
    seeds = sorted({r["seed"] for r in pool})
    rng = {s: (min(r[metric] for r in pool if r["seed"] == s),
               max(r[metric] for r in pool if r["seed"] == s)) for s in seeds}
    return rng, max(hi - lo for lo, hi in rng.values())
