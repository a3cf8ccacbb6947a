"""Shared helpers for the factor-consumer tests: golden fixture decoding and a
vectorised exact restatement of the reference scoring order for larger
synthetic cases (NumPy elementwise multiply then add == Python float ops)."""
import numpy as np

from conftest import load_golden

KS = (3, 11, 64)


def fixture(k):
    d = load_golden(f"serving_k{k}.npz")
    d["als_ids"] = {int(m): j for j, m in enumerate(d["als_keys"])}
    d["med"] = {int(m): float(v) for m, v in zip(d["med_keys"], d["med_vals"])}
    o = d["u_off"]
    d["lists"] = [[(int(m), float(r)) for m, r in zip(d["u_mid"][o[u]:o[u + 1]],
                                                      d["u_r"][o[u]:o[u + 1]])]
                  for u in range(len(o) - 1)]
    t = d["t_off"]
    d["t_lists"] = [[(int(m), float(r)) for m, r in zip(d["t_mid"][t[i]:t[i + 1]],
                                                        d["t_r"][t[i]:t[i + 1]])]
                    for i in range(len(t) - 1)]
    ro = d["rec_off"]
    d["recs"] = [[(float(s), int(m)) for s, m in zip(d["rec_score"][ro[u]:ro[u + 1]],
                                                    d["rec_mid"][ro[u]:ro[u + 1]])]
                 for u in range(len(ro) - 1)]
    return d


def exact_scores(X, Vc, med):
    """Reference order for many users x candidates: s = 0; s += x_j v_j ...;
    s += bias; s += median (models.py:725-731), all in fp64 without FMA."""
    X = np.atleast_2d(X)
    k = Vc.shape[1]
    s = np.zeros((X.shape[0], Vc.shape[0]))
    for j in range(k):
        s = s + X[:, j:j + 1] * Vc[None, :, j]
    s = s + X[:, k:k + 1]
    return s + med[None, :]


def exact_top_n(scores, mids, excluded, n):
    """recommend.py:93-106 on one score row: (score, movie id) descending,
    skipping excluded movie ids, first n."""
    order = np.lexsort((-mids.astype(np.int64), -scores))
    out = []
    for c in order:
        if int(mids[c]) in excluded:
            continue
        out.append((float(scores[c]), int(mids[c])))
        if len(out) >= n:
            break
    return out


def synthetic_table(k, n_als, n_med_only, seed, ties=20):
    rs = np.random.RandomState(seed)
    ids = rs.choice(np.arange(1, 10 * (n_als + n_med_only)), n_als + n_med_only, replace=False)
    V = rs.normal(0, 0.6, (n_als, k))
    med = rs.choice(np.arange(1, 11) / 2.0, n_als)
    for _ in range(ties):
        a, b = rs.choice(n_als, 2, replace=False)
        V[b], med[b] = V[a], med[a]
    als_ids = {int(m): j for j, m in enumerate(ids[:n_als])}
    keys = list(ids[:n_als]) + list(ids[n_als:])
    vals = list(med) + list(rs.choice(np.arange(1, 11) / 2.0, n_med_only))
    order = rs.permutation(len(keys))
    medians = {int(keys[i]): float(vals[i]) for i in order}
    return V.reshape(-1), als_ids, medians
