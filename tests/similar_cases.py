"""Decoding of the similar-movies fixtures (tests/golden/similar_*.npz)."""
from conftest import load_golden


def fixture(name):
    d = load_golden(f"similar_{name}.npz")
    o = d["off"]
    users, ratings = d["users"].tolist(), d["ratings"].tolist()
    d["movie_ratings"] = [(int(m), dict(zip(users[o[i]:o[i + 1]], ratings[o[i]:o[i + 1]])))
                          for i, m in enumerate(d["movie_ids"])]
    g = d["g_off"]
    vals = d["g_vals"].tolist()
    d["genres"] = {int(k): set(vals[g[i]:g[i + 1]]) for i, k in enumerate(d["g_keys"])}
    return d


def expected(d, nres):
    c = d[f"n{nres}_count"]
    out, o = [], 0
    for n in c:
        out.append((tuple(d[f"n{nres}_ids"][o:o + n].tolist()),
                    tuple(d[f"n{nres}_scores"][o:o + n].tolist())))
        o += n
    return out
