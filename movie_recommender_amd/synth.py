"""Seeded MovieLens-shaped synthetic ratings (host-side data preparation).

There is no MovieLens data in this environment, so benchmarks and statistical
tests run on a synthetic set with MovieLens' shape:

* user activity ~ LogNormal(0, 1.2); item popularity ~ rank^-0.9 with
  shuffled ranks; N (user, item) draws, de-duplicated;
* ratings on the half-star scale {0.5 .. 5.0}, either from a low-rank model
  plus noise (``model="lowrank"``, default) or uniform (``model="uniform"``,
  the variant the survey's CPU timing used);
* the ALS degree shrink of ``als_data_set_shrink_mp``
  (``python/full_data/movie_lens_data.py:565-591``: users need >= k+1
  ratings, movies >= k, iterated to a fixed point), zero-based id remap, and
  per-movie median subtraction (``movie_lens_data_proc.py:611-654``).

Configs: C1/C2 = ML-100K shape (610 users, 9,742 items,
100,836 ratings), C3/C4 = ML-full shape (283,228 / 58,098 / 27,753,444).
"""
from dataclasses import dataclass, field

import numpy as np

DATA_SEED = 20261015

SHAPES = {
    "ml-100k": (610, 9_742, 100_836),
    "ml-full": (283_228, 58_098, 27_753_444),
}


@dataclass
class RatingSet:
    user_ids: np.ndarray        # int32, zero-based, contiguous
    item_ids: np.ndarray        # int32, zero-based, contiguous
    ratings: np.ndarray         # float64, rating - movie median
    num_users: int
    num_items: int
    k: int
    test_user_ids: np.ndarray = field(default=None)
    test_item_ids: np.ndarray = field(default=None)
    test_ratings: np.ndarray = field(default=None)
    medians: np.ndarray = field(default=None)   # per (compact) item: train-split median
    meta: dict = field(default_factory=dict)

    @property
    def n(self):
        return len(self.ratings)


def _draw(rng, p, n, chunk=1 << 22):
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    out = np.empty(n, np.int64)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = np.searchsorted(cdf, rng.random(e - s), side="right")
    np.minimum(out, len(p) - 1, out=out)
    return out


def raw_pairs(n_users, n_items, n_draws, seed=DATA_SEED, model="lowrank",
              rank=8, noise=0.6):
    """De-duplicated (user, item, rating) draws, sorted by (user, item)."""
    rng = np.random.default_rng(seed)
    act = rng.lognormal(0.0, 1.2, n_users)
    pop = (rng.permutation(n_items) + 1.0) ** -0.9
    u = _draw(rng, act / act.sum(), n_draws)
    i = _draw(rng, pop / pop.sum(), n_draws)
    key = np.unique(u * n_items + i)
    u = (key // n_items).astype(np.int32)
    i = (key % n_items).astype(np.int32)
    if model == "uniform":
        r = rng.integers(1, 11, len(u)) / 2.0
    else:
        s = 1.0 / np.sqrt(rank)
        Ut = rng.normal(0, s, (n_users, rank)).astype(np.float32)
        Vt = rng.normal(0, s, (n_items, rank)).astype(np.float32)
        ub = rng.normal(0, 0.4, n_users)
        ib = rng.normal(0, 0.5, n_items)
        r = 3.5 + ub[u] + ib[i] + rng.normal(0, noise, len(u))
        for s0 in range(0, len(u), 1 << 22):
            e0 = min(len(u), s0 + (1 << 22))
            r[s0:e0] += np.einsum("nj,nj->n", Ut[u[s0:e0]], Vt[i[s0:e0]])
        r = np.clip(np.round(r * 2.0) / 2.0, 0.5, 5.0)
    return u, i, r


def shrink(u, i, k, n_users, n_items):
    """Degree pruning of ``als_data_set_shrink_mp``
    (``movie_lens_data.py:565-591``): drop users with < k+1 ratings, then
    movies with < k ratings, until nothing changes.  Returns a keep mask."""
    keep = np.ones(len(u), bool)
    while True:
        uc = np.bincount(u[keep], minlength=n_users)
        drop_u = keep & (uc[u] < k + 1)
        keep &= ~drop_u
        ic = np.bincount(i[keep], minlength=n_items)
        drop_i = keep & (ic[i] < k)
        keep &= ~drop_i
        if not drop_u.any() and not drop_i.any():
            return keep


def item_medians(i, r, n_items):
    """Per-item median rating (ties average, as ``numpy.median``)."""
    order = np.lexsort((r, i))
    i_s, r_s = i[order], r[order]
    cnt = np.bincount(i_s, minlength=n_items)
    off = np.zeros(n_items + 1, np.int64)
    np.cumsum(cnt, out=off[1:])
    med = np.zeros(n_items)
    nz = cnt > 0
    lo = off[:-1] + (cnt - 1) // 2
    hi = off[:-1] + cnt // 2
    med[nz] = 0.5 * (r_s[lo[nz]] + r_s[hi[nz]])
    return med


def movielens_like(shape="ml-full", k=64, seed=DATA_SEED, model="lowrank",
                   test_ratio=0.0, scale=1.0):
    """Build an ALS training set of the given MovieLens shape for factor k.

    ``test_ratio`` > 0 holds out that fraction of each user's ratings (the
    reference's per-user 80/20 split); held-out pairs whose user or item
    does not survive the shrink are dropped, as in the reference.
    ``scale`` < 1 shrinks users/items/draws proportionally (CPU samples).
    """
    nu, ni, nd = SHAPES[shape] if isinstance(shape, str) else shape
    nu, ni, nd = max(1, int(nu * scale)), max(1, int(ni * scale)), max(1, int(nd * scale))
    u, i, r = raw_pairs(nu, ni, nd, seed, model)
    rng = np.random.default_rng(seed + 1)
    test = np.zeros(len(u), bool)
    if test_ratio > 0:
        test = rng.random(len(u)) < test_ratio
    tu, ti, tr = u[~test], i[~test], r[~test]
    med = item_medians(ti, tr, ni)
    keep = shrink(tu, ti, k, nu, ni)
    tu, ti, tr = tu[keep], ti[keep], tr[keep]
    umap = np.full(nu, -1, np.int64)
    imap = np.full(ni, -1, np.int64)
    uu = np.unique(tu)
    ii = np.unique(ti)
    umap[uu] = np.arange(len(uu))
    imap[ii] = np.arange(len(ii))
    rs = RatingSet(umap[tu].astype(np.int32), imap[ti].astype(np.int32),
                   (tr - med[ti]).astype(np.float64), len(uu), len(ii), k)
    rs.medians = med[ii]
    if test_ratio > 0:
        hu, hi_, hr = u[test], i[test], r[test]
        ok = (umap[hu] >= 0) & (imap[hi_] >= 0)
        rs.test_user_ids = umap[hu[ok]].astype(np.int32)
        rs.test_item_ids = imap[hi_[ok]].astype(np.int32)
        rs.test_ratings = (hr[ok] - med[hi_[ok]]).astype(np.float64)
    rs.meta = {"shape": [nu, ni, nd], "seed": seed, "model": model,
               "raw_pairs": int(len(u)), "test_ratio": test_ratio}
    return rs


def dense_fixture(num_users, num_items, k, keep=0.8, seed=7, noise=0.1):
    """Fully-observed low-rank fixture of ``cpp/python/cpp_ls_test.py:73-147``
    (every user rates every item, noise N(0, noise), shuffled, ``keep``
    fraction used for training).  Returns (train u, i, r, test u, i, r)."""
    rs = np.random.default_rng(seed)
    Ut = rs.uniform(-1, 1, (num_users, k + 1))
    Vt = rs.uniform(-1, 1, (num_items, k))
    uu, ii = np.meshgrid(np.arange(num_users), np.arange(num_items), indexing="ij")
    uu = uu.ravel().astype(np.int32)
    ii = ii.ravel().astype(np.int32)
    r = np.einsum("nj,nj->n", Ut[uu, :k], Vt[ii]) + Ut[uu, k] + rs.normal(0, noise, len(uu))
    perm = rs.permutation(len(uu))
    n = int(np.ceil(len(uu) * keep))
    a, b = perm[:n], perm[n:]
    return uu[a], ii[a], r[a], uu[b], ii[b], r[b]


# ---------------------------------------------------------------------------
# C5: synthetic 10 M users x 1 M items x 1e9 ratings (SURVEY.md 8, configs[4])
# ---------------------------------------------------------------------------
C5_SHAPE = (10_000_000, 1_000_000, 1_000_000_000)


class C5Generator:
    """Streamed generator of the C5 roofline workload, never materialised
    whole on one host.  User activity ~ LogNormal(0, 1.2) fixes every user's
    degree up front (rounded, >= 1); item popularity ~ rank^-0.9 over
    shuffled ranks, drawn through a 2^24-entry inverse-CDF table; ratings are
    uniform half-stars minus 3.0 (rating - median).  Users are generated in
    blocks of ``block`` with their own seeded streams, so any rank can
    regenerate any block: a rank's user view is its own blocks, its item view
    a filtered pass over all blocks.  Duplicate (user, item) pairs are kept
    (the reference treats them as separate ratings) and there is no degree
    shrink (the reference's k+1 / k rule is MovieLens preparation; here users
    with fewer ratings than unknowns simply give singular blocks, which CG
    handles as the reference's CG does)."""

    LUT_BITS = 24

    def __init__(self, scale=1.0, seed=DATA_SEED, block=1 << 16, shape=C5_SHAPE):
        nu, ni, nr = shape
        self.num_users = max(1, int(nu * scale))
        self.num_items = max(1, int(ni * scale))
        n_target = max(1, int(nr * scale))
        self.seed = seed
        self.block = block
        rng = np.random.default_rng(seed)
        act = rng.lognormal(0.0, 1.2, self.num_users)
        self.deg = np.maximum(1, np.rint(act * (n_target / act.sum()))).astype(np.int64)
        self.off = np.zeros(self.num_users + 1, np.int64)
        np.cumsum(self.deg, out=self.off[1:])
        self.n = int(self.off[-1])
        pop = (rng.permutation(self.num_items) + 1.0) ** -0.9
        self.p_item = pop / pop.sum()
        cdf = np.cumsum(self.p_item)
        T = 1 << self.LUT_BITS
        self.lut = np.minimum(np.searchsorted(cdf, (np.arange(T) + 0.5) / T, side="right"),
                              self.num_items - 1).astype(np.int32)

    @property
    def n_blocks(self):
        return (self.num_users + self.block - 1) // self.block

    def gen_block(self, b):
        """(user ids, item ids, ratings) of users [b*block, (b+1)*block)."""
        u0 = b * self.block
        u1 = min(self.num_users, u0 + self.block)
        n = int(self.off[u1] - self.off[u0])
        rng = np.random.default_rng([self.seed, 5, b])
        uid = np.repeat(np.arange(u0, u1, dtype=np.int32), self.deg[u0:u1])
        iid = self.lut[rng.integers(0, 1 << self.LUT_BITS, n)]
        r = rng.integers(1, 11, n) / 2.0 - 3.0
        return uid, iid, r

    def expected_item_counts(self):
        return self.p_item * self.n

    def user_view(self, u0, u1):
        parts = [self.gen_block(b) for b in range(u0 // self.block,
                                                   (u1 + self.block - 1) // self.block)]
        uid, iid, r = (np.concatenate(x) for x in zip(*parts)) if parts else \
            (np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0))
        sel = (uid >= u0) & (uid < u1)
        return uid[sel], iid[sel], r[sel]

    def item_view(self, i0, i1):
        us, is_, rs = [], [], []
        for b in range(self.n_blocks):
            uid, iid, r = self.gen_block(b)
            sel = (iid >= i0) & (iid < i1)
            us.append(uid[sel]); is_.append(iid[sel]); rs.append(r[sel])
        return np.concatenate(us), np.concatenate(is_), np.concatenate(rs)

    def all_ratings(self):
        parts = [self.gen_block(b) for b in range(self.n_blocks)]
        return tuple(np.concatenate(x) for x in zip(*parts))
