"""Host restatement of the Gram work list (engine.hip build_side +
build_work_xcd), checked for the properties the XCD-aligned opposite-range cut
relies on: every rating in exactly one work item, each heavy entity's
partial records numbered consecutively in range order (slab_reduce sums them
in that order), a chunk of range x gathers opposite rows only from
[x n / 8, (x+1) n / 8) and sits on XCD x = (slot // 4) % 8 (a dry queue
yields to the fullest), chunks before the unsplit entities, and small tables
keep the plain layout.  The GPU tests test_full_size_context_build_exact and
test_c4_mlfull_k128_layout_and_gram compare the device work list with the
same restatement at full size."""
import numpy as np

from test_gpu_parity import expected_layout


def _case(seed=0, n_ent=300, n_other=5000, chunk=64, sorted_lists=True):
    rng = np.random.RandomState(seed)
    deg = np.minimum(rng.zipf(1.5, n_ent), 40 * chunk)
    ids = np.repeat(np.arange(n_ent), deg)
    other = np.concatenate([np.sort(rng.choice(n_other, d, replace=False)) for d in deg])
    # sorted_lists: input ordered by opposite id (as ML data ordered by user
    # is for the items side); else a random input order
    order = np.argsort(other, kind="stable") if sorted_lists else rng.permutation(len(ids))
    return ids[order].astype(np.int32), other[order].astype(np.int32), \
        rng.uniform(1, 5, len(ids)), n_ent, n_other, chunk


def _check(ids, other, r, E, n_other, chunk):
    off, idx, _, work = expected_layout(ids, other, r, E, chunk=chunk,
                                        xcd_table_bytes=64 << 20, k=64, n_other=n_other)
    cover = np.zeros(off[-1], np.int32)
    for b, ln, e, s in work:
        assert off[e] <= b and b + ln <= off[e + 1]
        cover[b:b + ln] += 1
    assert np.all(cover == 1)
    n_chunks = sum(1 for w in work if w[3] >= 0)
    assert all(w[3] >= 0 for w in work[:n_chunks]) and all(w[3] < 0 for w in work[n_chunks:])
    light = [w[1] for w in work[n_chunks:]]
    assert light == sorted(light, reverse=True)
    slabs = {}
    for b, ln, e, s in work[:n_chunks]:
        slabs.setdefault(e, []).append((s, b))
    for e, v in slabs.items():
        v.sort()
        assert [s for s, _ in v] == list(range(v[0][0], v[0][0] + len(v)))
        assert [b for _, b in v] == sorted(b for _, b in v)     # range order = rating order
    return off, idx, work, n_chunks


def test_xcd_ranges_sorted_lists():
    ids, other, r, E, n_other, chunk = _case()
    off, idx, work, n_chunks = _check(ids, other, r, E, n_other, chunk)
    assert n_chunks >= 64
    on_home = 0
    for p, (b, ln, e, s) in enumerate(work[:n_chunks]):
        lo, hi = int(idx[b]), int(idx[b + ln - 1])
        x = lo * 8 // n_other
        assert hi * 8 // n_other == x            # one opposite range per chunk
        on_home += (p // 4) % 8 == x
    assert on_home >= 0.75 * n_chunks           # the rest: dry queues yielding


def test_xcd_ranges_unsorted_lists_fall_back_to_fixed_chunks():
    ids, other, r, E, n_other, chunk = _case(seed=2, sorted_lists=False)
    off, idx, work, n_chunks = _check(ids, other, r, E, n_other, chunk)
    assert all(ln == chunk or b + ln == off[e + 1] for b, ln, e, s in work[:n_chunks])


def test_small_tables_are_not_placed():
    ids, other, r, E, n_other, chunk = _case(seed=1)
    _, _, _, base = expected_layout(ids, other, r, E, chunk=chunk)
    _, _, _, same = expected_layout(ids, other, r, E, chunk=chunk,
                                    xcd_table_bytes=16 << 20, k=64, n_other=n_other)
    assert base == same


def pair_pos(b, n):
    """Host restatement of kernels.hip pair_pos: the work-list position of
    block b of the NB = 8 pair Gram (one work item per 128-thread block)."""
    if b >= (n & ~31):
        return b
    return 32 * (b >> 5) + 4 * (b & 7) + ((b >> 3) & 3)


def test_pair_gram_block_placement():
    """The pair Gram keeps the work list's XCD placement: block b runs on XCD
    b mod 8 (dispatch round-robin) and takes the position p the list dealt
    to XCD (p // 4) % 8, for every block of a full group of 32; the mapping
    is a bijection on [0, n) for every n (the tail keeps p = b)."""
    for n in (1, 31, 32, 33, 64, 100, 1000, 4097):
        ps = [pair_pos(b, n) for b in range(n)]
        assert sorted(ps) == list(range(n)), n
        full = n & ~31
        assert all((ps[b] // 4) % 8 == b % 8 for b in range(full)), n


def test_pair_gram_block_partition():
    """The 36 upper 16 x 16 blocks at NB = 8 split 18 / 18 between the pair's
    waves (kernels.hip pair_owner / pair_local): role 0 the blocks inside
    segments 0-3 and (bi <= 3, bj in {4, 5}), role 1 the rest; each role's
    folded diagonal pairs (2m, 2m + 1) are its own."""
    def owner(bi, bj):
        return 0 if (bi <= 3 and bj <= 5) else 1

    blocks = [(bi, bj) for bi in range(8) for bj in range(bi, 8)]
    assert sum(owner(*b) == 0 for b in blocks) == 18 == sum(owner(*b) == 1 for b in blocks)
    for m in range(4):
        assert owner(2 * m, 2 * m) == owner(2 * m + 1, 2 * m + 1) == (0 if m < 2 else 1)
    # partner segments each role reads: role 0 only 4, 5; role 1 only 0-3
    need0 = {s for (bi, bj) in blocks if owner(bi, bj) == 0 for s in (bi, bj)} - {0, 1, 2, 3}
    need1 = {s for (bi, bj) in blocks if owner(bi, bj) == 1 for s in (bi, bj)} - {4, 5, 6, 7}
    assert need0 == {4, 5} and need1 == {0, 1, 2, 3}
