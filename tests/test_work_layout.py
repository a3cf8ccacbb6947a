"""Host restatement of the Gram work list (engine.hip build_side +
place_chunks_by_xcd), checked for the properties that make the XCD-aware chunk
placement bit-identical: it only permutes the full chunks of split entities
among their own slots, unsplit entities keep their positions (the fused CG
start sums its per-block pairs by position), and XCD x = (slot // 4) % 8
receives the x-th eighth of the chunks in opposite-id order.  The GPU test
test_full_size_context_build_exact compares the device work list with the
same restatement at the ML-full shape."""
import numpy as np

from test_gpu_parity import expected_layout


def _case(seed=0, n_ent=300, n_other=5000, chunk=64):
    rng = np.random.RandomState(seed)
    deg = np.minimum(rng.zipf(1.5, n_ent), 40 * chunk)
    ids = np.repeat(np.arange(n_ent), deg)
    other = np.concatenate([np.sort(rng.choice(n_other, d, replace=False)) for d in deg])
    order = rng.permutation(len(ids))       # input order is not entity-major
    return ids[order].astype(np.int32), other[order].astype(np.int32), \
        rng.uniform(1, 5, len(ids)), n_ent, chunk


def test_placement_is_a_slot_preserving_permutation():
    ids, other, r, E, chunk = _case()
    _, idx, _, base = expected_layout(ids, other, r, E, chunk=chunk)
    _, _, _, placed = expected_layout(ids, other, r, E, chunk=chunk,
                                      xcd_table_bytes=64 << 20)
    assert sorted(base) == sorted(placed)
    full = [p for p, w in enumerate(base) if w[3] >= 0 and w[1] == chunk]
    assert len(full) >= 64
    moved = [p for p in range(len(base)) if base[p] != placed[p]]
    assert moved and set(moved) <= set(full)          # only full chunks move
    assert all(placed[p][3] >= 0 and placed[p][1] == chunk for p in full)
    # XCD groups in opposite-id order: max key of XCD x <= min key of XCD x+1
    keys = {}
    for p in full:
        b, ln = placed[p][0], placed[p][1]
        keys.setdefault((p // 4) % 8, []).append(int(idx[b + ln // 2]))
    xs = sorted(keys)
    for a, b in zip(xs, xs[1:]):
        assert max(keys[a]) <= min(keys[b])


def test_small_tables_are_not_placed():
    ids, other, r, E, chunk = _case(seed=1)
    _, _, _, base = expected_layout(ids, other, r, E, chunk=chunk)
    _, _, _, same = expected_layout(ids, other, r, E, chunk=chunk,
                                    xcd_table_bytes=16 << 20)
    assert base == same
