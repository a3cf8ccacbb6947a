"""Pure-Python restatement of the reference's ALS training-set preparation --
TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Follows ``python/full_data/movie_lens_data.py:409-680`` and
``movie_lens_data_proc.py:393-654`` line by line, with the process pool
replaced by explicit per-process lists (``chunks``) merged exactly as the
``_proc`` helpers merge them.  Pinned by ``tests/golden/prep_*.npz``, made by
``tests/golden/make_golden_prep.py`` from the reference's own
``movie_lens_data_proc`` functions.
"""
import pickle

import numpy


def split_counts(length, num_splits):
    """``my_util.split`` chunk lengths (``my_util.py:17-50``)."""
    if length >= num_splits:
        idx = [int(length * i / num_splits) for i in range(num_splits)]
        return [idx[i + 1] - idx[i] for i in range(num_splits - 1)] + [length - idx[-1]]
    return [1 if i < length else 0 for i in range(num_splits)]


def movie_medians(user_ratings_train):
    """``_extract_movie_ratings`` (``:393-427``) + ``_compute_medians``
    (``:455-471``): numpy.median of every movie's ratings, ascending ids
    (the merged list is sorted by movie id, ``movie_lens_data.py:483-544``)."""
    ratings = {}
    for _, lst in user_ratings_train:
        for m, r in lst:
            ratings.setdefault(m, []).append(r)
    return {m: numpy.median(ratings[m]) for m in sorted(ratings)}


def _drop_users(train, test, min_ratings):
    """``_drop_users`` (``movie_lens_data_proc.py:494-535``)."""
    changed = any(len(l) < min_ratings for _, l in train)
    if changed:
        keep = [i for i in range(len(train)) if len(train[i][1]) >= min_ratings]
        train[:] = [train[i] for i in keep]
        if test is not None:
            test[:] = [test[i] for i in keep]
    return changed


def _count_movies(train, counts):
    """``_count_movies`` (``:538-556``), merged by adding (``add_merge_var_into_dict``)."""
    for _, lst in train:
        for m, _ in lst:
            counts[m] = counts.get(m, 0) + 1


def _drop_movies(train, drop):
    """``_drop_movies`` (``:559-586``)."""
    for _, lst in train:
        if any(m in drop for m, _ in lst):
            lst[:] = [(m, r) for m, r in lst if m not in drop]


def _collect(train):
    """``_collect_ids`` (``:589-608``)."""
    movies, users = set(), set()
    for u, lst in train:
        for m, _ in lst:
            movies.add(m)
            users.add(u)
    return movies, users


def _merge_sets(sets):
    """``update_var_into_set`` (``:246-261``): own set (last) copied, then
    updated with the pipes' sets (pickled through the pipe) in order."""
    merged = sets[-1].copy()
    for s in sets[:-1]:
        merged.update(pickle.loads(pickle.dumps(s)))
    return merged


def als_data_set_shrink(chunks_train, chunks_test, medians, factors_list):
    """``als_data_set_shrink_mp`` (``movie_lens_data.py:547-680``) over
    per-process lists (own process last).  Lists are shrunk in place.
    Returns ``[(k, als_user_ids, als_movie_ids, (u, m, r arrays), test list)]``."""
    out = []
    for k in factors_list:
        changed = True
        while changed:
            flags = [_drop_users(tr, te, k + 1) for tr, te in zip(chunks_train, chunks_test)]
            changed = any(flags)
            counts = {}
            for tr in chunks_train:
                _count_movies(tr, counts)
            uncommon = {m for m in counts if counts[m] < k}
            if uncommon:
                changed = True
                for tr in chunks_train:
                    _drop_movies(tr, uncommon)
        col = [_collect(tr) for tr in chunks_train]
        movie_ids = _merge_sets([c[0] for c in col])
        user_ids = _merge_sets([c[1] for c in col])
        als_movie_ids = {m: i for i, m in enumerate(movie_ids)}
        als_user_ids = {u: i for i, u in enumerate(user_ids)}
        u, m, r = [], [], []
        for tr in chunks_train:                      # concat: pipes, then own
            for uid, lst in tr:
                for mid, rating in lst:
                    u.append(als_user_ids[uid])
                    m.append(als_movie_ids[mid])
                    r.append(rating - medians[mid])
        test = None
        if chunks_test[0] is not None:
            test = [x for te in chunks_test for x in te]
        out.append((k, als_user_ids, als_movie_ids,
                    (numpy.array(u, numpy.int32), numpy.array(m, numpy.int32),
                     numpy.array(r, numpy.float64)), test))
    return out


def chunk(lst, counts):
    out, o = [], 0
    for c in counts:
        out.append(lst[o:o + c])
        o += c
    return out
