"""ALS model training driver: ``movie_lens_data.als_train`` on the GPU core.

Mirrors ``python/full_data/movie_lens_data.py:684-713``: for every factor k,
load ``als{k}_movie_ids.bin``, ``als{k}_user_ids.bin`` and
``als{k}_user_ratings_train.bin`` (pickled ``[int32 user ids, int32 movie
ids, float64 rating - median]``) from ``als_dir`` -- the files
``prep.als_data_set_shrink(..., out_dir=als_dir)`` writes in the reference's
format -- run ``cpp_ls.als`` (the drop-in wrapper: U0 then V0 drawn from
NumPy's global RNG, then the device-resident ALS behind ``als_from_python``)
and pickle the factor vectors to ``als{k}_user_factors.bin`` /
``als{k}_item_factors.bin`` (1-D float64 arrays, ``U: users * (k+1)``,
``V: movies * k``), as the reference does.

The ``.bin`` files read here are the ones this package (or the reference)
wrote into ``als_dir``; pickle is the reference's own file format.
"""
import os
import pickle
import time

from . import cpp_ls


def _current_time():
    return time.strftime("%H:%M:%S")


def _load(als_dir, name):
    with open(os.path.join(als_dir, name + ".bin"), "rb") as f:
        return pickle.load(f)


def _dump(als_dir, name, obj):
    with open(os.path.join(als_dir, name + ".bin"), "wb") as f:
        pickle.dump(obj, f)


def als_train(factors_list, als_dir, thread_count=None, algorithm=1, verbose=True):
    """Trains one ALS model per factor (``movie_lens_data.py:684-713``).

    Returns ``{k: (user_factors, item_factors, iterations)}`` besides writing
    the two factor files per k."""
    if thread_count is not None:
        cpp_ls.set_thread_count(thread_count)
    out = {}
    for factor in factors_list:
        num_items = len(_load(als_dir, f"als{factor}_movie_ids"))
        num_users = len(_load(als_dir, f"als{factor}_user_ids"))
        user_ids_train, item_ids_train, ratings_train = _load(
            als_dir, f"als{factor}_user_ratings_train")
        if verbose:
            print(_current_time(), "Building ALS factor", factor, "model")
        user_factors, item_factors, iterations = cpp_ls.als(
            user_ids_train, item_ids_train, ratings_train, factor,
            num_users, num_items, algorithm=algorithm)
        if verbose:
            print(_current_time(), "ALS took", iterations, "iterations.",
                  'Saving "user_factors" and "item_factors" to disk')
        _dump(als_dir, f"als{factor}_user_factors", user_factors)
        _dump(als_dir, f"als{factor}_item_factors", item_factors)
        out[factor] = (user_factors, item_factors, iterations)
    return out
