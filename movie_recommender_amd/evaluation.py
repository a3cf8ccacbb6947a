"""Ranking-agreement evaluation on the GPU, with the reference's interfaces.

* ``als_eval``                  -- ``python/full_data/worker_process.py:262-306``
  (``_als_eval``): every test user's held-out ratings scored with its trained
  factor row, one GPU pass for all users instead of the cluster fan-out;
* ``compute_ranking_agreement`` -- ``python/full_data/my_util.py:101-145``;
* ``ranking_agreements``        -- the same for many users at once.

Agreements are exact: predictions are the reference's fp64 expression in its
order, and the pair counts are integers divided as Python divides them.
"""
import numpy as np

from . import _lib
from .serving import MovieTable


def _lists_to_arrays(pairs):
    off = np.zeros(len(pairs) + 1, np.int64)
    off[1:] = np.cumsum([len(a) for a, _ in pairs])
    act = np.array([r for a, _ in pairs for r in a], np.float64)
    pred = np.array([p for _, p in pairs for p in p], np.float64)
    return off, act, pred


def ranking_agreements(pairs, device=0):
    """``pairs``: list of ``(actual, predicted)`` aligned rating sequences (one
    per user; NaN predicted = no prediction).  Returns ``(agreement, n_agree,
    n_disagree)`` arrays, agreement NaN where the reference returns None."""
    n = len(pairs)
    off, act, pred = _lists_to_arrays(pairs)
    agr = np.zeros(n)
    ag = np.zeros(n, np.int64)
    dis = np.zeros(n, np.int64)
    if n:
        a = act if act.size else np.zeros(1)
        p = pred if pred.size else np.zeros(1)
        _lib.check(_lib.lib().mr_rank_agreement(
            int(device), n, off.ctypes.data_as(_lib.LLP), a.ctypes.data_as(_lib.DP),
            p.ctypes.data_as(_lib.DP), agr.ctypes.data_as(_lib.DP),
            ag.ctypes.data_as(_lib.LLP), dis.ctypes.data_as(_lib.LLP)), "mr_rank_agreement")
    return agr, ag, dis


def compute_ranking_agreement(actual_ratings, predicted_ratings, device=0):
    """``my_util.compute_ranking_agreement``: ``actual_ratings`` and
    ``predicted_ratings`` are ``[(movie_id, rating)]``; returns the fraction of
    ordered actual pairs the predictions order the same way, or None."""
    if len(actual_ratings) == 1:                      # my_util.py:111-115
        return None
    pred = dict(predicted_ratings)
    a = [r for _, r in actual_ratings]
    p = [pred[m] for m, _ in actual_ratings]          # KeyError as in the reference
    v = ranking_agreements([(a, p)], device)[0][0]
    return None if np.isnan(v) else float(v)


def als_eval(user_ratings_test, movie_medians_train, als_user_factors, als_user_ids,
             als_movie_factors, als_movie_ids, num_item_factors, device=0, table=None,
             return_stats=False):
    """``_als_eval``: ``user_ratings_test`` is ``[(user_id, [(movie_id,
    rating)])]``; returns ``[(user_id, agreement)]`` for the users with an
    agreement, in input order.  With ``return_stats`` also a dict with the
    pair counts and the held-out squared error (an RMSE the reference does not
    report)."""
    k = int(num_item_factors)
    own = table is None
    if own:
        table = MovieTable(k, als_movie_factors, als_movie_ids, movie_medians_train, device)
    try:
        rows = [als_user_ids[uid] for uid, _ in user_ratings_test]
        res = table.evaluate(als_user_factors, rows, [l for _, l in user_ratings_test])
    finally:
        if own:
            table.close()
    out = [(uid, float(a)) for (uid, _), a in zip(user_ratings_test, res["agreement"])
           if not np.isnan(a)]
    if return_stats:
        n = int(res["n_pred"].sum())
        res["rmse"] = float(np.sqrt(res["sse"].sum() / n)) if n else float("nan")
        return out, res
    return out
