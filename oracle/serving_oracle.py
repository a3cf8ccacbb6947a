"""Pure-Python/NumPy restatement of the reference's factor *consumers* --
TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

SURVEY.md 8(f) rows 1-2: fold-in of a new user, prediction, top-N
recommendation with exclusion and rotation, and the per-user ranking-agreement
evaluation.  Every function follows the reference line by line, including its
arithmetic order (Python float64, one multiply and one add per factor, no
fused multiply-add), so scores and agreements can be compared bit for bit.

Pinned by ``tests/golden/serving_*.npz``, which
``tests/golden/make_golden_serving.py`` produces by importing the reference's
own ``app_local/models.py`` (``ALS_Model``) and ``full_data/my_util.py``
(``compute_ranking_agreement``) in the build container.  ``recommend.py`` and
``worker_process.py`` cannot be imported without unpickling reference data
files at import time, so their short control flow is restated here and pinned
through the imported functions they call.
"""
import numpy as np


# --------------------------------------------------------------------------
# fold-in  (python/app_local/models.py:657-700, ALS_Model.__init__)
# --------------------------------------------------------------------------
def fold_in(num_factors, movie_ratings, als_movie_factors, als_movie_ids):
    """Least-squares user factors from ``[(movie_id, rating)]``.

    ``models.py:672``: fewer than k+1 ratings -> invalid.  ``:676-691``: one
    row ``[V_m, 1]`` per rated movie that has factors, right-hand side the RAW
    rating (the movie median is not subtracted -- a reference quirk kept
    as-is).  ``:694``: fewer than k+1 usable rows -> invalid.  ``:697``:
    ``numpy.linalg.lstsq(A, b, rcond=None)``.  Returns ``(valid, x)`` with x of
    length k+1 (k factors, then the user bias) or ``None``."""
    if len(movie_ratings) < num_factors + 1:
        return False, None
    A, b = [], []
    for movie_id, rating in movie_ratings:
        if movie_id in als_movie_ids:
            i = als_movie_ids[movie_id]
            row = list(als_movie_factors[num_factors * i: num_factors * i + num_factors])
            row.append(1)
            A.append(row)
            b.append(rating)
    if len(A) < num_factors + 1:
        return False, None
    return True, np.linalg.lstsq(A, b, rcond=None)[0]


# --------------------------------------------------------------------------
# predict  (app_local/models.py:708-733 == full_data/als_predictor.py:35-60)
# --------------------------------------------------------------------------
def predict(user_factors, movie_id, movie_medians, als_movie_factors, als_movie_ids):
    """``None`` unless the movie has both a median and factors (``:713-715``);
    otherwise ``sum_i u_i v_i`` accumulated left to right from 0, then
    ``+ u_k`` (bias), then ``+ median`` (``:725-731``)."""
    if movie_id not in movie_medians or movie_id not in als_movie_ids:
        return None
    k = len(user_factors) - 1
    j = als_movie_ids[movie_id]
    v = als_movie_factors[k * j: k * (j + 1)]
    rating = 0
    for i in range(k):
        rating += float(user_factors[i]) * float(v[i])
    rating += float(user_factors[k])
    rating += float(movie_medians[movie_id])
    return rating


# --------------------------------------------------------------------------
# top-N  (python/app_local/recommend.py:86-110, get_recommendations)
# --------------------------------------------------------------------------
def recommend(user_factors, user_ratings_dict, movie_medians, als_movie_factors,
              als_movie_ids, num_results=400):
    """Full recommendation list before rotation: score every movie of
    ``movie_medians`` (``:88-91``), ``predictions.sort(reverse=True)`` on
    ``(score, movie_id)`` tuples -- descending score, ties by descending
    movie id (``:93``) -- then the first ``num_results`` movies the user has
    not rated (``:97-106``).  Returns ``[(score, movie_id)]``."""
    preds = []
    for movie_id in movie_medians:
        s = predict(user_factors, movie_id, movie_medians, als_movie_factors, als_movie_ids)
        if s is not None:
            preds.append((s, movie_id))
    preds.sort(reverse=True)
    out = []
    for s, movie_id in preds:
        if movie_id not in user_ratings_dict:
            out.append((s, movie_id))
            if len(out) >= num_results:
                break
    return out


def rotation(movie_ids, r, rotation_size=4):
    """``recommendation[rotation::rotation_size]`` (``recommend.py:115`` for
    rotation 0, ``user_data.py:118-121`` for the later rotations)."""
    return list(movie_ids)[r::rotation_size]


# --------------------------------------------------------------------------
# ranking agreement  (python/full_data/my_util.py:56-145)
# --------------------------------------------------------------------------
def ratings_to_list_of_lists(movie_ratings):
    """``convert_ratings_to_list_of_list`` (``my_util.py:56-80``): movie ids
    grouped by rating, groups in descending rating order."""
    groups = {}
    for movie_id, rating in movie_ratings:
        groups.setdefault(rating, []).append(movie_id)
    return [groups[r] for r in sorted(groups, reverse=True)]


def has_different_ratings(movie_ratings, start):
    """``my_util.py:83-98``."""
    r1 = movie_ratings[start][1]
    return any(movie_ratings[i][1] != r1 for i in range(start + 1, len(movie_ratings)))


def ranking_agreement(actual_ratings, predicted_ratings):
    """``compute_ranking_agreement`` (``my_util.py:101-145``): over every pair
    (m1, m2) with actual(m1) > actual(m2), agreement when predicted(m1) >
    predicted(m2) strictly, else disagreement; ``None`` for a single rating
    or all-equal ratings.  Returns (value, agree, disagree) -- value is
    ``agree / (agree + disagree)`` as Python computes it."""
    if len(actual_ratings) == 1 or not has_different_ratings(actual_ratings, 0):
        return None, 0, 0
    groups = ratings_to_list_of_lists(actual_ratings)
    pred = dict(predicted_ratings)
    agree = disagree = 0
    for i in range(len(groups) - 1):
        for m1 in groups[i]:
            for j in range(i + 1, len(groups)):
                for m2 in groups[j]:
                    if pred[m1] > pred[m2]:
                        agree += 1
                    else:
                        disagree += 1
    return agree / (agree + disagree), agree, disagree


def ranking_agreement_counts(actual, predicted):
    """Vectorised equivalent of the pair loop (same counts), for the larger
    golden cases: pairs with actual_i > actual_j, agree when pred_i > pred_j."""
    a = np.asarray(actual, np.float64)
    p = np.asarray(predicted, np.float64)
    gt = a[:, None] > a[None, :]
    agree = int(np.count_nonzero(gt & (p[:, None] > p[None, :])))
    return agree, int(np.count_nonzero(gt)) - agree


# --------------------------------------------------------------------------
# evaluation  (python/full_data/worker_process.py:229-306)
# --------------------------------------------------------------------------
def test_model(predict_fn, movie_ratings):
    """``_test_model`` (``worker_process.py:229-257``): predictions for the
    test movies the model can score; agreement only when more than one."""
    predicted, kept = [], []
    for movie_id, actual in movie_ratings:
        p = predict_fn(movie_id)
        if p is not None:
            predicted.append((movie_id, p))
            kept.append((movie_id, actual))
    if len(predicted) > 1:
        return ranking_agreement(kept, predicted)[0]
    return None


def als_eval(user_ratings_test, movie_medians_train, als_user_factors, als_user_ids,
             als_movie_factors, als_movie_ids, num_item_factors):
    """``_als_eval`` (``worker_process.py:262-306``): for each
    ``(user_id, [(movie_id, rating)])`` the user's factor row
    ``U[(k+1)u : (k+1)(u+1)]`` scores its test movies; returns
    ``[(user_id, agreement)]`` for the users with a defined agreement."""
    K = num_item_factors + 1
    out = []
    for user_id, movie_ratings in user_ratings_test:
        u = als_user_ids[user_id]
        uf = als_user_factors[K * u: K * (u + 1)]
        a = test_model(lambda m: predict(uf, m, movie_medians_train, als_movie_factors,
                                         als_movie_ids), movie_ratings)
        if a is not None:
            out.append((user_id, a))
    return out
