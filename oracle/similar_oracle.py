"""Pure-Python restatement of the reference's similar-movies search -- TEST
INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Follows ``python/full_data/build_similar_movies_db.py:41-163``
(``SimilarMovieFinder``) and ``movie_lens_data_proc.py:657-700``
(``_find_similar_movies``).  Pinned by ``tests/golden/similar_*.npz``, made by
``tests/golden/make_golden_similar.py`` with the reference's own
``SimilarMovieFinder`` class.
"""
import math

import numpy


def genres_similar(movie_genres, m1, m2):
    """``_genres_similar`` (``:41-66``)."""
    if m1 not in movie_genres or m2 not in movie_genres:
        return False
    g1, g2 = movie_genres[m1], movie_genres[m2]
    if len(g1) > len(g2):
        g1, g2 = g2, g1
    matches = sum(1 for g in g1 if g in g2)
    return matches / len(g1) >= 0.5


def scaled_dot_product(movie_ratings, i1, i2, buff_limit, buff_point):
    """``_scaled_dot_product`` (``:69-112``)."""
    ratings1, ratings2 = movie_ratings[i1][1], movie_ratings[i2][1]
    if len(ratings1) > len(ratings2):
        ratings1, ratings2 = ratings2, ratings1
    r1, r2 = [], []
    for u in ratings1:
        if u in ratings2:
            r1.append(ratings1[u])
            r2.append(ratings2[u])
    if len(r1) < 3:
        return 0.0, len(r1), 0.0
    r1, r2 = numpy.array(r1), numpy.array(r2)
    similarity = r1.dot(r2) / (numpy.linalg.norm(r1) * numpy.linalg.norm(r2))
    n = len(r1)
    x_limit = 3 * math.exp(buff_limit)
    x = 3 + (x_limit - 3) * (n - 3) / (buff_point - 3)
    buff = math.log(x) - math.log(3)
    if buff > buff_limit:
        buff = buff_limit
    if buff < 0:
        buff = 0
    return similarity * (1.0 + buff), n, similarity


def find_similar_movie(movie_genres, movie_ratings, index, buff_limit, buff_point,
                       num_results=20):
    """``find_similar_movie`` (``:138-163``)."""
    sim = []
    for j in range(len(movie_ratings)):
        if j == index:
            continue
        if not genres_similar(movie_genres, movie_ratings[index][0], movie_ratings[j][0]):
            continue
        score, n, _ = scaled_dot_product(movie_ratings, index, j, buff_limit, buff_point)
        if score > 0.3:
            sim.append((movie_ratings[j][0], score, n))
    if len(sim) > num_results * 20:
        sim.sort(key=lambda e: e[2], reverse=True)
        sim = sim[:num_results * 20]
    sim.sort(key=lambda e: e[1], reverse=True)
    if sim:
        ids, scores, _ = zip(*sim)
        return ids[:num_results], scores[:num_results]
    return [], []
