/* Similar-movies database on the GPU.
 *
 * Reference: python/full_data/build_similar_movies_db.py:19-163
 * (SimilarMovieFinder: genre gate _genres_similar :41-66, co-rating cosine
 * with the common-reviewer boost _scaled_dot_product :69-112, per-movie
 * ranking find_similar_movie :138-163) run over every movie by
 * movie_lens_data_proc.py:657-700 (_find_similar_movies) /
 * build_similar_movies_db.py:255-291 (build_locally).
 *
 * Movies are indexed by their position in the reference's movie_ratings list
 * (the query order).  Ratings must be multiples of 0.5 (MovieLens): the
 * co-rating sums are then exact integers (in quarter units) and every score is
 * bit-identical to the reference's NumPy expression
 *   similarity = r1.dot(r2) / (norm(r1) * norm(r2));  score = similarity * (1.0 + buff(n))
 * with buff(n) supplied by the caller (host Python math, the reference's
 * formula), so the filters (n >= 3, score > 0.3), the truncation to the
 * num_results * 20 movies with most common reviewers and the final score
 * order match exactly.
 *
 * Returns 0 on success, -1 on failure (mr_last_error()).
 */
#ifndef MR_SIMILAR_H
#define MR_SIMILAR_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mr_similar mr_similar;

/* n_movies movies (query order); movie m's ratings are entries
 * off[m] .. off[m+1]-1 of (user, rating2) with user in [0, n_users) (dense
 * user index) and rating2 = 2 * rating (an integer, 0..255).
 * genre_mask[m]: bit g set when the movie has genre g (dense ids < 64);
 * has_genres[m] = 0 when the movie is not in movie_genres (never similar). */
mr_similar* mr_similar_create(int device, int n_movies, int n_users, const long long* off,
                              const int* user, const unsigned char* rating2,
                              const unsigned long long* genre_mask,
                              const unsigned char* has_genres);
void mr_similar_destroy(mr_similar* ctx);

/* find_similar_movie for the n_query movie indices in query[] (all movies
 * when query is NULL and n_query == n_movies): boost1[n] = 1.0 + buff(n) for
 * n = 0 .. n_boost-1 (n >= n_boost uses boost1[n_boost-1]); num_results
 * results per query (num_results * 20 <= 1024).  out_index / out_score:
 * [n_query * num_results] (similar movies' indices, best first);
 * out_count[q] = results for query q. */
int mr_similar_find(mr_similar* ctx, int n_query, const int* query, const double* boost1,
                    int n_boost, int num_results, int* out_index, double* out_score,
                    int* out_count);

/* Device milliseconds of the last mr_similar_find. */
double mr_similar_last_ms(const mr_similar* ctx);

#ifdef __cplusplus
}
#endif
#endif
