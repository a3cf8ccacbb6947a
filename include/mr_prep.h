/* ALS training-set preparation on the GPU.
 *
 * Reference (Python, multiprocess over lists of (movie_id, rating) tuples):
 *   medians   python/full_data/movie_lens_data_proc.py:393-471
 *             (_extract_movie_ratings, _compute_medians: numpy.median of
 *             every movie's training ratings)
 *   shrink    python/full_data/movie_lens_data.py:564-591
 *             (als_data_set_shrink_mp: drop users with < k+1 ratings, then
 *             movies with < k ratings, until nothing changes;
 *             movie_lens_data_proc.py:494-586 _drop_users / _count_movies /
 *             _drop_movies)
 *   ids       movie_lens_data.py:593-612 + movie_lens_data_proc.py:589-608
 *             (_collect_ids: sets merged across processes, zero-based ids
 *             in set iteration order -- reproduced by the Python mirror
 *             movie_recommender_amd/prep.py from the first-appearance lists
 *             computed here)
 *   convert   movie_lens_data_proc.py:611-654 (_convert_training_data_to_numpy:
 *             zero-based ids, rating - median, in traversal order)
 *
 * Input ratings are the reference's user_ratings_train flattened in traversal
 * order (users in list order, each user's ratings in list order); user and
 * movie ids are the standard (MovieLens) ids, >= 0.  Every result is exact
 * (integer work and the correctly rounded fp64 median / subtraction).
 * Functions return 0 on success, -1 on failure (mr_last_error()).
 */
#ifndef MR_PREP_H
#define MR_PREP_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mr_prep mr_prep;

mr_prep* mr_prep_create(int device, long long n, const int* user_id, const int* movie_id,
                        const double* rating);
void mr_prep_destroy(mr_prep* ctx);

/* Largest user / movie id + 1 (sizes of the dense per-id output arrays). */
int mr_prep_id_bounds(const mr_prep* ctx, int* user_bound, int* movie_bound);

/* numpy.median of each movie's ratings over ALL input ratings:
 * median[m] for m < movie_bound (NaN for ids without ratings). */
int mr_prep_medians(mr_prep* ctx, double* median);

/* Shrink for factor k.  restart = 1 starts from all input ratings; 0
 * continues from the previous call's survivors, as the reference does when it
 * walks factors_list over lists it has already shrunk in place
 * (movie_lens_data.py:568).  keep[i] = 1 when rating i survives (may be
 * NULL); *rounds = passes of the reference's while loop; *n_kept / *n_users /
 * *n_movies = surviving ratings / users / movies. */
int mr_prep_shrink(mr_prep* ctx, int k, int restart, unsigned char* keep, int* rounds,
                   long long* n_kept, int* n_users, int* n_movies);

/* For each of n_chunks rating ranges [chunk_begin[c], chunk_begin[c+1]) of
 * the last shrink's survivors: the first surviving index of every user and
 * movie id in the chunk (INT64 max when absent).  first_user:
 * [n_chunks * user_bound], first_movie: [n_chunks * movie_bound]. */
int mr_prep_first_appearance(mr_prep* ctx, int n_chunks, const long long* chunk_begin,
                             long long* first_user, long long* first_movie);

/* Compacted training arrays of the last shrink, in input order:
 * out_user[j] = user_map[user], out_movie[j] = movie_map[movie],
 * out_rating[j] = rating - median[movie] (median: per movie id, as returned
 * by mr_prep_medians or any caller table).  Arrays hold *n_kept entries. */
int mr_prep_convert(mr_prep* ctx, const int* user_map, const int* movie_map,
                    const double* median, int* out_user, int* out_movie, double* out_rating);

/* Device milliseconds of the last call (HIP events on the context stream,
 * from its first upload or kernel to its last kernel; result copies to the
 * host are not included). */
double mr_prep_last_ms(const mr_prep* ctx);

#ifdef __cplusplus
}
#endif
#endif
