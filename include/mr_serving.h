/* Factor consumers on the GPU: fold-in, prediction, top-N recommendation and
 * the ranking-agreement evaluation.
 *
 * The reference implements these in Python over NumPy factor arrays:
 *   fold-in      python/app_local/models.py:657-700   (ALS_Model.__init__)
 *   predict      python/app_local/models.py:708-733,
 *                python/full_data/als_predictor.py:35-60
 *   top-N        python/app_local/recommend.py:86-110 (get_recommendations)
 *   evaluation   python/full_data/worker_process.py:229-306
 *                (_test_model, _als_eval) + my_util.py:101-145
 *                (compute_ranking_agreement)
 * The Python mirror of those interfaces is movie_recommender_amd/serving.py;
 * this header is the C ABI it binds (exported by cpp_ls_lib.so).
 *
 * Numerics: scores are computed in fp64 in the reference's order
 * (sum_i u_i * v_i from 0, then + bias, then + median; separate multiply and
 * add, no FMA), so they are bit-identical to the reference's, and the
 * (score, movie id) ordering, exclusions and agreement counts are exact.
 * Fold-in solves the normal equations of lstsq([V, 1], r) in fp64
 * (Cholesky); ill-conditioned or rank-deficient systems switch to a one-sided
 * Jacobi SVD with numpy's lstsq cut-off (eps * max(M, K) * s_max).
 *
 * All functions return 0 on success and -1 on failure (message via
 * mr_last_error(), declared in mr_als.h).  Buffers are caller-owned host
 * memory; nothing is retained after a call returns.
 */
#ifndef MR_SERVING_H
#define MR_SERVING_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mr_rec mr_rec;

/* Movie table on device `device`.
 *   als_movie_factors  f64[n_als * k], row j = movie with zero-based ALS id j
 *                      (the reference's als{k}_item_factors array)
 *   candidates         the movies predict() can score: a median AND factors
 *                      (models.py:713-715), in movie_medians iteration order:
 *                      cand_als[c] = ALS id, cand_mid[c] = standard movie id
 *                      (unique, >= 0), cand_med[c] = the movie's median. */
mr_rec* mr_rec_create(int device, int k, int n_als, const double* als_movie_factors,
                      int n_cand, const int* cand_als, const int* cand_mid,
                      const double* cand_med);
void mr_rec_destroy(mr_rec* ctx);
int mr_rec_num_candidates(const mr_rec* ctx);

/* Fold-in of n_users rating lists (models.py:676-697): user u's rows are
 * off[u] .. off[u+1]-1, each an ALS movie id and the RAW rating (median not
 * subtracted, as in the reference).  The caller applies the reference's
 * validity rules (models.py:672, :694) and passes only users with at least
 * k+1 rows.  x_out: f64[n_users * (k+1)] (k factors, then the bias);
 * method_out (optional): 1 = Cholesky, 2 = Jacobi SVD. */
int mr_rec_fold_in(mr_rec* ctx, int n_users, const long long* off, const int* als_idx,
                   const double* ratings, double* x_out, int* method_out);

/* predict() of every candidate for each user row x[u*(k+1) ..]:
 * out[u * n_cand + c] (models.py:725-731 arithmetic). */
int mr_rec_scores(mr_rec* ctx, int n_users, const double* x, double* out);

/* Top-N (recommend.py:86-106): candidates sorted by (score, movie id)
 * descending, skipping user u's excluded candidates
 * excl_cand[excl_off[u] .. excl_off[u+1]-1] (the movies the user rated;
 * excl_off may be NULL), first num_results (1 .. 1024) kept.
 * out_mid / out_score: [n_users * num_results]; out_count[u] = entries
 * written for user u (fewer when fewer candidates remain). */
int mr_rec_top_n(mr_rec* ctx, int n_users, const double* x, const long long* excl_off,
                 const int* excl_cand, int num_results, int* out_mid, double* out_score,
                 int* out_count);

/* Evaluation (worker_process.py:262-306): test user t uses factor row
 * U[user_row[t] * (k+1) ..] of the table U (f64[n_rows * (k+1)]) and scores
 * its test ratings off[t] .. off[t+1]-1 (cand[i] = candidate index of the
 * movie, or -1 when predict() returns None; actual[i] = held-out rating).
 * agreement[t] = compute_ranking_agreement of the scorable ratings, NaN when
 * the reference returns None; n_agree / n_disagree = its pair counts.
 * pred (optional): the prediction of every test rating (NaN for -1).
 * sse / n_pred (optional): [n_test] -- per test user, the sum over its
 * scorable ratings of (pred - actual)^2 and their number (the held-out RMSE
 * the reference does not report is sqrt(sum sse / sum n_pred)). */
int mr_rec_evaluate(mr_rec* ctx, int n_rows, const double* U, int n_test,
                    const int* user_row, const long long* off, const int* cand,
                    const double* actual, double* agreement, long long* n_agree,
                    long long* n_disagree, double* pred, double* sse, long long* n_pred);

/* compute_ranking_agreement (my_util.py:101-145) for n_users lists given as
 * aligned (actual, predicted) ratings: user u owns entries off[u] ..
 * off[u+1]-1; a NaN prediction drops the entry (predict() returned None).
 * agreement[u] is NaN where the reference returns None.  Needs no table. */
int mr_rank_agreement(int device, int n_users, const long long* off, const double* actual,
                      const double* predicted, double* agreement, long long* n_agree,
                      long long* n_disagree);

/* Kernel time of the last call, milliseconds, per class (HIP events on the
 * context stream): [0] scores, [1] exclusion, [2] top-N select,
 * [3] fold-in Gram + Cholesky, [4] fold-in SVD, [5] evaluation. */
int mr_rec_last_kernel_ms(const mr_rec* ctx, double* ms6);

#ifdef __cplusplus
}
#endif
#endif
