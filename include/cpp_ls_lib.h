/*
 * cpp_ls_lib.h -- drop-in C ABI of the reference CPU library, served by the
 * MI355X (gfx950) HIP implementation in movie_recommender_amd/lib/cpp_ls_lib.so.
 *
 * Each entry point replaces the symbol of the same name exported by the
 * reference `cpp_ls_lib.so` (louisyang2015/movie_recommender,
 * cpp/ls_lib/ls_linux_dll.cpp) and keeps its argument meaning, in/out
 * conventions and success-path return values.  Callers: the reference ctypes
 * wrapper cpp/python/cpp_ls.py and this repo's movie_recommender_amd.cpp_ls.
 *
 * Differences (documented in INTEGRATION.md):
 *   - failures return a negative value and log to stderr (the reference throws
 *     across extern "C" -> std::terminate, matrix.cpp:403-405, 422-424);
 *   - arithmetic runs on the GPU: ALS normal equations and factors in fp32,
 *     CG vectors, products and scalars in fp64; the general CG least squares
 *     in fp64;
 *   - no caller pointer is retained after return.
 */
#ifndef MR_CPP_LS_LIB_H
#define MR_CPP_LS_LIB_H

#ifdef __cplusplus
extern "C" {
#endif

/* Replaces ls_linux_dll.cpp:8-11.  Stores any int verbatim (cpp_ls.py:23-36
 * round-trips a random 1..100000); it does not size GPU work. */
void set_thread_count(int thread_count);

/* Replaces ls_linux_dll.cpp:13-16. */
int get_thread_count(void);

/* Replaces ls_linux_dll.cpp:28-50 (cg_least_squares, matrix.cpp:456-529).
 * Solves A x = b in the least-squares sense by CG on A^T A x = A^T b.
 * A: CSR, A_row_indices[A_rows+1], A_col_indices/A_values[nnz].
 * x (length x_length == A_cols) is in/out: caller-initialised warm start.
 * Returns the CG iteration count; writes *final_rr when non-null.  <0 on error. */
int cg_least_squares_from_python(int A_rows, int A_cols, int* A_row_indices,
                                 int* A_col_indices, double* A_values,
                                 int b_length, double* b_values,
                                 int x_length, double* x_values,
                                 double min_r_decrease, int max_iteration,
                                 double* final_rr);

/* Replaces ls_linux_dll.cpp:54-77 (cg_least_squares2, matrix.cpp:536-613):
 * the explicit-transpose variant.  Same math and return values; on the GPU
 * both variants use an explicit device-side transpose. */
int cg_least_squares2_from_python(int A_rows, int A_cols, int* A_row_indices,
                                  int* A_col_indices, double* A_values,
                                  int b_length, double* b_values,
                                  int x_length, double* x_values,
                                  double min_r_decrease, int max_iteration,
                                  double* final_rr);

/* Replaces ls_linux_dll.cpp:81-103 (als, matrix.cpp:744-893).
 * user_ids/item_ids: zero-based int32[ratings_length]; ratings: fp64.
 * user_factors: in/out, user_factors_length = num_users*(k+1), row u =
 *   [k factors, bias]; item_factors: in/out, item_factors_length = num_items*k.
 * Returns the ALS iteration index at exit (matrix.cpp:874, 892).
 * `algorithm` is accepted for ABI compatibility (1 and 2 are the same math). */
int als_from_python(int* user_ids, int* item_ids, int ratings_length,
                    double* ratings_values, int num_item_factors,
                    int user_factors_length, double* user_factors_values,
                    int item_factors_length, double* item_factors_values,
                    double min_r_decrease, int max_iteration, int algorithm);

#ifdef __cplusplus
}
#endif
#endif /* MR_CPP_LS_LIB_H */
