/*
 * mr_cg.h -- device-resident general sparse least squares (CG on A^T A x =
 * A^T b) for MI355X (gfx950).
 *
 * The reference exposes this solver as cg_least_squares_from_python /
 * cg_least_squares2_from_python (cpp/ls_lib/ls_linux_dll.cpp:28-77 ->
 * cg_least_squares, cpp/ls_lib/matrix.cpp:456-529), building its matrices
 * and scratch per call.  A context here uploads A once, builds its explicit
 * transpose on the device, and solves any number of right-hand sides with
 * every CG step on the GPU (3 kernels per CG iteration, no host round trip);
 * the two reference symbols (cpp_ls_lib.h) are create + solve + destroy.
 */
#ifndef MR_CG_H
#define MR_CG_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mr_cg mr_cg;

/* Kernel classes timed with HIP events when timing is enabled. */
enum {
  MR_CG_K_SPMV_A = 0,    /* t = A p (p = -r + beta p formed at the gather)       */
  MR_CG_K_SPMV_AT,       /* q = A^T t, p update, p.q partials, alpha              */
  MR_CG_K_UPDATE,        /* x += alpha p, r += alpha q, r.r, BETA rule + publish  */
  MR_CG_K_SETUP,         /* b2 = A^T b, A^T A x, the INIT update (per solve)      */
  MR_CG_K_COUNT
};

typedef struct mr_cg_stats {
  int last_iterations;            /* CG iterations of the last solve              */
  long long iterations_total;     /* over all solves since the last reset         */
  double solve_ms;                /* device time of the solves (setup .. stop)    */
  double kernel_ms[MR_CG_K_COUNT];
  long long kernel_launches[MR_CG_K_COUNT];  /* launches that did work           */
  long long rows, cols, nnz;
  long long blocks_a, blocks_at;  /* CSR-stream row blocks of A and of A^T        */
  long long block_max_nnz;        /* a row block's non-zero limit (longer rows:   */
                                  /* a block of their own)                        */
  long long block_max_rows;       /* a row block's row limit                      */
} mr_cg_stats;

/* A in the reference's CSR form: row_indices[rows+1] (int32, starting at 0,
 * non-decreasing), col_indices / values [row_indices[rows]].  Checked on the
 * host (column range, monotone rows); NULL on error (mr_last_error). */
mr_cg* mr_cg_create(int device, int rows, int cols, const int* row_indices,
                    const int* col_indices, const double* values);
void mr_cg_destroy(mr_cg* ctx);

/* cg_least_squares semantics (matrix.cpp:456-529): b[rows] read-only, x[cols]
 * in/out (the caller's start), stop when rr < 1e-6 at the loop top, after
 * two consecutive beta > 1 - min_r_decrease, or max_iteration; *final_rr (may
 * be NULL) = the last rr.  Returns the CG iteration count, < 0 on error. */
int mr_cg_solve(mr_cg* ctx, const double* b, double* x, double min_r_decrease,
                int max_iteration, double* final_rr);

int mr_cg_set_timing(mr_cg* ctx, int enable);
int mr_cg_get_stats(mr_cg* ctx, mr_cg_stats* out);
int mr_cg_reset_stats(mr_cg* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MR_CG_H */
