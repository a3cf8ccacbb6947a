/*
 * mr_als.h -- device-resident ALS engine for MI355X (gfx950).
 *
 * Richer native API beside the reference ABI of cpp_ls_lib.h (SURVEY.md
 * section 8(b), "Richer native API").  A context keeps the ratings (by-user
 * CSR and by-item CSR), both factor tables and every solver buffer resident
 * in HBM across iterations; only factors cross PCIe, on request.
 *
 * The hot path is one ALS iteration of the reference's als()
 * (cpp/ls_lib/matrix.cpp:814-890): user half-step (normal equations from
 * gathered item-factor rows, then the solve) and item half-step (the same with
 * user-factor rows and ratings minus user bias).
 *
 * Solvers:
 *   MR_SOLVER_CG        reference-faithful: one global conjugate-gradient run
 *                       per half-step over the block-diagonal A^T A with the
 *                       reference's scalars and stop rules (matrix.cpp:456-529)
 *   MR_SOLVER_CHOLESKY  exact per-entity solve (G_e + ridge I) x_e = c_e
 *
 * Sharding (multi-GPU, one process per GPU): a context may own a contiguous
 * range of users and of items (mr_als_create_shard); factor tables stay
 * replicated, and the freshly solved shard is exchanged between half-steps
 * (all-gather of equal, padded shards) and the two CG scalars per CG
 * iteration all-reduced -- natively over RCCL (mr_als_set_rccl) or through
 * the mr_comm callbacks.
 */
#ifndef MR_ALS_H
#define MR_ALS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mr_als mr_als;

enum { MR_SOLVER_CG = 0, MR_SOLVER_CHOLESKY = 1 };
enum { MR_SIDE_USERS = 0, MR_SIDE_ITEMS = 1 };

/* Kernel classes timed with HIP events when timing is enabled. */
enum {
  MR_K_GRAM_USERS = 0,   /* normal equations, user side (MFMA gather-Gram)   */
  MR_K_GRAM_ITEMS,       /* normal equations, item side                       */
  MR_K_SLAB_REDUCE,      /* combine partial normal equations of split entities */
  MR_K_MATVEC_USERS,     /* CG batched block GEMV, user side                  */
  MR_K_MATVEC_ITEMS,     /* CG batched block GEMV, item side                  */
  MR_K_CG_UPDATE,        /* CG x/r update + r.r partials (both sides)         */
  MR_K_CG_CONTROL,       /* CG scalar reduction / stop rule (both sides)      */
  MR_K_SOLVE,            /* batched Cholesky (exact mode)                      */
  MR_K_CG_START,         /* CG start of split entities (fused start)          */
  MR_K_CG_RES_USERS,     /* resident CG solve (all iterations), user side     */
  MR_K_CG_RES_ITEMS,     /* resident CG solve, item side                      */
  MR_K_EXCHANGE,         /* sharded: factor all-gather of a half-step (pack,
                            collective, unstage)                             */
  MR_K_COUNT
};

typedef struct mr_stats {
  int iterations;                 /* ALS iterations executed                  */
  int last_cg_users, last_cg_items;   /* CG iterations of the last half-steps */
  long long cg_users_total, cg_items_total;
  double last_final_rr;           /* item-side final rr of the last iteration */
  long long nonpd_users, nonpd_items; /* exact mode: blocks left unsolved     */
  double kernel_ms[MR_K_COUNT];   /* summed HIP-event time per kernel class   */
  long long kernel_launches[MR_K_COUNT]; /* timed (non-idle) launches        */
  double phase_ms[4];             /* gram users, solve users, gram items, solve items */
  long long kernel_units[MR_K_COUNT];   /* work units of the timed launches: CG
                                           iterations for the resident solves,
                                           launches for every other class   */
  double peer_wait_ms;            /* device time the finalizing waves spent in the
                                     peer all-reduce (sharded, peer scalars)  */
  long long peer_reductions;      /* peer all-reduces done                    */
} mr_stats;

/* Collective callbacks for sharded runs (one process per GPU).  The engine
 * stages the exchanged data through pinned host memory and calls:
 *   allreduce_f64(user, buf, count)   in-place sum over ranks of `count`
 *                                     doubles (the CG scalars p.Ap, r.r)
 *   allgather_rows(user, table, row_floats, row_begin, world)
 *                                     in-place all-gather of a row table:
 *                                     rank r owns rows [row_begin[r],
 *                                     row_begin[r+1]) of width row_floats
 *                                     (the engine passes its packed
 *                                     exchange buffer: ONE "row" per rank,
 *                                     row_floats = ag_block_floats(maxrows,
 *                                     ldk, with_bias) floats wide -- the
 *                                     rank's padded factor rows followed by
 *                                     its biases padded to 4 -- and
 *                                     row_begin[r] = r)
 * Both return 0 on success. */
typedef struct mr_comm {
  void* user;
  int rank, world;
  int (*allreduce_f64)(void* user, double* host_buf, int count);
  int (*allgather_rows)(void* user, float* host_table, long long row_floats,
                        const long long* row_begin, int world);
} mr_comm;

/* Context from host COO ratings (zero-based ids).  Builds the by-user and
 * by-item CSR on the device.  k <= 512 (k > 128 runs the streamed large-k
 * kernels; the exact solver needs k <= 128).  NULL on error (mr_last_error). */
mr_als* mr_als_create(int device, int k, int num_users, int num_items,
                      long long n_ratings, const int* user_ids,
                      const int* item_ids, const double* ratings);

/* Sharded context: this rank solves users [u_begin,u_end) and items
 * [i_begin,i_end).  The user view holds every rating of the rank's users,
 * the item view every rating of its items (global ids).  Factor tables stay
 * replicated (full U x (k+1) and I x k). */
mr_als* mr_als_create_shard(int device, int k, int num_users, int num_items,
                            long long n_user_view, const int* uv_user_ids,
                            const int* uv_item_ids, const double* uv_ratings,
                            long long n_item_view, const int* iv_user_ids,
                            const int* iv_item_ids, const double* iv_ratings,
                            int u_begin, int u_end, int i_begin, int i_end);

/* Attach collectives: user_begin/item_begin hold world+1 shard boundaries. */
int mr_als_set_comm(mr_als* ctx, const mr_comm* comm,
                    const long long* user_begin, const long long* item_begin);

/* Native RCCL collectives (over xGMI) instead of callbacks: rank 0 creates
 * an id with mr_rccl_unique_id and every rank passes the same 128 bytes.
 * All ranks must call mr_als_set_rccl concurrently (it builds the RCCL
 * communicator).  The CG scalars are then all-reduced on the device stream
 * and the factor shards exchanged by one all-gather of equal, padded shards
 * per half-step. */
int mr_rccl_unique_id(unsigned char out[128]);
int mr_als_set_rccl(mr_als* ctx, const unsigned char id[128], int rank, int world,
                    const long long* user_begin, const long long* item_begin);

/* Peer all-reduce of the CG scalars (sharded runs, any transport): instead
 * of an all-reduce launch per scalar, the thread that finalizes each CG
 * reduction writes its sum into every rank's exchange buffer (IPC-mapped
 * device memory; over xGMI between GPUs), waits for all ranks' records and
 * sums them in rank order -- identical bits on every rank, and the CG then
 * runs the single-GPU launch sequence (2 kernels per iteration).  Each rank:
 * mr_als_peer_handle (64 bytes), exchange them (rank order), then
 * mr_als_set_peer with the world x 64 bytes.  Reference scalars:
 * matrix.cpp:485, 497, 507.  A peer that does not arrive within
 * MR_OPT_PEER_TIMEOUT_S (default 30 s) fails the solve (< 0) instead of
 * hanging.  mr_als_set_peer runs once per context (a second call is
 * refused: the exchange buffers' sequence numbers are not reset); with
 * world = 0 (handles may be NULL) it switches back to the collective scalars
 * for good.  mr_als_peer_selftest (all ranks together) runs one reduction of
 * {rank + 1, 1} and checks the sums. */
int mr_als_peer_handle(mr_als* ctx, unsigned char out[64]);
int mr_als_set_peer(mr_als* ctx, const unsigned char* handles, int rank, int world);
int mr_als_peer_selftest(mr_als* ctx);
/* The user-side Gram's rhs path on the matrix cores needs every weight exact
 * in bf16 (checked per context on its own ratings).  A sharded run must take
 * one path on every rank: force < 0 returns this context's flag (0 / 1),
 * force = 0 clears it (the ranks AND their flags; distributed.py does). */
int mr_als_weights_bf16(mr_als* ctx, int force);
/* Latency probe of the peer all-reduce (collective, same iters on every
 * rank): `iters` reductions of one double back to back by one device thread;
 * *us = mean microseconds per reduction (HIP events around the kernel). */
int mr_als_peer_latency(mr_als* ctx, int iters, double* us);

void mr_als_destroy(mr_als* ctx);

/* Factor tables in the reference layout: U[num_users*(k+1)] (row = k factors,
 * bias), V[num_items*k]; fp64 on the host, fp32 on the device. */
int mr_als_set_factors(mr_als* ctx, const double* U, const double* V);
int mr_als_get_factors(mr_als* ctx, double* U, double* V);
/* Seeded uniform(-1, 1) initial factors generated on the device (the same
 * values on every rank of a sharded run; not the reference's NumPy RNG
 * stream).  For workloads whose host tables would be multi-GB (C5). */
int mr_als_init_factors(mr_als* ctx, unsigned long long seed);

int mr_als_set_solver(mr_als* ctx, int solver, double ridge);
/* Timing of every kernel launch with HIP events (off by default). */
int mr_als_set_timing(mr_als* ctx, int enable);
/* Engine options (mr_als_set_option; in a sharded run every rank must set
 * the same values -- they decide which launches and collectives are issued):
 *   MR_OPT_FUSE_START     1 (default): the Gram kernel also starts the CG solve
 *                         (r0, p0, q0 = G p0 from its accumulators); 0: the
 *                         reference's order, one matvec + update pass
 *   MR_OPT_CG_SPECULATE   0, 1 or 2 (others are rejected).
 *                         1 (default): enqueue CG iteration t+1 before t's
 *                         state is read back when t provably cannot stop
 *                         (decided on exact per-iteration states: identical
 *                         launches on every rank); 0: one iteration ahead;
 *                         2: always two ahead (an iteration launched after
 *                         the solve stopped exits at once: results identical)
 *   MR_OPT_WAIT_TIMEOUT_S host wait for a published CG state, seconds
 *                         (default 300; a stalled peer rank then fails the
 *                         call instead of hanging it)
 *   MR_OPT_CG_ONEPASS     1 (default): one kernel per CG iteration (the
 *                         previous iteration's x / r update deferred into
 *                         the next matvec, r'.r' from r.r, r.q, q.q; k <= 128,
 *                         unsharded or peer scalars); 0: matvec + update
 *   MR_OPT_GRAM_RHS_MFMA  1 (default): the user-side Gram at 64 < k <= 128
 *                         takes its rhs and row sums on the matrix cores when
 *                         every user-view rating is exact in bf16 (half-star
 *                         ratings, rating - median: always; measured -4 % at
 *                         k = 128, level at k = 64, where the VALU path
 *                         stays); 0: always on the VALU (fp32, rating order)
 *   MR_OPT_CG_SWEEP       sweep direction of the one-pass CG kernel over the
 *                         entity chunks: 1 (default) alternates, the first
 *                         iteration after the start backwards (it starts on
 *                         the lines the previous pass left in the Infinity
 *                         Cache); 2 alternates the other way; 0 always
 *                         forwards.  Results are identical in every mode (each
 *                         chunk's partial sums are order-independent terms)
 *   MR_OPT_PEER_TIMEOUT_S device wait for a peer rank's record in the peer
 *                         all-reduce, seconds (default 30, at most 1e5); on
 *                         expiry the solve ends with an error (< 0)
 *   MR_OPT_CG_TILE_NT     cache policy of the one-pass kernel's normal-
 *                         equation loads: -1 (default) by size -- non-
 *                         temporal when a side's per-iteration stream exceeds
 *                         320 MiB, else the default policy (a shard's side
 *                         can stay in the Infinity Cache between sweeps);
 *                         0 always default; 1 always non-temporal.  Results
 *                         are identical in every mode
 *   MR_OPT_CG_RESIDENT    1 (default): a one-pass solve runs ALL its CG
 *                         iterations in one resident launch (every block of
 *                         the grid on the chip at once, a per-iteration
 *                         broadcast instead of a kernel boundary; the host
 *                         waits once per solve); 0: one launch per
 *                         iteration.  Results are identical.  Ranks that
 *                         share one GPU must set 0 (their resident grids
 *                         would wait on each other): distributed.py does */
enum { MR_OPT_FUSE_START = 0, MR_OPT_CG_SPECULATE = 1, MR_OPT_WAIT_TIMEOUT_S = 2,
       MR_OPT_CG_ONEPASS = 3, MR_OPT_GRAM_RHS_MFMA = 4, MR_OPT_CG_SWEEP = 5,
       MR_OPT_PEER_TIMEOUT_S = 6, MR_OPT_CG_TILE_NT = 7, MR_OPT_CG_RESIDENT = 8 };
int mr_als_set_option(mr_als* ctx, int option, double value);
/* Ratings per Gram work item: heavier entities are split across waves and
 * their partial normal equations combined in order.  Applies to contexts
 * created afterwards (default 2048). */
int mr_set_gram_chunk(int chunk);

/* The reference loop (matrix.cpp:814-892): returns the iteration index at
 * exit, exactly as als_from_python.  <0 on error. */
int mr_als_run(mr_als* ctx, double min_r_decrease, int max_iteration);
/* Exactly n ALS iterations (no outer stop test).  0 on success. */
int mr_als_iterate(mr_als* ctx, int n);
/* One half-step: side MR_SIDE_USERS or MR_SIDE_ITEMS.  Returns the CG
 * iteration count (CG mode) or 0; *final_rr may be NULL. */
int mr_als_half_step(mr_als* ctx, int side, double* final_rr);

/* The same with the CG arguments of cg_least_squares (matrix.cpp:456):
 * min_r_decrease and max_iteration (max_iteration 0: only r0, rr = r0.r0). */
int mr_als_half_step_ex(mr_als* ctx, int side, double min_r_decrease, int max_iteration,
                        double* final_rr);

/* Build (only) the normal equations of one side from the current factors. */
int mr_als_build_normal_equations(mr_als* ctx, int side);
/* Copy the normal equations of n local entities of `side` (as last built):
 * G_out[n*K*K], c_out[n*K], K = k+1 for users (bias row/column last), k for
 * items.  For checking the Gram kernel at any problem size. */
int mr_als_get_normal_equations(mr_als* ctx, int side, int n, const int* entities,
                                double* G_out, double* c_out);

/* The CG vectors r, p, q (fp64, E*K each; K = k+1 per user with the bias
 * entry last, k per item) of the side's last solve; any may be NULL.  Tests. */
int mr_als_get_cg_vectors(mr_als* ctx, int side, double* r, double* p, double* q);

/* The side's device CSR (off[E+1], idx[nnz] = other side's id, val[nnz] as
 * fp32) and its Gram work list (n = mr_als_work_items entries, heavy first:
 * rating range [begin, begin+len) of local entity `entity`, slab >= 0 for a
 * chunk of a split entity).  Any pointer may be NULL.  Tests. */
long long mr_als_work_items(mr_als* ctx, int side);
/* Grid (workgroups) of a side's CG iteration kernels as launched: kind 0 the
 * one-pass kernel, 1 the resident solve (0: not available); nt 0 / 1 the
 * default-policy / non-temporal tile-load instantiation. */
int mr_als_cg_grid(mr_als* ctx, int side, int kind, int nt);
/* This context's entities of `side`: the first global id, how many (a shard
 * owns a contiguous range) and the ratings its CSR holds.  Any may be NULL. */
int mr_als_local_size(mr_als* ctx, int side, long long* first, long long* count,
                      long long* nnz);
int mr_als_get_layout(mr_als* ctx, int side, long long* off, int* idx, float* val,
                      long long* wbegin, int* wlen, int* went, int* wslab);

int mr_als_get_stats(mr_als* ctx, mr_stats* out);
int mr_als_reset_stats(mr_als* ctx);
/* Waits for all work queued on the context's stream. */
int mr_als_sync(mr_als* ctx);
/* The context's HIP stream (hipStream_t) for callers that enqueue around it. */
void* mr_als_stream(mr_als* ctx);

/* Sizes/counters for reporting: N (ratings held), U, I, k. */
long long mr_als_num_ratings(mr_als* ctx);

/* Device-side pointers of the fp32 factor tables (row stride ldk floats,
 * ldk = k rounded up to 16): Ufac[U*ldk], Ubias[U], Vfac[I*ldk]. */
int mr_als_device_tables(mr_als* ctx, float** Ufac, float** Ubias,
                         float** Vfac, int* ldk);

/* Predictions u[:k].v + u[k] for n (user,item) pairs, on the device. */
int mr_als_predict(mr_als* ctx, long long n, const int* user_ids,
                   const int* item_ids, double* out);

/* Test hooks: the sharded all-gather staging kernels on host arrays (the
 * engine runs them on its padded exchange buffers, Engine::allgather_side).
 *   pack:    send[n*ldk] = fac rows [r0, r0+n) of a rows x ldk table
 *            (+ send_b[n] = bias[r0 ..]; bias may be NULL)
 *   unstage: for every rank s != skip, rows j < rb[s+1]-rb[s] of block s of
 *            recv (world x maxrows x ldk) go to fac row rb[s]+j (+ bias from
 *            recv_b[s*maxrows + j]); fac / bias (rb[world] rows) are in/out.
 * ldk must be a multiple of 4; shapes are checked on the host first. */
int mr_test_pack_rows(int device, long long rows, int ldk, const float* fac, const float* bias,
                      long long r0, long long n, float* send, float* send_b);
/* Test hook: the one-pass CG's order-independent sum (an exact integer sum of
 * the terms truncated to multiples of 2^-192, converted to fp64) of n terms
 * dealt to the waves of `blocks` blocks; *out = the sum (NaN if a term is not
 * finite or >= 2^96 in magnitude). */
int mr_test_xsum(int device, const double* terms, long long n, int blocks, double* out);
int mr_test_unstage_rows(int device, int world, int skip, const long long* rb, long long maxrows,
                         int ldk, const float* recv, const float* recv_b, float* fac,
                         float* bias);

const char* mr_last_error(void);
int mr_device_count(void);
/* PCI bus id of a visible device ("domain:bus:device.function"): tells
 * ranks that share one physical GPU apart (MR_OPT_CG_RESIDENT). */
int mr_device_pci_bus_id(int device, char* out, int len);

#ifdef __cplusplus
}
#endif
#endif /* MR_ALS_H */
