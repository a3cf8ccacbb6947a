// extern "C" boundary of cpp_ls_lib.so.
//
// (1) The reference ABI (include/cpp_ls_lib.h), replacing
//     cpp/ls_lib/ls_linux_dll.cpp:8-103 symbol for symbol.
// (2) The device-resident engine API (include/mr_als.h).
// No torch types, plain pointers and sizes; failures return <0 / NULL and
// leave a message in mr_last_error() (also printed to stderr).
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <vector>

#include "../../include/cpp_ls_lib.h"
#include "../../include/mr_cg.h"
#include "engine.h"

struct mr_als {
  mr::Engine eng;
};

namespace {
int g_thread_count = 4;     // ls_linux_dll.cpp:6 (stored verbatim, not used on the GPU)
int g_gram_chunk = 2048;

int env_device() {
  const char* d = getenv("MR_DEVICE");
  return d ? atoi(d) : 0;
}

template <typename F>
int guarded(F&& f) {
  int rc = -1;
  try {
    rc = f();
  } catch (const std::bad_alloc&) {
    mr::set_error("host out of memory");
  } catch (...) {
    mr::set_error("unexpected C++ exception");
  }
  // a launch helper that failed inside a timed interval leaves its event pair
  // in this thread's launch-timing slot: never carry it into the next call
  if (rc < 0) mr::t_launch = mr::LaunchTiming{};
  return rc;
}
// Device scratch of the test hooks (freed with its stream).
struct DevScratch {
  hipStream_t s = nullptr;
  std::vector<void*> p;
  ~DevScratch() {
    if (s) (void)hipStreamSynchronize(s);
    for (void* q : p) (void)hipFree(q);
    if (s) (void)hipStreamDestroy(s);
  }
  template <typename T>
  int alloc(T** q, int64_t n) {
    MR_HIP(hipMalloc((void**)q, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
    p.push_back(*q);
    return 0;
  }
};
}  // namespace

extern "C" {

// ---- reference ABI ----------------------------------------------------------
void set_thread_count(int thread_count) { g_thread_count = thread_count; }
int get_thread_count(void) { return g_thread_count; }

int cg_least_squares_from_python(int A_rows, int A_cols, int* A_row_indices,
                                 int* A_col_indices, double* A_values,
                                 int b_length, double* b_values, int x_length,
                                 double* x_values, double min_r_decrease,
                                 int max_iteration, double* final_rr) {
  return guarded([&]() -> int {
    MR_CHECK(b_length == A_rows, "cg_least_squares: b_length != A_rows");
    MR_CHECK(x_length == A_cols, "cg_least_squares: x_length != A_cols");
    // a context per call, as the reference builds its matrices per call:
    // upload, device transpose, CG, download (include/mr_cg.h)
    mr_cg* h = mr_cg_create(env_device(), A_rows, A_cols, A_row_indices, A_col_indices,
                            A_values);
    if (!h) return -1;
    const int it = mr_cg_solve(h, b_values, x_values, min_r_decrease, max_iteration, final_rr);
    mr_cg_destroy(h);
    return it;
  });
}

int cg_least_squares2_from_python(int A_rows, int A_cols, int* A_row_indices,
                                  int* A_col_indices, double* A_values,
                                  int b_length, double* b_values, int x_length,
                                  double* x_values, double min_r_decrease,
                                  int max_iteration, double* final_rr) {
  return cg_least_squares_from_python(A_rows, A_cols, A_row_indices, A_col_indices,
                                      A_values, b_length, b_values, x_length, x_values,
                                      min_r_decrease, max_iteration, final_rr);
}

int als_from_python(int* user_ids, int* item_ids, int ratings_length,
                    double* ratings_values, int num_item_factors,
                    int user_factors_length, double* user_factors_values,
                    int item_factors_length, double* item_factors_values,
                    double min_r_decrease, int max_iteration, int algorithm) {
  (void)algorithm;
  return guarded([&]() -> int {
    const int k = num_item_factors;
    MR_CHECK(k >= 1, "als: num_item_factors must be >= 1");
    MR_CHECK(ratings_length >= 0, "als: negative ratings_length");
    MR_CHECK(user_factors_length % (k + 1) == 0,
             "als: user_factors_length is not a multiple of k+1");
    MR_CHECK(item_factors_length % k == 0, "als: item_factors_length is not a multiple of k");
    const int U = user_factors_length / (k + 1);
    const int I = item_factors_length / k;
    mr::Engine eng;
    eng.chunk = g_gram_chunk;
    if (eng.init(env_device(), k, U, I, ratings_length, user_ids, item_ids, ratings_values,
                 ratings_length, user_ids, item_ids, ratings_values, 0, U, 0, I))
      return -1;
    // The reference's loop body never runs for max_iteration <= 0 and the
    // factors come back untouched (matrix.cpp:814); keep them bit-exact
    // instead of round-tripping through the fp32 device tables.
    if (max_iteration <= 0) return 0;
    if (eng.set_factors(user_factors_values, item_factors_values)) return -1;
    const int ret = eng.run(min_r_decrease, max_iteration);
    if (ret < 0) return -1;
    // Entities without ratings have all-zero normal equations: the reference
    // CG leaves their x exactly as given (r = p = 0 there).  Restore those
    // rows in fp64 so they, too, are bit-identical.
    std::vector<char> seen_u(U, 0), seen_i(I, 0);
    for (int n = 0; n < ratings_length; ++n) {
      seen_u[user_ids[n]] = 1;
      seen_i[item_ids[n]] = 1;
    }
    std::vector<double> u_keep, i_keep;
    for (int u = 0; u < U; ++u)
      if (!seen_u[u])
        u_keep.insert(u_keep.end(), user_factors_values + (int64_t)u * (k + 1),
                      user_factors_values + (int64_t)(u + 1) * (k + 1));
    for (int i = 0; i < I; ++i)
      if (!seen_i[i])
        i_keep.insert(i_keep.end(), item_factors_values + (int64_t)i * k,
                      item_factors_values + (int64_t)(i + 1) * k);
    if (eng.get_factors(user_factors_values, item_factors_values)) return -1;
    size_t pu = 0, pi = 0;
    for (int u = 0; u < U; ++u)
      if (!seen_u[u]) {
        std::copy(u_keep.begin() + pu, u_keep.begin() + pu + k + 1,
                  user_factors_values + (int64_t)u * (k + 1));
        pu += k + 1;
      }
    for (int i = 0; i < I; ++i)
      if (!seen_i[i]) {
        std::copy(i_keep.begin() + pi, i_keep.begin() + pi + k, item_factors_values + (int64_t)i * k);
        pi += k;
      }
    return ret;
  });
}

// ---- engine API -------------------------------------------------------------
mr_als* mr_als_create_shard(int device, int k, int num_users, int num_items,
                            long long n_u, const int* uv_uid, const int* uv_iid,
                            const double* uv_r, long long n_i, const int* iv_uid,
                            const int* iv_iid, const double* iv_r, int u_begin,
                            int u_end, int i_begin, int i_end) {
  mr_als* ctx = nullptr;
  const int rc = guarded([&]() -> int {
    ctx = new mr_als();
    ctx->eng.chunk = g_gram_chunk;
    return ctx->eng.init(device, k, num_users, num_items, n_u, uv_uid, uv_iid, uv_r, n_i,
                         iv_uid, iv_iid, iv_r, u_begin, u_end, i_begin, i_end);
  });
  if (rc) {
    delete ctx;
    return nullptr;
  }
  return ctx;
}

mr_als* mr_als_create(int device, int k, int num_users, int num_items,
                      long long n_ratings, const int* user_ids, const int* item_ids,
                      const double* ratings) {
  return mr_als_create_shard(device, k, num_users, num_items, n_ratings, user_ids,
                             item_ids, ratings, n_ratings, user_ids, item_ids, ratings, 0,
                             num_users, 0, num_items);
}

int mr_als_set_comm(mr_als* ctx, const mr_comm* comm, const long long* user_begin,
                    const long long* item_begin) {
  MR_CHECK(ctx && comm, "null argument");
  return guarded([&]() -> int {
    MR_CHECK(comm->world >= 1 && comm->rank >= 0 && comm->rank < comm->world, "bad comm");
    MR_CHECK(comm->world == 1 || (comm->allreduce_f64 && comm->allgather_rows),
             "comm callbacks missing");
    ctx->eng.comm = *comm;
    ctx->eng.has_comm = true;
    ctx->eng.row_begin_u.assign(user_begin, user_begin + comm->world + 1);
    ctx->eng.row_begin_i.assign(item_begin, item_begin + comm->world + 1);
    // the padded all-gather staging the RCCL transport uses, too
    return comm->world > 1 ? ctx->eng.alloc_ag(comm->world) : 0;
  });
}

int mr_rccl_unique_id(unsigned char out[128]) {
  return guarded([&]() -> int {
    ncclUniqueId id;
    MR_CHECK(ncclGetUniqueId(&id) == ncclSuccess, "ncclGetUniqueId failed");
    memcpy(out, id.internal, 128);
    return 0;
  });
}

int mr_als_set_rccl(mr_als* ctx, const unsigned char id[128], int rank, int world,
                    const long long* user_begin, const long long* item_begin) {
  MR_CHECK(ctx && id, "null argument");
  return guarded([&]() -> int {
    ctx->eng.row_begin_u.assign(user_begin, user_begin + world + 1);
    ctx->eng.row_begin_i.assign(item_begin, item_begin + world + 1);
    return ctx->eng.set_rccl(id, rank, world);
  });
}

int mr_als_peer_handle(mr_als* ctx, unsigned char out[64]) {
  MR_CHECK(ctx && out, "null argument");
  return guarded([&]() { return ctx->eng.peer_handle(out); });
}

int mr_als_set_peer(mr_als* ctx, const unsigned char* handles, int rank, int world) {
  MR_CHECK(ctx && (handles || world == 0), "null argument");
  return guarded([&]() { return ctx->eng.set_peer(handles, rank, world); });
}

int mr_als_weights_bf16(mr_als* ctx, int force) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.weights_bf16(force); });
}

int mr_als_peer_selftest(mr_als* ctx) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.peer_selftest(); });
}

int mr_als_peer_latency(mr_als* ctx, int iters, double* us) {
  MR_CHECK(ctx && us, "null argument");
  return guarded([&]() { return ctx->eng.peer_latency(iters, us); });
}

void mr_als_destroy(mr_als* ctx) { delete ctx; }

int mr_als_set_factors(mr_als* ctx, const double* U, const double* V) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.set_factors(U, V); });
}

int mr_als_init_factors(mr_als* ctx, unsigned long long seed) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() -> int {
    mr::Engine& E = ctx->eng;
    MR_HIP(hipSetDevice(E.device));
    if (mr::launch_init_factors(E.stream, E.U, E.k, E.ldk, seed, 0, E.Ufac, E.Ubias) ||
        mr::launch_init_factors(E.stream, E.I, E.k, E.ldk, seed, 1, E.Vfac, nullptr))
      return -1;
    MR_HIP(hipStreamSynchronize(E.stream));
    return 0;
  });
}

int mr_als_get_factors(mr_als* ctx, double* U, double* V) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.get_factors(U, V); });
}

int mr_als_set_solver(mr_als* ctx, int solver, double ridge) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(solver == MR_SOLVER_CG || solver == MR_SOLVER_CHOLESKY, "unknown solver");
  MR_CHECK(ridge >= 0.0, "ridge must be >= 0");
  ctx->eng.solver = solver;
  ctx->eng.ridge = ridge;
  return 0;
}

int mr_als_set_timing(mr_als* ctx, int enable) {
  MR_CHECK(ctx, "null context");
  ctx->eng.timing = enable != 0;
  return 0;
}

int mr_als_set_option(mr_als* ctx, int option, double value) {
  MR_CHECK(ctx, "null context");
  switch (option) {
    case MR_OPT_FUSE_START: ctx->eng.fuse_start = value != 0.0; return 0;
    case MR_OPT_CG_ONEPASS: ctx->eng.onepass = value != 0.0; return 0;
    case MR_OPT_CG_RESIDENT: ctx->eng.resident = value != 0.0; return 0;
    case MR_OPT_GRAM_RHS_MFMA: ctx->eng.rhs_mfma = value != 0.0; return 0;
    case MR_OPT_CG_SWEEP:
      MR_CHECK(value == 0.0 || value == 1.0 || value == 2.0, "cg_sweep must be 0, 1 or 2");
      ctx->eng.sweep = (int)value;
      return 0;
    case MR_OPT_CG_SPECULATE:
      // every rank of a sharded run must use the same level (it decides which
      // launches, and with them which collectives, are issued)
      MR_CHECK(value == 0.0 || value == 1.0 || value == 2.0, "cg_speculate must be 0, 1 or 2");
      ctx->eng.speculate = (int)value;
      return 0;
    case MR_OPT_WAIT_TIMEOUT_S:
      MR_CHECK(value > 0.0, "timeout must be > 0");
      ctx->eng.wait_timeout_s = value;
      return 0;
    case MR_OPT_CG_TILE_NT:
      MR_CHECK(value == -1.0 || value == 0.0 || value == 1.0, "cg_tile_nt must be -1, 0 or 1");
      ctx->eng.tile_nt = (int)value;
      return 0;
    case MR_OPT_PEER_TIMEOUT_S:
      return guarded([&]() { return ctx->eng.set_peer_timeout(value); });
    default: MR_CHECK(false, "unknown option");
  }
}

// Diagnostics (tools/op_timeline.py; not part of the reference ABI): the
// s_memrealtime timeline of the last one-pass CG launch in an MR_OP_PROF
// build (returns the number of values copied, 0 in a product build).
int mr_debug_op_timeline(long long* out, int n) {
  MR_CHECK(out && n > 0, "bad buffer");
  return mr::op_prof_read(reinterpret_cast<int64_t*>(out), n);
}

int mr_set_gram_chunk(int chunk) {
  MR_CHECK(chunk >= 64 && chunk <= (1 << 30), "chunk must be in [64, 2^30]");
  g_gram_chunk = chunk;
  return 0;
}

int mr_als_run(mr_als* ctx, double min_r_decrease, int max_iteration) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.run(min_r_decrease, max_iteration); });
}

int mr_als_iterate(mr_als* ctx, int n) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.iterate(n); });
}

int mr_als_half_step(mr_als* ctx, int side, double* final_rr) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(side == MR_SIDE_USERS || side == MR_SIDE_ITEMS, "unknown side");
  return guarded(
      [&]() { return ctx->eng.half_step(side == MR_SIDE_USERS, 0.01, 200, final_rr); });
}

int mr_als_half_step_ex(mr_als* ctx, int side, double min_r_decrease, int max_iteration,
                        double* final_rr) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(side == MR_SIDE_USERS || side == MR_SIDE_ITEMS, "unknown side");
  MR_CHECK(max_iteration >= 0, "max_iteration must be >= 0");
  return guarded([&]() {
    return ctx->eng.half_step(side == MR_SIDE_USERS, min_r_decrease, max_iteration, final_rr);
  });
}

int mr_als_build_normal_equations(mr_als* ctx, int side) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(side == MR_SIDE_USERS || side == MR_SIDE_ITEMS, "unknown side");
  return guarded([&]() -> int {
    MR_HIP(hipSetDevice(ctx->eng.device));
    if (ctx->eng.gram(side == MR_SIDE_USERS ? ctx->eng.su : ctx->eng.si)) return -1;
    if (ctx->eng.resolve_timing()) return -1;
    MR_HIP(hipStreamSynchronize(ctx->eng.stream));
    return 0;
  });
}

int mr_als_get_cg_vectors(mr_als* ctx, int side, double* r, double* p, double* q) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(side == MR_SIDE_USERS || side == MR_SIDE_ITEMS, "unknown side");
  return guarded([&]() { return ctx->eng.get_cg_vectors(side == MR_SIDE_USERS, r, p, q); });
}

int mr_als_local_size(mr_als* ctx, int side, long long* first, long long* count,
                      long long* nnz) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(side == MR_SIDE_USERS || side == MR_SIDE_ITEMS, "unknown side");
  const mr::Side& S = side == MR_SIDE_USERS ? ctx->eng.su : ctx->eng.si;
  if (first) *first = S.e0;
  if (count) *count = S.E;
  if (nnz) *nnz = S.nnz;
  return 0;
}

int mr_als_cg_grid(mr_als* ctx, int side, int kind, int nt) {
  MR_CHECK(ctx && (kind == 0 || kind == 1) && (nt == 0 || nt == 1), "bad argument");
  const mr::Side& S = side == MR_SIDE_USERS ? ctx->eng.su : ctx->eng.si;
  return kind == 0 ? S.n_part_op[nt] : S.n_part_rs[nt];
}

long long mr_als_work_items(mr_als* ctx, int side) {
  if (!ctx) return -1;
  return side == MR_SIDE_USERS ? ctx->eng.su.n_work : ctx->eng.si.n_work;
}

int mr_als_get_layout(mr_als* ctx, int side, long long* off, int* idx, float* val,
                      long long* wbegin, int* wlen, int* went, int* wslab) {
  MR_CHECK(ctx, "null context");
  MR_CHECK(side == MR_SIDE_USERS || side == MR_SIDE_ITEMS, "unknown side");
  return guarded([&]() {
    return ctx->eng.get_layout(side == MR_SIDE_USERS, off, idx, val, wbegin, wlen, went, wslab);
  });
}

int mr_als_get_normal_equations(mr_als* ctx, int side, int n, const int* entities,
                                double* G_out, double* c_out) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() {
    return ctx->eng.get_normal_equations(side == MR_SIDE_USERS, n, entities, G_out, c_out);
  });
}

int mr_als_get_stats(mr_als* ctx, mr_stats* out) {
  MR_CHECK(ctx && out, "null argument");
  return guarded([&]() {
    if (ctx->eng.resolve_timing()) return -1;
    if (ctx->eng.peer_account(&ctx->eng.stats.peer_wait_ms, &ctx->eng.stats.peer_reductions, false))
      return -1;
    *out = ctx->eng.stats;
    return 0;
  });
}

int mr_als_reset_stats(mr_als* ctx) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() {
    if (ctx->eng.resolve_timing()) return -1;   // drop launches timed before the reset
    ctx->eng.stats = mr_stats{};
    double w;
    long long n;
    return ctx->eng.peer_account(&w, &n, true);
  });
}

int mr_als_sync(mr_als* ctx) {
  MR_CHECK(ctx, "null context");
  MR_HIP(hipSetDevice(ctx->eng.device));
  MR_HIP(hipStreamSynchronize(ctx->eng.stream));
  return 0;
}

void* mr_als_stream(mr_als* ctx) { return ctx ? (void*)ctx->eng.stream : nullptr; }

long long mr_als_num_ratings(mr_als* ctx) { return ctx ? ctx->eng.N : -1; }

int mr_als_device_tables(mr_als* ctx, float** Ufac, float** Ubias, float** Vfac, int* ldk) {
  MR_CHECK(ctx, "null context");
  if (Ufac) *Ufac = ctx->eng.Ufac;
  if (Ubias) *Ubias = ctx->eng.Ubias;
  if (Vfac) *Vfac = ctx->eng.Vfac;
  if (ldk) *ldk = ctx->eng.ldk;
  return 0;
}

int mr_als_predict(mr_als* ctx, long long n, const int* user_ids, const int* item_ids,
                   double* out) {
  MR_CHECK(ctx, "null context");
  return guarded([&]() { return ctx->eng.predict(n, user_ids, item_ids, out); });
}

// ---- test hooks: the all-gather staging kernels on host arrays ----------------

int mr_test_pack_rows(int device, long long rows, int ldk, const float* fac, const float* bias,
                      long long r0, long long n, float* send, float* send_b) {
  return guarded([&]() -> int {
    MR_CHECK(ldk > 0 && ldk % 4 == 0, "ldk must be a positive multiple of 4");
    MR_CHECK(rows >= 0 && r0 >= 0 && n >= 0 && r0 + n <= rows, "row range outside the table");
    MR_HIP(hipSetDevice(device));
    DevScratch d;
    MR_HIP(hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking));
    float *dfac, *dbias = nullptr, *dsend, *dsend_b = nullptr;
    if (d.alloc(&dfac, rows * ldk) || d.alloc(&dsend, n * ldk)) return -1;
    if (bias && (d.alloc(&dbias, rows) || d.alloc(&dsend_b, n))) return -1;
    MR_H2D(dfac, fac, rows * ldk * 4, d.s);
    if (bias) MR_H2D(dbias, bias, rows * 4, d.s);
    if (mr::launch_pack_rows(d.s, r0, n, ldk, dfac, dbias, dsend, dsend_b)) return -1;
    MR_D2H(send, dsend, n * ldk * 4, d.s);
    if (bias) MR_D2H(send_b, dsend_b, n * 4, d.s);
    return 0;
  });
}

int mr_test_xsum(int device, const double* terms, long long n, int blocks, double* out) {
  return guarded([&]() -> int {
    MR_CHECK(n >= 0 && blocks >= 1 && blocks <= 65535 && out, "bad arguments");
    MR_HIP(hipSetDevice(device));
    DevScratch d;
    MR_HIP(hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking));
    double *dt, *dout;
    int64_t* bins;
    if (d.alloc(&dt, std::max<long long>(n, 1)) || d.alloc(&dout, 1) || d.alloc(&bins, 16 * 11))
      return -1;
    MR_HIP(hipMemsetAsync(bins, 0, 16 * 11 * 8, d.s));
    if (n) MR_H2D(dt, terms, n * 8, d.s);
    if (mr::launch_xsum_test(d.s, dt, n, blocks, bins, dout)) return -1;
    MR_D2H(out, dout, 8, d.s);
    return 0;
  });
}

int mr_test_unstage_rows(int device, int world, int skip, const long long* rb, long long maxrows,
                         int ldk, const float* recv, const float* recv_b, float* fac,
                         float* bias) {
  return guarded([&]() -> int {
    MR_CHECK(world >= 1 && skip >= -1 && skip < world, "bad world / skip");
    MR_CHECK(ldk > 0 && ldk % 4 == 0, "ldk must be a positive multiple of 4");
    MR_CHECK(rb[0] == 0 && maxrows >= 1, "bad row boundaries");
    for (int r = 0; r < world; ++r)
      MR_CHECK(rb[r + 1] >= rb[r] && rb[r + 1] - rb[r] <= maxrows,
               "row boundaries not monotone or a shard exceeds maxrows");
    const int64_t rows = rb[world];
    MR_HIP(hipSetDevice(device));
    DevScratch d;
    MR_HIP(hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking));
    // the gathered layout: one block per rank, factors then the padded bias
    const int64_t per = mr::ag_block_floats(maxrows, ldk, bias != nullptr);
    std::vector<float> packed((size_t)world * per, 0.f);
    for (int r = 0; r < world; ++r) {
      memcpy(packed.data() + (size_t)r * per, recv + (size_t)r * maxrows * ldk,
             (size_t)maxrows * ldk * 4);
      if (bias)
        memcpy(packed.data() + (size_t)r * per + maxrows * ldk, recv_b + (size_t)r * maxrows,
               (size_t)maxrows * 4);
    }
    float *dfac, *dbias = nullptr, *drecv;
    int64_t* drb;
    if (d.alloc(&dfac, rows * ldk) || d.alloc(&drecv, (int64_t)world * per) ||
        d.alloc(&drb, world + 1))
      return -1;
    if (bias && d.alloc(&dbias, rows)) return -1;
    std::vector<int64_t> rb64(rb, rb + world + 1);
    MR_H2D(drb, rb64.data(), (world + 1) * 8, d.s);
    MR_H2D(dfac, fac, rows * ldk * 4, d.s);
    MR_H2D(drecv, packed.data(), (int64_t)world * per * 4, d.s);
    if (bias) MR_H2D(dbias, bias, rows * 4, d.s);
    if (mr::launch_unstage_rows(d.s, world, skip, drb, maxrows, ldk, drecv, dfac, dbias))
      return -1;
    MR_D2H(fac, dfac, rows * ldk * 4, d.s);
    if (bias) MR_D2H(bias, dbias, rows * 4, d.s);
    return 0;
  });
}

const char* mr_last_error(void) { return mr::last_error(); }

int mr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mr_device_pci_bus_id(int device, char* out, int len) {
  MR_CHECK(out && len > 0, "null argument");
  MR_HIP(hipDeviceGetPCIBusId(out, len, device));
  return 0;
}

}  // extern "C"
