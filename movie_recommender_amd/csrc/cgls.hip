// General sparse least squares on the GPU: the reference's cg_least_squares
// (cpp/ls_lib/matrix.cpp:456-529), reached through cg_least_squares_from_python
// / cg_least_squares2_from_python (ls_linux_dll.cpp:28-77), as a
// device-resident context (include/mr_cg.h).
//
// Per context: A uploaded once (CSR, int64 offsets on the device), its
// explicit transpose built on the device (sparse_matrix_transpose,
// matrix.cpp:617-692, as a stable radix sort), and the CSR-stream row blocks
// of both; A's rows are held ordered by first column (a row permutation,
// b permuted alike per solve).  Per solve: b2 = A^T b, r0 = A^T A x - b2, p0 = -r0, then three
// kernels per CG iteration (kernels.hip: csr_spmv_kernel x 2, cgls_update);
// the scalars and stop rules live in the device CgState and every BETA step
// publishes the state into a host-mapped seqlock ring (as the ALS engine), so
// the host keeps a few iterations enqueued ahead and never synchronises the
// stream inside the solve.
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/mr_cg.h"
#include "engine.h"

namespace mr {

namespace {

// Row blocks for the CSR-stream SpMV: consecutive rows with <= kSpTile
// non-zeros in all and <= kSpMaxRows rows; a row longer than kSpTile is a
// block of its own (blk[0] = 0, blk[n] = rows).
std::vector<int64_t> row_blocks(const std::vector<int64_t>& off) {
  const int64_t rows = (int64_t)off.size() - 1;
  std::vector<int64_t> blk{0};
  int64_t r = 0;
  while (r < rows) {
    const int64_t s = r;
    if (off[r + 1] - off[r] > kSpTile) {
      ++r;
    } else {
      while (r < rows && r - s < kSpMaxRows && off[r + 1] - off[s] <= kSpTile) ++r;
    }
    blk.push_back(r);
  }
  return blk;
}

template <typename T>
int dmalloc(T** p, int64_t n, std::vector<void*>& owned) {
  *p = nullptr;
  MR_HIP(hipMalloc((void**)p, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
  owned.push_back(*p);
  return 0;
}

}  // namespace

struct CgLs {
  int device = 0;
  hipStream_t s = nullptr;
  int64_t rows = 0, cols = 0, nnz = 0;
  std::vector<void*> owned;
  int64_t *rp = nullptr, *tp = nullptr, *blk_a = nullptr, *blk_t = nullptr;
  int64_t n_blk_a = 0, n_blk_t = 0;
  int32_t *ci = nullptr, *ti = nullptr, *perm = nullptr;
  double *v = nullptr, *tv = nullptr;
  // rp: the CG's r and p interleaved (rp[2j] = r_j, rp[2j+1] = p_j)
  double *b_in = nullptr, *b = nullptr, *b2 = nullptr, *x = nullptr, *rp2 = nullptr, *q = nullptr,
         *t = nullptr, *partials = nullptr;
  CgState* st = nullptr;
  CgState* h_init = nullptr;
  CgMirror *h_mirror = nullptr, *d_mirror = nullptr;
  int seq = 0;
  bool timing = false;
  struct Timed {
    int cls, it;
    hipEvent_t a, b;
  };
  std::vector<Timed> pend;
  std::vector<hipEvent_t> pool;
  mr_cg_stats stats{};

  ~CgLs() {
    if (!s) return;
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(s);
    for (void* q_ : owned) (void)hipFree(q_);
    if (h_init) (void)hipHostFree(h_init);
    if (h_mirror) (void)hipHostFree(h_mirror);
    for (auto& e : pool) (void)hipEventDestroy(e);
    for (auto& e : pend) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
    (void)hipStreamDestroy(s);
  }

  int ev(hipEvent_t* e) {
    if (!pool.empty()) {
      *e = pool.back();
      pool.pop_back();
      return 0;
    }
    MR_HIP(hipEventCreate(e));
    return 0;
  }
  // a timed launch takes an event pair through the launch-timing slot
  int tic(int cls, int it) {
    if (!timing) return 0;
    Timed tm{cls, it, nullptr, nullptr};
    if (ev(&tm.a) || ev(&tm.b)) return -1;
    t_launch.start = tm.a;
    t_launch.stop = tm.b;
    pend.push_back(tm);
    return 0;
  }
  int toc() {
    if (!timing) return 0;
    if (t_launch.start) {   // nothing was launched: an empty interval
      MR_HIP(hipEventRecord(pend.back().a, s));
      MR_HIP(hipEventRecord(pend.back().b, s));
    }
    t_launch = LaunchTiming{};
    return 0;
  }

  int init(int dev, int rows_, int cols_, const int* hrp, const int* hci, const double* hv) {
    MR_CHECK(rows_ >= 0 && cols_ >= 0, "negative matrix dimension");
    MR_CHECK(hrp && hrp[0] == 0, "row indices must start at 0");
    for (int i = 0; i < rows_; ++i) MR_CHECK(hrp[i + 1] >= hrp[i], "row indices not monotone");
    MR_CHECK((hci && hv) || hrp[rows_] == 0, "null column indices or values");
    device = dev;
    rows = rows_;
    cols = cols_;
    nnz = hrp[rows_];
    for (int64_t j = 0; j < nnz; ++j)
      MR_CHECK(hci[j] >= 0 && hci[j] < cols_, "column index out of range");
    MR_HIP(hipSetDevice(device));
    MR_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    MR_HIP(hipHostMalloc((void**)&h_init, sizeof(CgState), hipHostMallocDefault));
    MR_HIP(hipHostMalloc((void**)&h_mirror, kMirrorSlots * sizeof(CgMirror),
                         hipHostMallocMapped | hipHostMallocCoherent));
    memset(h_mirror, 0, kMirrorSlots * sizeof(CgMirror));
    MR_HIP(hipHostGetDevicePointer((void**)&d_mirror, h_mirror, 0));
    int32_t *rp32 = nullptr, *rowof = nullptr, *ci0 = nullptr;
    int64_t* rp0 = nullptr;
    double* v0 = nullptr;
    // ids / values padded by kSpPad entries: the SpMV's 16-byte row-block
    // loads may run up to 7 entries past a block's (and the array's) end
    if (dmalloc(&rp, rows + 1, owned) || dmalloc(&ci, nnz + kSpPad, owned) ||
        dmalloc(&v, nnz + kSpPad, owned) ||
        dmalloc(&perm, rows, owned) || dmalloc(&tp, cols + 1, owned) ||
        dmalloc(&ti, nnz + kSpPad, owned) || dmalloc(&tv, nnz + kSpPad, owned) || dmalloc(&b_in, rows, owned) ||
        dmalloc(&b, rows, owned) || dmalloc(&t, rows, owned) || dmalloc(&b2, cols, owned) ||
        dmalloc(&x, cols, owned) || dmalloc(&rp2, 2 * cols, owned) ||
        dmalloc(&q, cols, owned) || dmalloc(&partials, kMaxParts, owned) ||
        dmalloc(&st, 1, owned))
      return -1;
    std::vector<void*> tmp;
    struct TmpFree {
      std::vector<void*>& v;
      hipStream_t s;
      ~TmpFree() {
        (void)hipStreamSynchronize(s);
        for (void* q_ : v) (void)hipFree(q_);
      }
    } tmp_free{tmp, s};
    if (dmalloc(&rp32, rows + 1, tmp) || dmalloc(&rp0, rows + 1, tmp) ||
        dmalloc(&ci0, nnz, tmp) || dmalloc(&v0, nnz, tmp))
      return -1;
    MR_H2D(rp32, hrp, (rows + 1) * 4, s);
    if (nnz) {
      MR_H2D(ci0, hci, nnz * 4, s);
      MR_H2D(v0, hv, nnz * 8, s);
    }
    if (launch_i32_to_i64(s, rows + 1, rp32, rp0)) return -1;
    // rows ordered by first column (a row permutation: same solution, same
    // row sums), so A^T's rows read t in runs and A's rows gather r, p from
    // neighbouring columns (csr_build.hip sort_rows_by_first_col)
    if (sort_rows_by_first_col(s, rows, cols, rp0, ci0, v0, perm, rp, ci, v)) return -1;
    for (void* q_ : {(void*)rp32, (void*)rp0, (void*)ci0, (void*)v0}) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(q_);
    }
    tmp.clear();
    if (dmalloc(&rowof, nnz, tmp)) return -1;
    // explicit transpose (sparse_matrix_transpose, matrix.cpp:617-692): a
    // stable sort of the non-zeros by column keeps each column's rows in order
    if (launch_rows_of(s, rows, rp, rowof)) return -1;
    if (build_csr<double, double>(s, nnz, cols, ci, 0, rowof, v, tp, ti, tv)) return -1;
    // row blocks of A and of A^T (offsets read back once)
    std::vector<int64_t> offa(rows + 1), offt(cols + 1);
    MR_D2H(offa.data(), rp, (rows + 1) * 8, s);
    MR_D2H(offt.data(), tp, (cols + 1) * 8, s);
    // uploaded as (first row, its first non-zero) pairs: the kernels read a
    // block's bounds with no dependent load through the row offsets
    auto pairs = [](const std::vector<int64_t>& bl, const std::vector<int64_t>& off) {
      std::vector<int64_t> pr(2 * bl.size());
      for (size_t i = 0; i < bl.size(); ++i) {
        pr[2 * i] = bl[i];
        pr[2 * i + 1] = off[bl[i]];
      }
      return pr;
    };
    const std::vector<int64_t> ba = pairs(row_blocks(offa), offa),
                               bt = pairs(row_blocks(offt), offt);
    n_blk_a = (int64_t)ba.size() / 2 - 1;
    n_blk_t = (int64_t)bt.size() / 2 - 1;
    if (dmalloc(&blk_a, (int64_t)ba.size(), owned) || dmalloc(&blk_t, (int64_t)bt.size(), owned))
      return -1;
    MR_H2D(blk_a, ba.data(), ba.size() * 8, s);
    MR_H2D(blk_t, bt.data(), bt.size() * 8, s);
    MR_HIP(hipStreamSynchronize(s));
    stats.rows = rows;
    stats.cols = cols;
    stats.nnz = nnz;
    stats.blocks_a = n_blk_a;
    stats.blocks_at = n_blk_t;
    stats.block_max_nnz = kSpTile;
    stats.block_max_rows = kSpMaxRows;
    return 0;
  }

  // t = A p (p formed from r, p and beta for it > 0); q = A^T t with the p
  // update and alpha; x, r update with the BETA rule, published under `sq`.
  int iteration(int it, int sq) {
    if (tic(MR_CG_K_SPMV_A, it) ||
        launch_csr_spmv(s, it > 0 ? SPG_P : SPG_P0, SPO_STORE, st, n_blk_a, blk_a, rp, ci, v,
                        rp2, nullptr, 2 * cols, t, nullptr, nullptr, 0, nullptr, kMaxParts,
                        nullptr) ||
        toc())
      return -1;
    if (tic(MR_CG_K_SPMV_AT, it) ||
        launch_csr_spmv(s, SPG_X, SPO_CG, st, n_blk_t, blk_t, tp, ti, tv, t, nullptr, rows, q, rp2, nullptr,
                        it > 0 ? 1 : 0, partials, kMaxParts, st) ||
        toc())
      return -1;
    if (tic(MR_CG_K_UPDATE, it) ||
        launch_cgls_update(s, st, UPD_STEP, cols, x, rp2, q, b2, partials, kUpdParts, st,
                           d_mirror, sq) ||
        toc())
      return -1;
    return 0;
  }

  int solve(const double* hb, double* hx, double min_dec, int max_it, double* final_rr) {
    MR_CHECK((hb || rows == 0) && (hx || cols == 0), "null b or x");
    MR_HIP(hipSetDevice(device));
    if (rows) {
      MR_H2D(b_in, hb, rows * 8, s);
      if (launch_gather_f64(s, rows, perm, b_in, b)) return -1;   // b in the rows' order
    }
    if (cols) MR_H2D(x, hx, cols * 8, s);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
      if (ev(&e0) || ev(&e1)) return -1;
      MR_HIP(hipEventRecord(e0, s));
    }
    memset(h_init, 0, sizeof(CgState));
    h_init->min_dec = min_dec;
    h_init->max_it = max_it;
    MR_HIP(hipMemcpyAsync(st, h_init, sizeof(CgState), hipMemcpyHostToDevice, s));
    // b2 = A^T b (:463); r0 = A^T (A x) - b2, p0 = -r0, rr (:466-485)
    if (tic(MR_CG_K_SETUP, -1) ||
        launch_csr_spmv(s, SPG_X, SPO_STORE, nullptr, n_blk_t, blk_t, tp, ti, tv, b, nullptr,
                        rows, b2, nullptr, nullptr, 0, nullptr, kMaxParts, nullptr) ||
        launch_csr_spmv(s, SPG_X, SPO_STORE, nullptr, n_blk_a, blk_a, rp, ci, v, x, nullptr, cols, t,
                        nullptr, nullptr, 0, nullptr, kMaxParts, nullptr) ||
        launch_csr_spmv(s, SPG_X, SPO_STORE, nullptr, n_blk_t, blk_t, tp, ti, tv, t, nullptr, rows, q,
                        nullptr, nullptr, 0, nullptr, kMaxParts, nullptr) ||
        launch_cgls_update(s, st, UPD_INIT, cols, x, rp2, q, b2, partials, kUpdParts, st,
                           d_mirror, ++seq) ||
        toc())
      return -1;
    const int seq_init = seq;
    // Enqueue up to kAhead iterations beyond the last known state; an
    // iteration enqueued after the solve stopped exits at once (done flag).
    constexpr int kAhead = 3;
    std::vector<int> seq_of;
    int launched = 0;
    auto enqueue_to = [&](int n) -> int {
      while (launched < std::min(n, max_it)) {
        seq_of.push_back(++seq);
        if (iteration(launched, seq_of.back())) return -1;
        ++launched;
      }
      return 0;
    };
    if (enqueue_to(kAhead)) return -1;
    CgMirror ms{};
    if (wait_published(h_mirror, seq_init, s, 300.0, &ms)) return -1;
    int known = -1;   // ms = the state after iteration `known` (-1: the start)
    while (!ms.done) {
      if (enqueue_to(known + 1 + kAhead)) return -1;
      MR_CHECK(known + 1 < (int)seq_of.size(), "CG did not terminate");
      if (wait_published(h_mirror, seq_of[known + 1], s, 300.0, &ms)) return -1;
      ++known;
    }
    if (timing) MR_HIP(hipEventRecord(e1, s));
    if (cols) MR_D2H(hx, x, cols * 8, s);
    MR_HIP(hipStreamSynchronize(s));
    if (timing) {
      float ms_ = 0.f;
      MR_HIP(hipEventElapsedTime(&ms_, e0, e1));
      stats.solve_ms += ms_;
      pool.push_back(e0);
      pool.push_back(e1);
      for (auto& tm : pend) {
        if (tm.it < ms.n_matvec) {   // setup (-1) and the iterations that did work
          MR_HIP(hipEventElapsedTime(&ms_, tm.a, tm.b));
          stats.kernel_ms[tm.cls] += ms_;
          stats.kernel_launches[tm.cls] += 1;
        }
        pool.push_back(tm.a);
        pool.push_back(tm.b);
      }
      pend.clear();
    }
    stats.last_iterations = ms.ret;
    stats.iterations_total += ms.ret;
    if (final_rr) *final_rr = ms.final_rr;
    return ms.ret;
  }
};

}  // namespace mr

struct mr_cg {
  mr::CgLs c;
};

namespace {
template <typename F>
int cg_guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    mr::set_error("host out of memory");
  } catch (...) {
    mr::set_error("unexpected C++ exception");
  }
  return -1;
}
}  // namespace

extern "C" {

mr_cg* mr_cg_create(int device, int rows, int cols, const int* row_indices,
                    const int* col_indices, const double* values) {
  mr_cg* h = nullptr;
  const int rc = cg_guarded([&]() -> int {
    h = new mr_cg();
    return h->c.init(device, rows, cols, row_indices, col_indices, values);
  });
  if (rc) {
    delete h;
    return nullptr;
  }
  return h;
}

void mr_cg_destroy(mr_cg* ctx) { delete ctx; }

int mr_cg_solve(mr_cg* ctx, const double* b, double* x, double min_r_decrease, int max_iteration,
                double* final_rr) {
  MR_CHECK(ctx, "null context");
  const int rc =
      cg_guarded([&]() { return ctx->c.solve(b, x, min_r_decrease, max_iteration, final_rr); });
  // a launch helper that failed inside a timed interval left its event pair
  // in this thread's launch-timing slot: drop it, so that the next launch on
  // the thread (any context) does not record into this context's events
  mr::t_launch = mr::LaunchTiming{};
  return rc;
}

int mr_cg_set_timing(mr_cg* ctx, int enable) {
  MR_CHECK(ctx, "null context");
  ctx->c.timing = enable != 0;
  return 0;
}

int mr_cg_get_stats(mr_cg* ctx, mr_cg_stats* out) {
  MR_CHECK(ctx && out, "null argument");
  *out = ctx->c.stats;
  return 0;
}

int mr_cg_reset_stats(mr_cg* ctx) {
  MR_CHECK(ctx, "null context");
  const mr_cg_stats keep = ctx->c.stats;
  ctx->c.stats = mr_cg_stats{};
  ctx->c.stats.rows = keep.rows;
  ctx->c.stats.cols = keep.cols;
  ctx->c.stats.nnz = keep.nnz;
  ctx->c.stats.blocks_a = keep.blocks_a;
  ctx->c.stats.blocks_at = keep.blocks_at;
  ctx->c.stats.block_max_nnz = keep.block_max_nnz;
  ctx->c.stats.block_max_rows = keep.block_max_rows;
  return 0;
}

}  // extern "C"
