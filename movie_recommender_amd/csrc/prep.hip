// ALS training-set preparation on MI355X (gfx950).  C ABI: include/mr_prep.h.
//
// The reference prepares the ALS input with a pool of Python processes over
// lists of (movie_id, rating) tuples (movie_lens_data.py:547-680,
// movie_lens_data_proc.py:393-654).  Here the flattened ratings stay on the
// device: per-id counters with atomics for the iterative degree shrink, a
// two-pass stable radix sort (rating, then movie) for the exact medians, and a
// scan-based stable compaction for the training arrays.  Everything is
// integer work or a single correctly rounded fp64 operation, so results are
// exact.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/mr_als.h"
#include "../../include/mr_prep.h"
#include "mr_internal.h"

namespace mr {

static unsigned pgrid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384));
}
#define GRID_STRIDE(i, n)                                                     \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
       i += (int64_t)gridDim.x * blockDim.x)

__global__ void prep_bounds_kernel(int64_t n, const int* __restrict__ uid,
                                   const int* __restrict__ mid, int* __restrict__ mx) {
  int mu = -1, mm = -1, bad = 0;
  GRID_STRIDE(i, n) {
    mu = max(mu, uid[i]);
    mm = max(mm, mid[i]);
    bad |= (uid[i] < 0) | (mid[i] < 0);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mu = max(mu, __shfl_xor(mu, o, 64));
    mm = max(mm, __shfl_xor(mm, o, 64));
    bad |= __shfl_xor(bad, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&mx[0], mu);
    atomicMax(&mx[1], mm);
    if (bad) atomicOr(&mx[2], 1);
  }
}

// _drop_users (movie_lens_data_proc.py:494-535): users still listed with
// fewer than min_ratings ratings are removed.
__global__ void prep_drop_users_kernel(int U, const int* __restrict__ cnt,
                                       uint8_t* __restrict__ present, int min_ratings,
                                       int* __restrict__ changed) {
  GRID_STRIDE(u, U) {
    if (present[u] && cnt[u] < min_ratings) {
      present[u] = 0;
      *changed = 1;
    }
  }
}

// _count_movies + als_data_set_shrink_mp:578-587: movies that appear with
// fewer than k ratings are dropped.
__global__ void prep_drop_movies_kernel(int M, const int* __restrict__ cnt,
                                        uint8_t* __restrict__ dead, int min_count,
                                        int* __restrict__ changed) {
  GRID_STRIDE(m, M) {
    if (cnt[m] >= 1 && cnt[m] < min_count) {
      dead[m] = 1;
      *changed = 1;
    }
  }
}

// ---- run-aggregated updates --------------------------------------------------
// A wave holds 64 consecutive elements of an order in which equal keys are
// contiguous (input order for users, sorted orders otherwise).  A segmented
// inclusive scan over equal keys leaves each run's total in its last lane,
// which alone touches memory: one atomic per run instead of one per element
// (the per-element atomics serialised on popular ids: 2.2 ms per pass).
// run index of each lane: equal keys in non-adjacent lanes are different runs
__device__ __forceinline__ int run_id(int64_t key) {
  const int lane = threadIdx.x & 63;
  const int64_t pk = __shfl_up(key, 1, 64);
  const unsigned long long heads = __ballot(lane == 0 || pk != key);
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  return __popcll(heads & upto);
}

__device__ __forceinline__ void run_add(int64_t key, int val, int* __restrict__ cnt, int64_t skip) {
  const int lane = threadIdx.x & 63;
  const int rid = run_id(key);
  int sum = val;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int ov = __shfl_up(sum, d, 64);
    const int orid = __shfl_up(rid, d, 64);
    if (lane >= d && orid == rid) sum += ov;
  }
  const int nrid = __shfl_down(rid, 1, 64);
  if ((lane == 63 || nrid != rid) && key != skip && sum != 0) atomicAdd(&cnt[key], sum);
}

__device__ __forceinline__ void run_min(int64_t key, unsigned long long val,
                                        unsigned long long* __restrict__ out, int64_t slot,
                                        int64_t skip) {
  const int lane = threadIdx.x & 63;
  const int rid = run_id(key);
  unsigned long long m = val;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long ov = __shfl_up(m, d, 64);
    const int orid = __shfl_up(rid, d, 64);
    if (lane >= d && orid == rid) m = min(m, ov);
  }
  const int nrid = __shfl_down(rid, 1, 64);
  if ((lane == 63 || nrid != rid) && key != skip && m != ~0ull) atomicMin(&out[slot], m);
}

// wave-contiguous grid stride: every lane of a wave runs the same iterations
#define WAVE_STRIDE(j, n)                                                        \
  for (int64_t j##_b = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)); \
       j##_b < (n); j##_b += (int64_t)gridDim.x * blockDim.x)                    \
    for (int64_t j = j##_b + (threadIdx.x & 63), j##_once = 0; j##_once < 1; ++j##_once)

__global__ void prep_iota_kernel(int64_t n, uint32_t* __restrict__ o) {
  GRID_STRIDE(i, n) o[i] = (uint32_t)i;
}

// counts over a sorted order (key[j] = id of element perm[j])
__global__ void prep_count_sorted_kernel(int64_t n, const uint32_t* __restrict__ key,
                                         const uint32_t* __restrict__ perm,
                                         const uint8_t* __restrict__ alive, int* __restrict__ cnt) {
  WAVE_STRIDE(j, n) {
    const bool in = j < n;
    const int64_t kk = in ? (int64_t)key[j] : -1;
    const int v = (in && alive[perm[j]]) ? 1 : 0;
    run_add(kk, v, cnt, -1);
  }
}

// ratings of dropped users / movies die; their counts are decremented (users
// run-aggregated in input order, movies per element -- deaths are rare)
__global__ void prep_kill_dec_kernel(int64_t n, const int* __restrict__ uid,
                                     const int* __restrict__ mid,
                                     const uint8_t* __restrict__ present,
                                     const uint8_t* __restrict__ dead,
                                     uint8_t* __restrict__ alive, int* __restrict__ ucnt,
                                     int* __restrict__ mcnt) {
  WAVE_STRIDE(i, n) {
    const bool in = i < n;
    int u = -1;
    bool dies = false;
    if (in) {
      u = uid[i];
      if (alive[i]) {
        const int m = mid[i];
        dies = !present[u] || dead[m];
        if (dies) {
          alive[i] = 0;
          atomicSub(&mcnt[m], 1);
        }
      }
    }
    run_add(u, dies ? -1 : 0, ucnt, -1);
  }
}

__global__ void prep_present_from_counts_kernel(int U, const int* __restrict__ ucnt,
                                                uint8_t* __restrict__ present) {
  GRID_STRIDE(u, U) present[u] = ucnt[u] > 0;
}

// first surviving index per (id, chunk) over an id-sorted order (indices
// ascend within an id, so chunks are runs too)
__global__ void prep_first_sorted_kernel(int64_t n, const uint32_t* __restrict__ key,
                                         const uint32_t* __restrict__ perm,
                                         const uint8_t* __restrict__ alive,
                                         const int64_t* __restrict__ cb, int n_chunks, int bound,
                                         unsigned long long* __restrict__ out) {
  WAVE_STRIDE(j, n) {
    const bool in = j < n;
    int64_t kk = -1, slot = 0;
    unsigned long long v = ~0ull;
    if (in) {
      const uint32_t i = perm[j];
      int lo = 0, hi = n_chunks;   // chunk c: cb[c] <= i < cb[c+1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (cb[mid] <= (int64_t)i) lo = mid;
        else hi = mid;
      }
      const bool inside = (int64_t)i >= cb[0] && (int64_t)i < cb[n_chunks];
      kk = inside ? (int64_t)key[j] * n_chunks + lo : -1;
      slot = (int64_t)lo * bound + key[j];
      if (inside && alive[i]) v = i;
    }
    run_min(kk, v, out, slot, -1);
  }
}

__device__ __forceinline__ uint64_t ord_key(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ void prep_rating_keys_kernel(int64_t n, const double* __restrict__ r,
                                        uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
  GRID_STRIDE(i, n) {
    key[i] = ord_key(r[i]);
    idx[i] = (uint32_t)i;
  }
}

__global__ void prep_gather_movie_kernel(int64_t n, const uint32_t* __restrict__ perm,
                                         const int* __restrict__ mid, uint32_t* __restrict__ out) {
  GRID_STRIDE(i, n) out[i] = (uint32_t)mid[perm[i]];
}

__global__ void prep_movie_offsets_kernel(int64_t n, int M, const uint32_t* __restrict__ keys,
                                          int64_t* __restrict__ off) {
  GRID_STRIDE(j, n) {
    const int64_t kj = keys[j];
    const int64_t kp = (j == 0) ? -1 : (int64_t)keys[j - 1];
    for (int64_t e = kp + 1; e <= kj; ++e) off[e] = j;
    if (j == n - 1)
      for (int64_t e = kj + 1; e <= M; ++e) off[e] = n;
  }
}

// numpy.median of each movie's ratings: the middle value, or the mean of the
// two middle values ((a + b) / 2, as np.mean computes it) for even counts.
__global__ void prep_median_kernel(int M, const int64_t* __restrict__ off,
                                   const uint32_t* __restrict__ perm,
                                   const double* __restrict__ r, double* __restrict__ med) {
  GRID_STRIDE(m, M) {
    const int64_t b = off[m], c = off[m + 1] - b;
    double v = NAN;
    if (c > 0) {
      if (c & 1) {
        v = r[perm[b + c / 2]];
      } else {
        const double lo = r[perm[b + c / 2 - 1]], hi = r[perm[b + c / 2]];
        v = (lo + hi) / 2.0;
      }
    }
    med[m] = v;
  }
}

__global__ void prep_fill_u64_kernel(int64_t n, unsigned long long* p, unsigned long long v) {
  GRID_STRIDE(i, n) p[i] = v;
}

__global__ void prep_u8_to_i64_kernel(int64_t n, const uint8_t* __restrict__ a,
                                      int64_t* __restrict__ o) {
  GRID_STRIDE(i, n) o[i] = a[i];
}

// _convert_training_data_to_numpy (movie_lens_data_proc.py:640-651)
__global__ void prep_convert_kernel(int64_t n, const uint8_t* __restrict__ alive,
                                    const int64_t* __restrict__ pos, const int* __restrict__ uid,
                                    const int* __restrict__ mid, const double* __restrict__ r,
                                    const int* __restrict__ umap, const int* __restrict__ mmap,
                                    const double* __restrict__ med, int* __restrict__ ou,
                                    int* __restrict__ om, double* __restrict__ orr,
                                    int* __restrict__ bad) {
  GRID_STRIDE(i, n) {
    if (!alive[i]) continue;
    const int64_t j = pos[i];
    const int u = umap[uid[i]], m = mmap[mid[i]];
    if (u < 0 || m < 0) *bad = 1;
    ou[j] = u;
    om[j] = m;
    orr[j] = r[i] - med[mid[i]];
  }
}

// ---------------------------------------------------------------------------
struct Prep {
  int device = 0;
  hipStream_t s = nullptr;
  int64_t n = 0;
  int U = 0, M = 0;            // id bounds (max id + 1)
  int* uid = nullptr;
  int* mid = nullptr;
  double* r = nullptr;
  uint8_t* alive = nullptr;    // survivors of the last shrink
  int64_t n_kept = -1;
  int* ucnt = nullptr;         // alive ratings per user / movie (kept current)
  int* mcnt = nullptr;
  uint32_t *su_key = nullptr, *su_perm = nullptr;   // id-sorted orders (stable)
  uint32_t *sm_key = nullptr, *sm_perm = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  double ms = 0.0;
  ~Prep() {
    if (s) {
      (void)hipFree(uid);
      (void)hipFree(mid);
      (void)hipFree(r);
      (void)hipFree(alive);
      (void)hipFree(ucnt);
      (void)hipFree(mcnt);
      (void)hipFree(su_key);
      (void)hipFree(su_perm);
      (void)hipFree(sm_key);
      (void)hipFree(sm_perm);
      (void)hipStreamDestroy(s);
    }
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
  int begin() {
    MR_HIP(hipEventRecord(ev[0], s));
    return 0;
  }
  // mark(): device work of the call is done (before result copies);
  // end(): wait for the copies, ms = begin .. mark
  int mark() {
    MR_HIP(hipEventRecord(ev[1], s));
    return 0;
  }
  int end() {
    MR_HIP(hipStreamSynchronize(s));
    float t = 0.f;
    MR_HIP(hipEventElapsedTime(&t, ev[0], ev[1]));
    ms = t;
    return 0;
  }
};

template <typename T>
struct PBuf {
  T* p = nullptr;
  ~PBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(int64_t n) {
    MR_HIP(hipMalloc((void**)&p, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
    return 0;
  }
};

static int prep_init(Prep* P, int device, int64_t n, const int* uid, const int* mid,
                     const double* r) {
  MR_CHECK(n >= 0 && n < (1LL << 32), "prep: rating count must be in [0, 2^32)");
  P->device = device;
  P->n = n;
  MR_HIP(hipSetDevice(device));
  MR_HIP(hipStreamCreateWithFlags(&P->s, hipStreamNonBlocking));
  MR_HIP(hipEventCreate(&P->ev[0]));
  MR_HIP(hipEventCreate(&P->ev[1]));
  const size_t nn = std::max<int64_t>(n, 1);
  MR_HIP(hipMalloc((void**)&P->uid, nn * 4));
  MR_HIP(hipMalloc((void**)&P->mid, nn * 4));
  MR_HIP(hipMalloc((void**)&P->r, nn * 8));
  MR_HIP(hipMalloc((void**)&P->alive, nn));
  if (n) {
    MR_H2D(P->uid, uid, n * 4, P->s);
    MR_H2D(P->mid, mid, n * 4, P->s);
    MR_H2D(P->r, r, n * 8, P->s);
  }
  PBuf<int> mx;
  if (mx.alloc(3)) return -1;
  const int init[3] = {-1, -1, 0};
  MR_H2D(mx.p, init, sizeof init, P->s);
  prep_bounds_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->uid, P->mid, mx.p);
  MR_HIP(hipGetLastError());
  int h[3];
  MR_D2H(h, mx.p, sizeof h, P->s);
  MR_HIP(hipStreamSynchronize(P->s));
  MR_CHECK(h[2] == 0, "prep: user and movie ids must be >= 0");
  P->U = h[0] + 1;
  P->M = h[1] + 1;
  return 0;
}

static int prep_medians(Prep* P, double* med_out) {
  const int64_t n = P->n;
  const int M = P->M;
  if (P->begin()) return -1;
  PBuf<uint64_t> k0, k1;
  PBuf<uint32_t> i0, i1, m0, m1;
  PBuf<int64_t> off;
  PBuf<double> med;
  if (k0.alloc(n) || k1.alloc(n) || i0.alloc(n) || i1.alloc(n) || m0.alloc(n) || m1.alloc(n) ||
      off.alloc((int64_t)M + 1) || med.alloc(M))
    return -1;
  if (n > 0) {
    prep_rating_keys_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->r, k0.p, i0.p);
    size_t tmp_bytes = 0;
    MR_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0.p, k1.p, i0.p, i1.p, (size_t)n, 0,
                                     64, P->s));
    size_t tmp2 = 0;
    MR_HIP(rocprim::radix_sort_pairs(nullptr, tmp2, m0.p, m1.p, i1.p, i0.p, (size_t)n, 0, 32,
                                     P->s));
    PBuf<char> tmp;
    if (tmp.alloc((int64_t)std::max(tmp_bytes, tmp2))) return -1;
    MR_HIP(rocprim::radix_sort_pairs(tmp.p, tmp_bytes, k0.p, k1.p, i0.p, i1.p, (size_t)n, 0, 64,
                                     P->s));
    prep_gather_movie_kernel<<<pgrid(n), 256, 0, P->s>>>(n, i1.p, P->mid, m0.p);
    // stable: equal movies keep ascending rating order
    MR_HIP(rocprim::radix_sort_pairs(tmp.p, tmp2, m0.p, m1.p, i1.p, i0.p, (size_t)n, 0, 32,
                                     P->s));
    prep_movie_offsets_kernel<<<pgrid(n), 256, 0, P->s>>>(n, M, m1.p, off.p);
    prep_median_kernel<<<pgrid(M), 256, 0, P->s>>>(M, off.p, i0.p, P->r, med.p);
    MR_HIP(hipGetLastError());
  } else {
    std::vector<double> nanv(M, NAN);
    MR_H2D(med.p, nanv.data(), M * 8, P->s);
  }
  if (P->mark()) return -1;
  MR_D2H(med_out, med.p, (size_t)M * 8, P->s);
  return P->end();
}

// Stable sort of the ratings by user and by movie (once per context).
static int prep_orders(Prep* P) {
  if (P->su_perm) return 0;
  const int64_t n = P->n;
  const size_t nn = std::max<int64_t>(n, 1);
  MR_HIP(hipMalloc((void**)&P->su_key, nn * 4));
  MR_HIP(hipMalloc((void**)&P->su_perm, nn * 4));
  MR_HIP(hipMalloc((void**)&P->sm_key, nn * 4));
  MR_HIP(hipMalloc((void**)&P->sm_perm, nn * 4));
  if (n == 0) return 0;
  PBuf<uint32_t> iota;
  if (iota.alloc(n)) return -1;
  prep_iota_kernel<<<pgrid(n), 256, 0, P->s>>>(n, iota.p);
  size_t tb = 0;
  MR_HIP(rocprim::radix_sort_pairs(nullptr, tb, (const uint32_t*)P->uid, P->su_key,
                                   (const uint32_t*)iota.p, P->su_perm, (size_t)n, 0, 32, P->s));
  PBuf<char> tmp;
  if (tmp.alloc((int64_t)tb)) return -1;
  MR_HIP(rocprim::radix_sort_pairs(tmp.p, tb, (const uint32_t*)P->uid, P->su_key,
                                   (const uint32_t*)iota.p, P->su_perm, (size_t)n, 0, 32, P->s));
  MR_HIP(rocprim::radix_sort_pairs(tmp.p, tb, (const uint32_t*)P->mid, P->sm_key,
                                   (const uint32_t*)iota.p, P->sm_perm, (size_t)n, 0, 32, P->s));
  MR_HIP(hipStreamSynchronize(P->s));   // iota / tmp are released on return
  return 0;
}

static int prep_shrink(Prep* P, int k, int restart, unsigned char* keep, int* rounds,
                       long long* n_kept, int* n_users, int* n_movies) {
  MR_CHECK(k >= 0, "prep: k must be >= 0");
  MR_CHECK(restart || P->n_kept >= 0, "prep: nothing to continue from (restart = 0)");
  const int64_t n = P->n;
  const int U = P->U, M = P->M;
  if (P->begin()) return -1;
  if (!P->ucnt) {
    MR_HIP(hipMalloc((void**)&P->ucnt, (size_t)std::max(U, 1) * 4));
    MR_HIP(hipMalloc((void**)&P->mcnt, (size_t)std::max(M, 1) * 4));
  }
  if (prep_orders(P)) return -1;
  PBuf<int> flag;
  PBuf<uint8_t> present, dead;
  if (flag.alloc(2) || present.alloc(U) || dead.alloc(M)) return -1;
  // the reference shrinks its lists in place, so factor after factor
  // continues from the previous survivors (restart = 0) -- and so do the
  // counters, which every kill pass keeps current
  if (restart) {
    MR_HIP(hipMemsetAsync(P->alive, 1, std::max<int64_t>(n, 1), P->s));
    MR_HIP(hipMemsetAsync(P->ucnt, 0, (size_t)std::max(U, 1) * 4, P->s));
    MR_HIP(hipMemsetAsync(P->mcnt, 0, (size_t)std::max(M, 1) * 4, P->s));
    if (n) {
      prep_count_sorted_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->su_key, P->su_perm, P->alive,
                                                           P->ucnt);
      prep_count_sorted_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->sm_key, P->sm_perm, P->alive,
                                                           P->mcnt);
    }
  }
  if (U) prep_present_from_counts_kernel<<<pgrid(U), 256, 0, P->s>>>(U, P->ucnt, present.p);
  MR_HIP(hipMemsetAsync(dead.p, 0, std::max(M, 1), P->s));
  int it = 0;
  int h[2] = {0, 0};
  do {
    ++it;
    MR_HIP(hipMemsetAsync(flag.p, 0, 8, P->s));
    // _drop_users, then _count_movies / _drop_movies on what is left
    if (U) prep_drop_users_kernel<<<pgrid(U), 256, 0, P->s>>>(U, P->ucnt, present.p, k + 1, flag.p);
    if (n)
      prep_kill_dec_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->uid, P->mid, present.p, dead.p,
                                                       P->alive, P->ucnt, P->mcnt);
    if (M) prep_drop_movies_kernel<<<pgrid(M), 256, 0, P->s>>>(M, P->mcnt, dead.p, k, flag.p + 1);
    if (n)
      prep_kill_dec_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->uid, P->mid, present.p, dead.p,
                                                       P->alive, P->ucnt, P->mcnt);
    MR_HIP(hipGetLastError());
    MR_D2H(h, flag.p, 8, P->s);
    MR_HIP(hipStreamSynchronize(P->s));
  } while (h[0] || h[1]);
  // survivors: every present user now has >= k+1 ratings and every counted
  // movie >= k (the last round changed nothing)
  if (P->mark()) return -1;
  std::vector<int> uc(U), mc(M);
  MR_D2H(uc.data(), P->ucnt, (size_t)U * 4, P->s);
  MR_D2H(mc.data(), P->mcnt, (size_t)M * 4, P->s);
  if (keep && n) MR_D2H(keep, P->alive, n, P->s);
  if (P->end()) return -1;
  long long nk = 0;
  int nu = 0, nm = 0;
  for (int m = 0; m < M; ++m) {
    nm += mc[m] > 0;
    nk += mc[m];
  }
  for (int u = 0; u < U; ++u) nu += uc[u] > 0;
  P->n_kept = nk;
  if (rounds) *rounds = it;
  if (n_kept) *n_kept = nk;
  if (n_users) *n_users = nu;
  if (n_movies) *n_movies = nm;
  return 0;
}

static int prep_first(Prep* P, int n_chunks, const long long* cb, long long* fu_out,
                      long long* fm_out) {
  MR_CHECK(P->n_kept >= 0, "prep: run mr_prep_shrink first");
  MR_CHECK(n_chunks >= 1, "prep: n_chunks must be >= 1");
  for (int c = 0; c < n_chunks; ++c)
    MR_CHECK(cb[c] >= 0 && cb[c] <= cb[c + 1] && cb[c + 1] <= P->n, "prep: bad chunk bounds");
  if (P->begin()) return -1;
  PBuf<unsigned long long> fu, fm;
  PBuf<int64_t> dcb;
  const int64_t nu = (int64_t)n_chunks * P->U, nm = (int64_t)n_chunks * P->M;
  if (fu.alloc(nu) || fm.alloc(nm) || dcb.alloc(n_chunks + 1)) return -1;
  MR_H2D(dcb.p, cb, (n_chunks + 1) * 8, P->s);
  const unsigned long long inf = 0x7fffffffffffffffull;
  prep_fill_u64_kernel<<<pgrid(nu), 256, 0, P->s>>>(nu, fu.p, inf);
  prep_fill_u64_kernel<<<pgrid(nm), 256, 0, P->s>>>(nm, fm.p, inf);
  if (P->n) {
    prep_first_sorted_kernel<<<pgrid(P->n), 256, 0, P->s>>>(P->n, P->su_key, P->su_perm, P->alive,
                                                           dcb.p, n_chunks, P->U, fu.p);
    prep_first_sorted_kernel<<<pgrid(P->n), 256, 0, P->s>>>(P->n, P->sm_key, P->sm_perm, P->alive,
                                                           dcb.p, n_chunks, P->M, fm.p);
  }
  MR_HIP(hipGetLastError());
  if (P->mark()) return -1;
  MR_D2H(fu_out, fu.p, nu * 8, P->s);
  MR_D2H(fm_out, fm.p, nm * 8, P->s);
  return P->end();
}

static int prep_convert(Prep* P, const int* umap, const int* mmap, const double* med_h, int* ou,
                        int* om, double* orr) {
  MR_CHECK(P->n_kept >= 0, "prep: run mr_prep_shrink first");
  const int64_t n = P->n, nk = P->n_kept;
  if (P->begin()) return -1;
  PBuf<int64_t> flags, pos;
  PBuf<int> du, dm, bad, dou, dom;
  PBuf<double> dmed, dor;
  if (flags.alloc(n) || pos.alloc(n) || du.alloc(P->U) || dm.alloc(P->M) || bad.alloc(1) ||
      dou.alloc(nk) || dom.alloc(nk) || dmed.alloc(P->M) || dor.alloc(nk))
    return -1;
  MR_H2D(du.p, umap, (size_t)P->U * 4, P->s);
  MR_H2D(dm.p, mmap, (size_t)P->M * 4, P->s);
  MR_H2D(dmed.p, med_h, (size_t)P->M * 8, P->s);
  MR_HIP(hipMemsetAsync(bad.p, 0, 4, P->s));
  if (n) {
    prep_u8_to_i64_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->alive, flags.p);
    size_t tb = 0;
    MR_HIP(rocprim::exclusive_scan(nullptr, tb, flags.p, pos.p, (int64_t)0, (size_t)n,
                                   rocprim::plus<int64_t>(), P->s));
    PBuf<char> tmp;
    if (tmp.alloc((int64_t)tb)) return -1;
    MR_HIP(rocprim::exclusive_scan(tmp.p, tb, flags.p, pos.p, (int64_t)0, (size_t)n,
                                   rocprim::plus<int64_t>(), P->s));
    prep_convert_kernel<<<pgrid(n), 256, 0, P->s>>>(n, P->alive, pos.p, P->uid, P->mid, P->r,
                                                    du.p, dm.p, dmed.p, dou.p, dom.p, dor.p,
                                                    bad.p);
    MR_HIP(hipGetLastError());
  }
  if (P->mark()) return -1;
  int hb = 0;
  MR_D2H(&hb, bad.p, 4, P->s);
  if (nk) {
    MR_D2H(ou, dou.p, nk * 4, P->s);
    MR_D2H(om, dom.p, nk * 4, P->s);
    MR_D2H(orr, dor.p, nk * 8, P->s);
  }
  if (P->end()) return -1;
  MR_CHECK(hb == 0, "prep: a surviving user or movie has no entry in the id map");
  return 0;
}

}  // namespace mr

struct mr_prep {
  mr::Prep p;
};

namespace {
template <typename F>
int prep_guard(F&& f) {
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

mr_prep* mr_prep_create(int device, long long n, const int* user_id, const int* movie_id,
                        const double* rating) {
  mr_prep* ctx = nullptr;
  const int rc = prep_guard([&]() -> int {
    ctx = new mr_prep();
    return mr::prep_init(&ctx->p, device, n, user_id, movie_id, rating);
  });
  if (rc) {
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void mr_prep_destroy(mr_prep* ctx) { delete ctx; }

int mr_prep_id_bounds(const mr_prep* ctx, int* user_bound, int* movie_bound) {
  if (!ctx) return -1;
  if (user_bound) *user_bound = ctx->p.U;
  if (movie_bound) *movie_bound = ctx->p.M;
  return 0;
}

int mr_prep_medians(mr_prep* ctx, double* median) {
  if (!ctx) return -1;
  return prep_guard([&]() { return mr::prep_medians(&ctx->p, median); });
}

int mr_prep_shrink(mr_prep* ctx, int k, int restart, unsigned char* keep, int* rounds,
                   long long* n_kept, int* n_users, int* n_movies) {
  if (!ctx) return -1;
  return prep_guard([&]() {
    return mr::prep_shrink(&ctx->p, k, restart, keep, rounds, n_kept, n_users, n_movies);
  });
}

int mr_prep_first_appearance(mr_prep* ctx, int n_chunks, const long long* chunk_begin,
                             long long* first_user, long long* first_movie) {
  if (!ctx) return -1;
  return prep_guard([&]() {
    return mr::prep_first(&ctx->p, n_chunks, chunk_begin, first_user, first_movie);
  });
}

int mr_prep_convert(mr_prep* ctx, const int* user_map, const int* movie_map, const double* median,
                    int* out_user, int* out_movie, double* out_rating) {
  if (!ctx) return -1;
  return prep_guard([&]() {
    return mr::prep_convert(&ctx->p, user_map, movie_map, median, out_user, out_movie,
                            out_rating);
  });
}

double mr_prep_last_ms(const mr_prep* ctx) { return ctx ? ctx->p.ms : -1.0; }

}  // extern "C"
