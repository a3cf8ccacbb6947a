// Similar-movies database on MI355X (gfx950).  C ABI: include/mr_similar.h.
//
// Reference: build_similar_movies_db.py:19-163 (SimilarMovieFinder), run for
// every movie by movie_lens_data_proc.py:657-700.  The reference compares a
// movie with every other movie through Python dicts of co-rating users (22
// minutes on 36 vCPU for ML-full).  Here one workgroup owns a query movie and
// walks, for each of its raters, that user's movie list: every (query, other
// movie) pair accumulates its common-reviewer count n and the exact integer
// sums D = sum r1 r2, A = sum r1^2, B = sum r2^2 (ratings in half-star units)
// in LDS with 64-bit atomics (two fields per word), over ranges of 4096
// movies.  The per-user start of each range is precomputed, and each rater's
// slice of a range is flattened across the workgroup (scan + LDS search), so
// lanes stay busy although a slice averages a handful of movies.  Candidates
// (n >= 3, genre gate, score > 0.3) go to an LDS list that is cut to the
// num_results*20 movies with most common reviewers
// whenever it fills (exact: the cut only happens once more than that many
// exist), and the final ordering is a bitonic sort on the reference's stable
// sort keys.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/mr_als.h"
#include "../../include/mr_similar.h"
#include "mr_internal.h"

namespace mr {

constexpr int SM_RS = 4096;    // movies per accumulation range
constexpr int SM_CAP = 2048;   // candidate list capacity (LDS)
constexpr int SM_NT = 1024;    // threads per query workgroup
#ifndef MR_SM_U
#define MR_SM_U 4
#endif
constexpr int SM_U = MR_SM_U;   // (movie, rating) entries per thread in flight

static unsigned sgrid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384));
}
#define SGRID_STRIDE(i, n)                                                    \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
       i += (int64_t)gridDim.x * blockDim.x)

// (user, movie, rating2) packed for one radix sort: user-major, movie-minor
__global__ void sim_pack_kernel(int M, const int64_t* __restrict__ off,
                                const int* __restrict__ user, const uint8_t* __restrict__ r2,
                                uint64_t* __restrict__ key) {
  for (int m = blockIdx.x; m < M; m += gridDim.x)
    for (int64_t p = off[m] + threadIdx.x; p < off[m + 1]; p += blockDim.x)
      key[p] = ((uint64_t)(uint32_t)user[p] << 32) | ((uint64_t)(uint32_t)m << 8) | r2[p];
}

__global__ void sim_unpack_kernel(int64_t n, const uint64_t* __restrict__ key,
                                  int* __restrict__ umov, uint8_t* __restrict__ ur2,
                                  int* __restrict__ uu) {
  SGRID_STRIDE(p, n) {
    const uint64_t k = key[p];
    uu[p] = (int)(k >> 32);
    umov[p] = (int)((k >> 8) & 0xffffff);
    ur2[p] = (uint8_t)(k & 255);
  }
}

__global__ void sim_user_offsets_kernel(int64_t n, int U, const int* __restrict__ uu,
                                        int64_t* __restrict__ uoff) {
  SGRID_STRIDE(j, n) {
    const int64_t kj = uu[j];
    const int64_t kp = (j == 0) ? -1 : (int64_t)uu[j - 1];
    for (int64_t e = kp + 1; e <= kj; ++e) uoff[e] = j;
    if (j == n - 1)
      for (int64_t e = kj + 1; e <= U; ++e) uoff[e] = n;
  }
  if (n == 0 && blockIdx.x == 0)
    for (int e = threadIdx.x; e <= U; e += blockDim.x) uoff[e] = 0;
}

// ustart[u*(NR+1) + r] = first position of user u's (sorted) list whose movie
// is >= r * SM_RS
__global__ void sim_range_start_kernel(int U, int NR, const int64_t* __restrict__ uoff,
                                       const int* __restrict__ umov,
                                       int* __restrict__ ustart) {
  SGRID_STRIDE(u, U) {
    int64_t p = uoff[u];
    const int64_t e = uoff[u + 1];
    for (int r = 0; r <= NR; ++r) {
      const int lim = r * SM_RS;
      while (p < e && umov[p] < lim) ++p;
      ustart[u * (int64_t)(NR + 1) + r] = (int)p;
    }
  }
}

struct Cand {
  int j, n;
  double s;
};

// a before b in the order of the reference's stable sorts:
//   mode 0: n desc, then list (index) order   (the num_results*20 cut)
//   mode 1: score desc, then index order      (no cut happened)
//   mode 2: score desc, n desc, index order   (after the cut)
__device__ __forceinline__ bool before(const Cand& a, const Cand& b, int mode) {
  if (mode == 0) return a.n > b.n || (a.n == b.n && a.j < b.j);
  if (a.s != b.s) return a.s > b.s;
  if (mode == 2 && a.n != b.n) return a.n > b.n;
  return a.j < b.j;
}

__device__ void block_sort(int* cj, int* cn, double* cs, int count, int mode) {
  int sz = 64;
  while (sz < count) sz <<= 1;
  for (int i = count + threadIdx.x; i < sz; i += blockDim.x) {
    cj[i] = 0x7fffffff;
    cn[i] = -1;
    cs[i] = -INFINITY;
  }
  __syncthreads();
  for (int k = 2; k <= sz; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < sz; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const Cand a{cj[i], cn[i], cs[i]}, b{cj[l], cn[l], cs[l]};
          const bool asc = (i & k) == 0;
          if (asc ? before(b, a, mode) : before(a, b, mode)) {
            cj[i] = b.j;
            cn[i] = b.n;
            cs[i] = b.s;
            cj[l] = a.j;
            cn[l] = a.n;
            cs[l] = a.s;
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(SM_NT) void sim_find_kernel(
    int M, int NR, const int* __restrict__ query, const int64_t* __restrict__ moff,
    const int* __restrict__ muser, const uint8_t* __restrict__ mr2,
    const int* __restrict__ umov, const uint8_t* __restrict__ ur2,
    const int* __restrict__ ustart, const unsigned long long* __restrict__ gmask,
    const uint8_t* __restrict__ ghas, const double* __restrict__ boost1, int n_boost, int T,
    int nres, int* __restrict__ out_j, double* __restrict__ out_s, int* __restrict__ out_cnt) {
  extern __shared__ unsigned long long lds_u64[];
  unsigned long long* accA = lds_u64;            // (D << 32) | n
  unsigned long long* accB = accA + SM_RS;       // (A << 32) | B
  int* cj = reinterpret_cast<int*>(accB + SM_RS);
  int* cn = cj + SM_CAP;
  double* cs = reinterpret_cast<double*>(cn + SM_CAP);
  __shared__ int s_nbuf;
  __shared__ long long s_total;
  __shared__ int s_pre[SM_NT], s_lo[SM_NT], s_wsum[SM_NT / 64], s_tot;
  __shared__ uint8_t s_ri[SM_NT];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = SM_NT / 64;
  const int i = query ? query[q] : q;
  const unsigned long long gi = gmask[i];
  const bool hi_ok = ghas[i] != 0;
  const int li = __popcll(gi);
  if (tid == 0) {
    s_nbuf = 0;
    s_total = 0;
  }
  for (int r = 0; r < NR; ++r) {
    const int base = r * SM_RS;
    for (int t = tid; t < SM_RS; t += SM_NT) {
      accA[t] = 0;
      accB[t] = 0;
    }
    __syncthreads();
    if (hi_ok) {   // a movie without genres is never similar to anything
      // Raters in chunks of SM_NT; their entries in this range are flattened
      // (block scan of the per-rater counts) so every lane gets work however
      // short each rater's slice of the range is.
      for (int64_t t0 = moff[i]; t0 < moff[i + 1]; t0 += SM_NT) {
        const int64_t t = t0 + tid;
        int lo = 0, len = 0;
        unsigned ri = 0;
        if (t < moff[i + 1]) {
          const int u = muser[t];
          ri = mr2[t];
          lo = ustart[u * (int64_t)(NR + 1) + r];
          len = ustart[u * (int64_t)(NR + 1) + r + 1] - lo;
        }
        // exclusive scan of len over the block
        int incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int o = __shfl_up(incl, d, 64);
          if (lane >= d) incl += o;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        if (tid == 0) {
          int acc = 0;
          for (int w = 0; w < NW; ++w) {
            const int v = s_wsum[w];
            s_wsum[w] = acc;
            acc += v;
          }
          s_tot = acc;
        }
        __syncthreads();
        s_pre[tid] = s_wsum[wave] + incl - len;
        s_lo[tid] = lo;
        s_ri[tid] = (uint8_t)ri;
        __syncthreads();
        const int total = s_tot;
        const int nu = (int)min<int64_t>(SM_NT, moff[i + 1] - t0);
        // SM_U entries per thread: their (movie, rating) loads all issued
        // before the first is used (one load pair, one wait and two LDS
        // atomics per trip kept one entry per thread in flight); integer
        // atomics, so the order does not matter
        auto locate = [&](int e, int& p, unsigned& rk) {
          int a = 0, b = nu;   // last rater k with s_pre[k] <= e
          while (b - a > 1) {
            const int mid = (a + b) >> 1;
            if (s_pre[mid] <= e) a = mid;
            else b = mid;
          }
          p = s_lo[a] + (e - s_pre[a]);
          rk = s_ri[a];
        };
        auto add = [&](int jj, unsigned rk, unsigned rj) {
          atomicAdd(&accA[jj], ((unsigned long long)(rk * rj) << 32) | 1ull);
          atomicAdd(&accB[jj], ((unsigned long long)(rk * rk) << 32) | (unsigned long long)(rj * rj));
        };
        int e = tid;
        for (; e + (SM_U - 1) * SM_NT < total; e += SM_U * SM_NT) {
          int pp[SM_U];
          unsigned rkk[SM_U];
#pragma unroll
          for (int j = 0; j < SM_U; ++j) locate(e + j * SM_NT, pp[j], rkk[j]);
          int jv[SM_U];
          unsigned rjv[SM_U];
#pragma unroll
          for (int j = 0; j < SM_U; ++j) {
            jv[j] = umov[pp[j]];
            rjv[j] = ur2[pp[j]];
          }
#pragma unroll
          for (int j = 0; j < SM_U; ++j) add(jv[j] - base, rkk[j], rjv[j]);
        }
        for (; e < total; e += SM_NT) {
          int p;
          unsigned rk;
          locate(e, p, rk);
          add(umov[p] - base, rk, ur2[p]);
        }
        __syncthreads();
      }
    }
    __syncthreads();
    for (int c0 = 0; c0 < SM_RS; c0 += SM_NT) {
      if (s_nbuf + SM_NT > SM_CAP) {   // block-uniform: keep the T with most reviewers
        block_sort(cj, cn, cs, s_nbuf, 0);
        if (tid == 0) s_nbuf = min(s_nbuf, T);
        __syncthreads();
      }
      const int jj = c0 + tid, j = base + jj;
      if (hi_ok && j < M && j != i && ghas[j]) {
        const unsigned long long a = accA[jj];
        const int n = (int)(a & 0xffffffffull);
        const unsigned long long gj = gmask[j];
        const int lj = __popcll(gj);
        // _genres_similar: matches / len(shorter set) >= 0.5
        if (n >= 3 && 2 * __popcll(gi & gj) >= min(li, lj)) {
          const unsigned long long b = accB[jj];
          const double D = (double)(a >> 32) * 0.25;
          const double A = (double)(b >> 32) * 0.25, B = (double)(b & 0xffffffffull) * 0.25;
          const double sim = D / (sqrt(A) * sqrt(B));
          const double score = sim * boost1[min(n, n_boost - 1)];
          if (score > 0.3) {
            const int slot = atomicAdd(&s_nbuf, 1);
            cj[slot] = j;
            cn[slot] = n;
            cs[slot] = score;
            atomicAdd((unsigned long long*)&s_total, 1ull);
          }
        }
      }
      __syncthreads();
    }
  }
  int mode = 1;
  if (s_total > T) {   // find_similar_movie:146-148
    block_sort(cj, cn, cs, s_nbuf, 0);
    if (tid == 0) s_nbuf = min(s_nbuf, T);
    __syncthreads();
    mode = 2;
  }
  const int cnt = s_nbuf;
  block_sort(cj, cn, cs, cnt, mode);
  const int k = min(cnt, nres);
  for (int t = tid; t < k; t += SM_NT) {
    out_j[(int64_t)q * nres + t] = cj[t];
    out_s[(int64_t)q * nres + t] = cs[t];
  }
  if (tid == 0) out_cnt[q] = k;
}

// ---------------------------------------------------------------------------
struct Similar {
  int device = 0, M = 0, U = 0, NR = 0;
  int64_t nnz = 0;
  hipStream_t s = nullptr;
  int64_t* moff = nullptr;
  int* muser = nullptr;
  uint8_t* mr2 = nullptr;
  int* umov = nullptr;
  uint8_t* ur2 = nullptr;
  int* ustart = nullptr;
  unsigned long long* gmask = nullptr;
  uint8_t* ghas = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  double ms = 0.0;
  ~Similar() {
    if (s) {
      (void)hipFree(moff);
      (void)hipFree(muser);
      (void)hipFree(mr2);
      (void)hipFree(umov);
      (void)hipFree(ur2);
      (void)hipFree(ustart);
      (void)hipFree(gmask);
      (void)hipFree(ghas);
      (void)hipStreamDestroy(s);
    }
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

template <typename T>
struct SBuf {
  T* p = nullptr;
  ~SBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(int64_t n) {
    MR_HIP(hipMalloc((void**)&p, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
    return 0;
  }
};

static int sim_init(Similar* S, int device, int M, int U, const long long* off, const int* user,
                    const uint8_t* r2, const unsigned long long* gmask, const uint8_t* ghas) {
  MR_CHECK(M >= 0 && U >= 0 && M < (1 << 24), "similar: 0 <= n_movies < 2^24 required");
  const int64_t nnz = off[M];
  MR_CHECK(off[0] == 0 && nnz >= 0 && nnz < (1LL << 31), "similar: bad offsets");
  int max_r2 = 0;
  int64_t max_deg = 0;
  for (int m = 0; m < M; ++m) {
    MR_CHECK(off[m + 1] >= off[m], "similar: offsets must not decrease");
    max_deg = std::max<int64_t>(max_deg, off[m + 1] - off[m]);
  }
  for (int64_t p = 0; p < nnz; ++p) {
    MR_CHECK(user[p] >= 0 && user[p] < U, "similar: user index out of range");
    max_r2 = std::max<int>(max_r2, r2[p]);
  }
  // sums per pair: n <= common raters, A, B, D <= max_r2^2 * common raters
  MR_CHECK((double)max_r2 * max_r2 * (double)max_deg < 4294967295.0,
           "similar: rating sums would overflow 32-bit fields");
  S->device = device;
  S->M = M;
  S->U = U;
  S->nnz = nnz;
  S->NR = (M + SM_RS - 1) / SM_RS;
  MR_HIP(hipSetDevice(device));
  MR_HIP(hipStreamCreateWithFlags(&S->s, hipStreamNonBlocking));
  MR_HIP(hipEventCreate(&S->ev[0]));
  MR_HIP(hipEventCreate(&S->ev[1]));
  const size_t nn = std::max<int64_t>(nnz, 1), mm = std::max(M, 1);
  MR_HIP(hipMalloc((void**)&S->moff, (mm + 1) * 8));
  MR_HIP(hipMalloc((void**)&S->muser, nn * 4));
  MR_HIP(hipMalloc((void**)&S->mr2, nn));
  MR_HIP(hipMalloc((void**)&S->umov, nn * 4));
  MR_HIP(hipMalloc((void**)&S->ur2, nn));
  MR_HIP(hipMalloc((void**)&S->ustart, (size_t)std::max(U, 1) * (S->NR + 1) * 4));
  MR_HIP(hipMalloc((void**)&S->gmask, mm * 8));
  MR_HIP(hipMalloc((void**)&S->ghas, mm));
  MR_H2D(S->moff, off, ((size_t)M + 1) * 8, S->s);
  if (nnz) {
    MR_H2D(S->muser, user, nnz * 4, S->s);
    MR_H2D(S->mr2, r2, nnz, S->s);
  }
  if (M) {
    MR_H2D(S->gmask, gmask, (size_t)M * 8, S->s);
    MR_H2D(S->ghas, ghas, M, S->s);
  }
  // user lists sorted by movie index (one 64-bit radix sort)
  SBuf<uint64_t> k0, k1;
  SBuf<int> uu;
  SBuf<int64_t> uoff;
  if (k0.alloc(nnz) || k1.alloc(nnz) || uu.alloc(nnz) || uoff.alloc((int64_t)U + 1)) return -1;
  if (nnz) {
    sim_pack_kernel<<<std::min(M, 65535), 256, 0, S->s>>>(M, S->moff, S->muser, S->mr2, k0.p);
    size_t tb = 0;
    MR_HIP(rocprim::radix_sort_keys(nullptr, tb, k0.p, k1.p, (size_t)nnz, 0, 64, S->s));
    SBuf<char> tmp;
    if (tmp.alloc((int64_t)tb)) return -1;
    MR_HIP(rocprim::radix_sort_keys(tmp.p, tb, k0.p, k1.p, (size_t)nnz, 0, 64, S->s));
    sim_unpack_kernel<<<sgrid(nnz), 256, 0, S->s>>>(nnz, k1.p, S->umov, S->ur2, uu.p);
    MR_HIP(hipStreamSynchronize(S->s));
  }
  sim_user_offsets_kernel<<<sgrid(nnz), 256, 0, S->s>>>(nnz, U, uu.p, uoff.p);
  if (U) sim_range_start_kernel<<<sgrid(U), 256, 0, S->s>>>(U, S->NR, uoff.p, S->umov, S->ustart);
  MR_HIP(hipGetLastError());
  MR_HIP(hipStreamSynchronize(S->s));
  return 0;
}

static int sim_find(Similar* S, int n_query, const int* query, const double* boost1, int n_boost,
                    int nres, int* out_j, double* out_s, int* out_cnt) {
  MR_CHECK(nres >= 1 && nres * 20 <= SM_CAP / 2, "similar: num_results must be in 1..51");
  MR_CHECK(n_boost >= 1, "similar: boost table is empty");
  MR_CHECK(query || n_query == S->M, "similar: query == NULL needs n_query == n_movies");
  if (query)
    for (int q = 0; q < n_query; ++q)
      MR_CHECK(query[q] >= 0 && query[q] < S->M, "similar: query index out of range");
  if (n_query == 0) return 0;
  SBuf<int> dq, dj, dc;
  SBuf<double> db, ds;
  if ((query && dq.alloc(n_query)) || db.alloc(n_boost) || dj.alloc((int64_t)n_query * nres) ||
      ds.alloc((int64_t)n_query * nres) || dc.alloc(n_query))
    return -1;
  if (query) MR_H2D(dq.p, query, n_query * 4, S->s);
  MR_H2D(db.p, boost1, (size_t)n_boost * 8, S->s);
  const size_t lds = 2 * SM_RS * 8 + SM_CAP * (4 + 4 + 8);
  MR_HIP(hipFuncSetAttribute((const void*)sim_find_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  MR_HIP(hipEventRecord(S->ev[0], S->s));
  sim_find_kernel<<<n_query, SM_NT, lds, S->s>>>(S->M, S->NR, query ? dq.p : nullptr, S->moff,
                                                 S->muser, S->mr2, S->umov, S->ur2, S->ustart,
                                                 S->gmask, S->ghas, db.p, n_boost, nres * 20,
                                                 nres, dj.p, ds.p, dc.p);
  MR_HIP(hipGetLastError());
  MR_HIP(hipEventRecord(S->ev[1], S->s));
  MR_D2H(out_j, dj.p, (size_t)n_query * nres * 4, S->s);
  MR_D2H(out_s, ds.p, (size_t)n_query * nres * 8, S->s);
  MR_D2H(out_cnt, dc.p, (size_t)n_query * 4, S->s);
  MR_HIP(hipStreamSynchronize(S->s));
  float t = 0.f;
  MR_HIP(hipEventElapsedTime(&t, S->ev[0], S->ev[1]));
  S->ms = t;
  return 0;
}

}  // namespace mr

struct mr_similar {
  mr::Similar s;
};

namespace {
template <typename F>
int sim_guard(F&& f) {
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

mr_similar* mr_similar_create(int device, int n_movies, int n_users, const long long* off,
                              const int* user, const unsigned char* rating2,
                              const unsigned long long* genre_mask,
                              const unsigned char* has_genres) {
  mr_similar* ctx = nullptr;
  const int rc = sim_guard([&]() -> int {
    ctx = new mr_similar();
    return mr::sim_init(&ctx->s, device, n_movies, n_users, off, user, rating2, genre_mask,
                        has_genres);
  });
  if (rc) {
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void mr_similar_destroy(mr_similar* ctx) { delete ctx; }

int mr_similar_find(mr_similar* ctx, int n_query, const int* query, const double* boost1,
                    int n_boost, int num_results, int* out_index, double* out_score,
                    int* out_count) {
  if (!ctx) return -1;
  return sim_guard([&]() {
    return mr::sim_find(&ctx->s, n_query, query, boost1, n_boost, num_results, out_index,
                        out_score, out_count);
  });
}

double mr_similar_last_ms(const mr_similar* ctx) { return ctx ? ctx->s.ms : -1.0; }

}  // extern "C"
