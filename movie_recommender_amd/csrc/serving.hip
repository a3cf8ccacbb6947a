// Factor consumers on MI355X (gfx950): fold-in, scoring, top-N, evaluation.
// C ABI: include/mr_serving.h.  Reference behaviour:
//   fold-in   python/app_local/models.py:657-700
//   predict   python/app_local/models.py:708-733 (== full_data/als_predictor.py:35-60)
//   top-N     python/app_local/recommend.py:86-110
//   eval      python/full_data/worker_process.py:229-306, my_util.py:101-145
//
// Scores are fp64 in the reference's order: s = 0; s += u_i * v_i for
// i = 0..k-1 (separate, correctly rounded multiply and add -- no FMA); s += bias;
// s += median.  That makes every score bit-identical to the Python
// reference, so rankings, exclusions and agreement counts are exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/mr_als.h"
#include "../../include/mr_serving.h"
#include "mr_internal.h"

namespace mr {

// ---------------------------------------------------------------------------
// fp64 helpers
// ---------------------------------------------------------------------------
// The reference's Python evaluates u*v and s + (u*v) as two correctly rounded
// operations.  hipcc contracts a*b + c into v_fmac_f64 by default, which
// changes the last bit, so contraction is switched off for these two.
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

// Order-preserving 64-bit key of a score (larger score -> larger key); -0.0
// and +0.0 map to the same key as they compare equal in Python's sort.  Key 0
// is reserved for "excluded" (it would be a negative NaN with every bit set).
__device__ __forceinline__ uint64_t score_key(double s) {
  if (s == 0.0) s = 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(s);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_score(uint64_t key) {
  const uint64_t b = (key >> 63) ? (key & 0x7fffffffffffffffull) : ~key;
  return __longlong_as_double((long long)b);
}

template <typename T>
__device__ __forceinline__ T wave_sum_t(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum (fixed order: per-wave butterfly, then waves in order).
template <typename T, int NT>
__device__ T block_sum_t(T v, T* sh) {
  v = wave_sum_t(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  T t = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += sh[i];
  return t;
}

// ---------------------------------------------------------------------------
// K-S1: scores of a tile of 32 users x 256 candidates (exact reference order).
// Thread (tx = lane, ty = wave) owns users ty*8 .. ty*8+7 and candidates
// tx + 64q, q = 0..3: 32 fp64 accumulators.  User rows are wave-uniform LDS
// broadcasts; candidate rows are staged 16 factors at a time.
// ---------------------------------------------------------------------------
constexpr int SC_U = 32, SC_C = 256, SC_KC = 16;
typedef uint32_t sc_u32x2 __attribute__((ext_vector_type(2)));

template <bool KEYS>
__global__ __launch_bounds__(256) void rec_score_kernel(
    int n_users, int n_cand, int k, const double* __restrict__ X,
    const double* __restrict__ Vc, const double* __restrict__ med, void* __restrict__ out,
    int64_t ld, unsigned long long* __restrict__ kmin, unsigned long long* __restrict__ kmax) {
  // LDS tiles factor-major: the j loop reads the 8 users' values of one
  // factor as ds_read_b128 broadcasts and the 4 candidates conflict-free;
  // rows padded so the staging writes (16 lanes, one factor each) spread
  // over the banks
  __shared__ __attribute__((aligned(16))) double xs[SC_KC][SC_U + 2];
  __shared__ double vs[SC_KC][SC_C + 1];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  // user tile fastest: the blocks in flight share a few candidate tiles
  // (each XCD's L2 holds the current 128 KB V tile) instead of streaming all
  // of V; probe: 0.49 -> 0.52 of the no-FMA ceiling with the LDS change
  const int u0 = blockIdx.x * SC_U, c0 = blockIdx.y * SC_C;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  // staging: thread owns factor column jj = tid & 15 of rows (tid >> 4) + 16 i.
  // The next k-chunk is loaded into registers while this one is multiplied
  // (one chunk ahead), so the L2 / MALL latency of the staging loads overlaps
  // the arithmetic; LDS holds only the current chunk.
  const int jj = tid & 15, rr = tid >> 4;
  static_assert(SC_U * SC_KC / 2 == 256, "one x pair per thread");
  double vreg[SC_C / 16], xreg[2];
  auto load_chunk = [&](int j0) {
    const int kc = min(SC_KC, k - j0);
    const bool jok = jj < kc;
    const double* src = Vc + (int64_t)(c0 + rr) * k + j0 + jj;
#pragma unroll
    for (int i = 0; i < SC_C / 16; ++i) {
      const bool ok = jok && (c0 + rr + 16 * i) < n_cand;
      vreg[i] = ok ? src[(int64_t)16 * i * k] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = rr + 16 * i, u = u0 + r;
      xreg[i] = (jok && u < n_users) ? X[(int64_t)u * (k + 1) + j0 + jj] : 0.0;
    }
  };
  load_chunk(0);
  for (int j0 = 0; j0 < k; j0 += SC_KC) {
    const int kc = min(SC_KC, k - j0);
#pragma unroll
    for (int i = 0; i < SC_C / 16; ++i) vs[jj][rr + 16 * i] = vreg[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) xs[jj][rr + 16 * i] = xreg[i];
    __syncthreads();
    if (j0 + SC_KC < k) load_chunk(j0 + SC_KC);
    for (int j = 0; j < kc; ++j) {
      double xv[8], vv[4];
      const double2* xp = reinterpret_cast<const double2*>(&xs[j][ty * 8]);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const double2 t = xp[p];
        xv[2 * p] = t.x;
        xv[2 * p + 1] = t.y;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = vs[j][tx + 64 * q];
      // products first (16 independent multiplies in flight), then the adds
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double pr[4][4];
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
          for (int q = 0; q < 4; ++q) pr[p][q] = mul_rn(xv[4 * h + p], vv[q]);
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[4 * h + p][q] = add_rn(acc[4 * h + p][q], pr[p][q]);
      }
    }
    __syncthreads();
  }
  // Epilogue, branch-free but for the wave-uniform user test: the 8 users'
  // biases and the 4 candidates' medians are loaded together (clamped
  // indices) before any use, and each user's row goes out through a buffer
  // resource ending at n_cand, so a candidate past the end is a store the
  // hardware drops, not a branch.  With per-(user, candidate) range tests the
  // wait-count pass put a vmcnt(0) at every store's block -- each one waited
  // for the previous stores and atomics to complete, 32 serialized memory
  // round trips per thread.
  double medv[4], biasv[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + tx + 64 * q;
    medv[q] = med[c < n_cand ? c : n_cand - 1];
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    biasv[p] = X[(int64_t)(u < n_users ? u : n_users - 1) * (k + 1) + k];
  }
  const int nrow = n_cand - c0;   // candidates of this tile in range (> 0)
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = __builtin_amdgcn_readfirstlane(u0 + ty * 8 + p);   // wave-uniform
    if (u >= n_users) continue;
    const __amdgpu_buffer_rsrc_t row = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char*>(out) + ((int64_t)u * ld + c0) * 8, (short)0,
        (int)(min(nrow, SC_C) * 8), 0x00020000);
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cl = tx + 64 * q;   // candidate c0 + cl
      const double s = add_rn(add_rn(acc[p][q], biasv[p]), medv[q]);
      if constexpr (KEYS) {
        const uint64_t key = score_key(s);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(sc_u32x2, key), row, cl * 8, 0, 0);
        const bool ok = cl < nrow;
        lo = min(lo, ok ? (unsigned long long)key : ~0ull);
        hi = max(hi, ok ? (unsigned long long)key : 0ull);
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(sc_u32x2, s), row, cl * 8, 0, 0);
      }
    }
    if constexpr (KEYS) {   // per-user key range: the select skips the common prefix
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (unsigned long long)__shfl_xor(lo, o, 64));
        hi = max(hi, (unsigned long long)__shfl_xor(hi, o, 64));
      }
      if (tx == 0) {
        atomicMin(&kmin[u], lo);
        atomicMax(&kmax[u], hi);
      }
    }
  }
}

__global__ void rec_range_init_kernel(int n, unsigned long long* kmin, unsigned long long* kmax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    kmin[i] = ~0ull;
    kmax[i] = 0ull;
  }
}

// K-S2: the user's rated movies are not recommended (recommend.py:99).
__global__ __launch_bounds__(256) void rec_exclude_kernel(uint64_t* __restrict__ keys,
                                                          int64_t ld,
                                                          const int64_t* __restrict__ off,
                                                          const int* __restrict__ cand) {
  const int u = blockIdx.x;
  // 4 candidate ids loaded before the stores: with a store pending every
  // load wait is a full drain, so one id per trip serialized the stores
  const int64_t e = off[u + 1];
  int64_t i = off[u] + threadIdx.x;
  for (; i + 3 * (int64_t)blockDim.x < e; i += 4 * (int64_t)blockDim.x) {
    int c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = cand[i + j * (int64_t)blockDim.x];
#pragma unroll
    for (int j = 0; j < 4; ++j) keys[(int64_t)u * ld + c[j]] = 0;
  }
  for (; i < e; i += blockDim.x) keys[(int64_t)u * ld + cand[i]] = 0;
}

// ---------------------------------------------------------------------------
// K-S3: exact top-N per user by MSB radix select on the composite
// (score key, movie id) -- the order of Python's sort(reverse=True) on
// (score, movie_id) tuples, held as a 128-bit integer key:mid:0 -- then a
// bitonic sort of the <= CAP survivors in LDS.  The select starts at the
// first bit where the user's smallest and largest keys differ (the score
// kernel records the range), takes 11-bit digits, and stops at the first
// level where every element at or above the boundary bin fits in CAP; on
// MovieLens-like scores that is one histogram pass and one collect pass.
// ---------------------------------------------------------------------------
constexpr int SEL_NT = 512, SEL_CAP = 2048, SEL_D = 11, SEL_BINS = 1 << SEL_D;
#ifndef MR_SEL_U
#define MR_SEL_U 4
#endif
constexpr int SEL_U = MR_SEL_U;   // keys in flight per thread in the passes over a user's row
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 composite(uint64_t key, uint32_t mid) {
  return ((u128)key << 64) | ((u128)mid << 32);
}

__global__ __launch_bounds__(SEL_NT) void rec_select_kernel(
    const uint64_t* __restrict__ keys, int64_t ld, int n_cand, const int* __restrict__ mid,
    const unsigned long long* __restrict__ kmin, const unsigned long long* __restrict__ kmax,
    int N, int* __restrict__ out_mid, double* __restrict__ out_score,
    int* __restrict__ out_count) {
  __shared__ uint32_t hist[SEL_BINS];
  __shared__ uint64_t ck[SEL_CAP];
  __shared__ uint32_t cm[SEL_CAP];
  __shared__ int s_b, s_stop, s_n;
  __shared__ long long s_gt;
  const int u = blockIdx.x, tid = threadIdx.x;
  const uint64_t* K = keys + (int64_t)u * ld;
  // Fast path: SEL_BINS equal-width score bins over the user's [min, max]
  // (a monotone map, so the boundary bin is exact); one histogram pass, then
  // collect bins >= boundary if they fit.  Else the radix select below.
  const double smin = key_score(kmin[u]), smax = key_score(kmax[u]);
  const double scale = (double)SEL_BINS / (smax - smin);
  const bool lin = smax > smin && isfinite(scale);
  auto bin_of = [&](uint64_t key) {
    return min(SEL_BINS - 1, (int)((key_score(key) - smin) * scale));
  };
  int lin_b = -1;
  if (lin) {
    for (int i = tid; i < SEL_BINS; i += SEL_NT) hist[i] = 0;
    __syncthreads();
    // SEL_U keys per thread in flight before any is used (one load, one
    // wait and one LDS atomic per trip left a block one 512-thread row of
    // keys in flight); counts are order-free, so the result is unchanged
    int c = tid;
    for (; c + (SEL_U - 1) * SEL_NT < n_cand; c += SEL_U * SEL_NT) {
      uint64_t kk[SEL_U];
#pragma unroll
      for (int j = 0; j < SEL_U; ++j) kk[j] = K[c + j * SEL_NT];
#pragma unroll
      for (int j = 0; j < SEL_U; ++j)
        if (kk[j] != 0) atomicAdd(&hist[bin_of(kk[j])], 1u);
    }
    for (; c < n_cand; c += SEL_NT) {
      const uint64_t key = K[c];
      if (key != 0) atomicAdd(&hist[bin_of(key)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      long long cum = 0;
      int b = SEL_BINS - 1;
      for (; b > 0; --b) {
        if (cum + hist[b] >= N) break;
        cum += hist[b];
      }
      s_b = (cum + hist[b] <= SEL_CAP) ? b : -1;
    }
    __syncthreads();
    lin_b = s_b;
    __syncthreads();
  }
  // bits above `pos` (counted from the MSB of the 128-bit composite) are
  // common to every element: the first differing bit of the key range, or the
  // movie-id part when all keys are equal
  const uint64_t dk = kmin[u] ^ kmax[u];
  int pos = dk ? __clzll((long long)dk) : 64;
  u128 P = composite(kmin[u], 0) & ~(~(u128)0 >> pos);   // common prefix
  u128 Msk = ~(~(u128)0 >> pos);
  long long above = 0;   // elements strictly above the prefix range
  while (lin_b < 0) {
    const int D = min(SEL_D, 96 - pos);
    const int sh = 128 - pos - D;
    for (int i = tid; i < SEL_BINS; i += SEL_NT) hist[i] = 0;
    __syncthreads();
    for (int c = tid; c < n_cand; c += SEL_NT) {
      const uint64_t key = K[c];
      if (key == 0) continue;
      const u128 x = composite(key, (uint32_t)mid[c]);
      if ((x & Msk) != P) continue;
      atomicAdd(&hist[(uint32_t)(x >> sh) & ((1u << D) - 1)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      long long cum = 0;   // elements in bins above b
      int b = (1 << D) - 1;
      for (; b > 0; --b) {   // ends at bin 0 when fewer than N remain: take all
        if (above + cum + hist[b] >= N) break;
        cum += hist[b];
      }
      s_b = b;
      s_gt = cum;
      s_stop = (above + cum + hist[b] <= SEL_CAP || pos + D >= 96) ? 1 : 0;
    }
    __syncthreads();
    const int b = s_b;
    P |= (u128)b << sh;   // lower bound of the boundary bin (lower bits zero)
    Msk |= (((u128)1 << D) - 1) << sh;
    pos += D;
    const bool stop = s_stop != 0;
    const long long gt = s_gt;
    __syncthreads();
    if (stop) break;
    above += gt;
  }
  // collect every element with composite >= P
  if (tid == 0) s_n = 0;
  __syncthreads();
  // (SEL_U keys and ids in flight per thread, as in the histogram; the slot
  // order depends on the atomics' order, the sort below fixes the result)
  auto take = [&](uint64_t key, uint32_t m) {
    if (key == 0) return;
    if (lin_b >= 0 ? bin_of(key) >= lin_b : composite(key, m) >= P) {
      const int slot = atomicAdd(&s_n, 1);
      if (slot < SEL_CAP) {
        ck[slot] = key;
        cm[slot] = m;
      }
    }
  };
  {
    int c = tid;
    for (; c + (SEL_U - 1) * SEL_NT < n_cand; c += SEL_U * SEL_NT) {
      uint64_t kk[SEL_U];
      uint32_t mm[SEL_U];
#pragma unroll
      for (int j = 0; j < SEL_U; ++j) {
        kk[j] = K[c + j * SEL_NT];
        mm[j] = (uint32_t)mid[c + j * SEL_NT];
      }
#pragma unroll
      for (int j = 0; j < SEL_U; ++j) take(kk[j], mm[j]);
    }
    for (; c < n_cand; c += SEL_NT) take(K[c], (uint32_t)mid[c]);
  }
  __syncthreads();
  const int n = min(s_n, SEL_CAP);
  int sz = 64;
  while (sz < n) sz <<= 1;
  for (int i = n + tid; i < sz; i += SEL_NT) {
    ck[i] = 0;
    cm[i] = 0;
  }
  __syncthreads();
  // bitonic sort, descending by (key, mid)
  for (int w = 2; w <= sz; w <<= 1) {
    for (int j = w >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < sz; i += SEL_NT) {
        const int l = i ^ j;
        if (l > i) {
          const bool desc = (i & w) == 0;
          const uint64_t ka = ck[i], kb = ck[l];
          const uint32_t ma = cm[i], mb = cm[l];
          const bool a_less = ka < kb || (ka == kb && ma < mb);
          if (a_less == desc) {
            ck[i] = kb;
            ck[l] = ka;
            cm[i] = mb;
            cm[l] = ma;
          }
        }
      }
      __syncthreads();
    }
  }
  const int cnt = min(n, N);
  for (int i = tid; i < cnt; i += SEL_NT) {
    out_mid[(int64_t)u * N + i] = (int)cm[i];
    out_score[(int64_t)u * N + i] = key_score(ck[i]);
  }
  if (tid == 0) out_count[u] = (s_n > SEL_CAP) ? -1 : cnt;
}

// ---------------------------------------------------------------------------
// K-S4: fold-in normal equations + Cholesky, one block per user.
// Rows [V_m, 1 | r] are staged FI_R at a time; each thread owns NE entries of
// the upper triangle of [G | c] (K = k+1 columns + rhs) and accumulates them
// in registers in row order; then G is formed in LDS and factored.
// Pivot ratio below `cond_limit` (or a non-positive pivot) flags the user for
// the SVD path (method 2).
// ---------------------------------------------------------------------------
constexpr int FI_NE = 9;   // entries per thread per pass (no spills at 256 threads)

__global__ __launch_bounds__(256) void fold_in_kernel(
    int k, int rows_per_stage, const int64_t* __restrict__ off,
    const int* __restrict__ als_idx, const double* __restrict__ rating,
    const double* __restrict__ V, double* __restrict__ X, int* __restrict__ method,
    double cond_limit) {
  extern __shared__ double lds[];
  __shared__ int s_bad;
  __shared__ double s_pmin, s_pmax;
  const int K = k + 1, W = K + 1;   // row width: k factors, 1, rating
  const int u = blockIdx.x, tid = threadIdx.x;
  const int64_t b = off[u];
  const int M = (int)(off[u + 1] - b);
  const int T = K * (K + 1) / 2;
  double* G = lds;                  // [K][W]: G and the rhs in column K
  double* As = lds + K * W;         // [rows_per_stage][W]
  // passes over the rows, FI_NE * 256 entries of [G | c] each (one pass for k <= 63)
  for (int g0 = 0; g0 < T + K; g0 += 256 * FI_NE) {
    int ei[FI_NE], ej[FI_NE];
    double acc[FI_NE];
#pragma unroll
    for (int t = 0; t < FI_NE; ++t) {
      int f = g0 + tid + 256 * t;
      acc[t] = 0.0;
      ei[t] = -1;
      ej[t] = -1;
      if (f < T) {
        int i = 0, len = K;
        while (f >= len) {
          f -= len;
          ++i;
          --len;
        }
        ei[t] = i;
        ej[t] = i + f;
      } else if (f < T + K) {
        ei[t] = f - T;
        ej[t] = K;   // rhs column (the rating)
      }
    }
    for (int r0 = 0; r0 < M; r0 += rows_per_stage) {
      const int nr = min(rows_per_stage, M - r0);
      for (int q = tid; q < nr * W; q += 256) {
        const int r = q / W, j = q % W;
        double v;
        if (j < k) v = V[(int64_t)als_idx[b + r0 + r] * k + j];
        else if (j == k) v = 1.0;
        else v = rating[b + r0 + r];
        As[r * W + j] = v;
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < FI_NE; ++t) {
        if (ei[t] < 0) continue;
        double s = acc[t];
        for (int r = 0; r < nr; ++r) s = fma(As[r * W + ei[t]], As[r * W + ej[t]], s);
        acc[t] = s;
      }
      __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < FI_NE; ++t) {
      if (ei[t] < 0) continue;
      G[ei[t] * W + ej[t]] = acc[t];
      if (ej[t] < K) G[ej[t] * W + ei[t]] = acc[t];
    }
  }
  if (tid == 0) {
    s_bad = 0;
    s_pmin = INFINITY;
    s_pmax = 0.0;
  }
  __syncthreads();
  for (int j = 0; j < K; ++j) {
    if (tid == 0) {
      const double d = G[j * W + j];
      if (!(d > 0.0)) {
        s_bad = 1;
      } else {
        s_pmin = fmin(s_pmin, d);
        s_pmax = fmax(s_pmax, d);
        G[j * W + j] = sqrt(d);
      }
    }
    __syncthreads();
    if (s_bad) break;
    const double ljj = G[j * W + j];
    for (int i = j + 1 + tid; i < K; i += 256) G[i * W + j] /= ljj;
    __syncthreads();
    const int m = K - j - 1;
    for (int q = tid; q < m * m; q += 256) {
      const int ii = j + 1 + q / m, ll = j + 1 + q % m;
      if (ll <= ii) G[ii * W + ll] -= G[ii * W + j] * G[ll * W + j];
    }
    __syncthreads();
  }
  const bool bad = s_bad || s_pmin < cond_limit * s_pmax;
  if (bad) {
    if (tid == 0) method[u] = 2;
    return;
  }
  // L y = c (right-looking), then L^T x = y
  for (int p = 0; p < K; ++p) {
    if (tid == 0) G[p * W + K] /= G[p * W + p];
    __syncthreads();
    for (int i = p + 1 + tid; i < K; i += 256) G[i * W + K] -= G[i * W + p] * G[p * W + K];
    __syncthreads();
  }
  for (int p = K - 1; p >= 0; --p) {
    if (tid == 0) G[p * W + K] /= G[p * W + p];
    __syncthreads();
    for (int i = tid; i < p; i += 256) G[i * W + K] -= G[p * W + i] * G[p * W + K];
    __syncthreads();
  }
  for (int i = tid; i < K; i += 256) X[(int64_t)u * K + i] = G[i * W + K];
  if (tid == 0) method[u] = 1;
}

// ---------------------------------------------------------------------------
// K-S5: minimum-norm least squares by one-sided (Hestenes) Jacobi SVD for the
// users the Cholesky path flagged.  A (M x K, column-major) lives in global
// scratch, the right singular vectors in LDS.  Singular values at or below
// eps * max(M, K) * s_max are dropped -- numpy.linalg.lstsq(rcond=None).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fold_in_svd_kernel(
    const int* __restrict__ users, int k, const int64_t* __restrict__ off,
    const int* __restrict__ als_idx, const double* __restrict__ rating,
    const double* __restrict__ V, double* __restrict__ scratch,
    const int64_t* __restrict__ scr_off, double* __restrict__ X) {
  extern __shared__ double Vm[];   // [K][K]
  __shared__ double sh[3][4];
  __shared__ int s_rot;
  const int K = k + 1, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int u = users[blockIdx.x];
  const int64_t b = off[u];
  const int M = (int)(off[u + 1] - b);
  double* A = scratch + scr_off[blockIdx.x];
  double* bv = A + (int64_t)K * M;
  for (int r = tid; r < M; r += 256) {
    const int64_t m = als_idx[b + r];
    for (int j = 0; j < k; ++j) A[(int64_t)j * M + r] = V[m * k + j];
    A[(int64_t)k * M + r] = 1.0;
    bv[r] = rating[b + r];
  }
  for (int i = tid; i < K * K; i += 256) Vm[i] = (i / K == i % K) ? 1.0 : 0.0;
  __syncthreads();
  auto sum3 = [&](double& x, double& y, double& z) {
    x = wave_sum_t(x);
    y = wave_sum_t(y);
    z = wave_sum_t(z);
    if (lane == 0) {
      sh[0][w] = x;
      sh[1][w] = y;
      sh[2][w] = z;
    }
    __syncthreads();
    x = (sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3]);
    y = (sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3]);
    z = (sh[2][0] + sh[2][1]) + (sh[2][2] + sh[2][3]);
    __syncthreads();
  };
  for (int sweep = 0; sweep < 60; ++sweep) {
    if (tid == 0) s_rot = 0;
    __syncthreads();
    for (int p = 0; p < K - 1; ++p) {
      for (int q = p + 1; q < K; ++q) {
        double* ap = A + (int64_t)p * M;
        double* aq = A + (int64_t)q * M;
        double al = 0.0, be = 0.0, ga = 0.0;
        for (int r = tid; r < M; r += 256) {
          const double x = ap[r], y = aq[r];
          al = fma(x, x, al);
          be = fma(y, y, be);
          ga = fma(x, y, ga);
        }
        sum3(al, be, ga);
        if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
        const double zeta = (be - al) / (2.0 * ga);
        const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        for (int r = tid; r < M; r += 256) {
          const double x = ap[r], y = aq[r];
          ap[r] = c * x - s * y;
          aq[r] = s * x + c * y;
        }
        for (int i = tid; i < K; i += 256) {
          const double x = Vm[i * K + p], y = Vm[i * K + q];
          Vm[i * K + p] = c * x - s * y;
          Vm[i * K + q] = s * x + c * y;
        }
        if (tid == 0) s_rot = 1;
        __syncthreads();
      }
    }
    __syncthreads();
    if (!s_rot) break;
    __syncthreads();
  }
  // x = sum_i [s_i > cut] (a_i . b / s_i^2) v_i
  double smax = 0.0;
  for (int i = 0; i < K; ++i) {
    double nn = 0.0, ab = 0.0, z = 0.0;
    const double* ai = A + (int64_t)i * M;
    for (int r = tid; r < M; r += 256) {
      nn = fma(ai[r], ai[r], nn);
      ab = fma(ai[r], bv[r], ab);
    }
    sum3(nn, ab, z);
    smax = fmax(smax, sqrt(nn));
    if (tid == 0) {
      bv[M + 2 * i] = nn;   // scratch tail: |a_i|^2, a_i . b
      bv[M + 2 * i + 1] = ab;
    }
  }
  __syncthreads();
  const double cut = 2.220446049250313e-16 * (double)max(M, K) * smax;
  for (int j = tid; j < K; j += 256) {
    double x = 0.0;
    for (int i = 0; i < K; ++i) {
      const double nn = bv[M + 2 * i], ab = bv[M + 2 * i + 1];
      if (sqrt(nn) > cut) x += (ab / nn) * Vm[j * K + i];
    }
    X[(int64_t)u * K + j] = x;
  }
}

// ---------------------------------------------------------------------------
// K-S6: evaluation, one block per test user.  PRED: exact predictions of its
// test ratings (worker_process.py:245, the reference predict) written to
// `pred`; otherwise `pred` is given and NaN marks "no prediction".  Then the
// ranking-agreement pair counts (my_util.py:128-143) over the predicted
// ratings: pairs with actual_i > actual_j, agreement when pred_i > pred_j, and
// the squared error of the predictions.
// ---------------------------------------------------------------------------
constexpr int EV_CH = 1024;

template <bool PRED>
__global__ __launch_bounds__(256) void rec_eval_kernel(
    int k, const double* __restrict__ U, const int* __restrict__ user_row,
    const int64_t* __restrict__ off, const int* __restrict__ cand,
    const double* __restrict__ actual, const double* __restrict__ Vc,
    const double* __restrict__ med, double* __restrict__ pred, double* __restrict__ agreement,
    long long* __restrict__ n_agree, long long* __restrict__ n_dis, double* __restrict__ sse,
    long long* __restrict__ n_pred) {
  __shared__ double xs[kMaxK + 1];
  __shared__ double aj[EV_CH], pj[EV_CH];
  __shared__ double shd[4];
  __shared__ long long shl[4];
  const int t = blockIdx.x, tid = threadIdx.x;
  const int64_t b = off[t];
  const int n = (int)(off[t + 1] - b);
  double e2 = 0.0;
  long long np = 0;
  if constexpr (PRED) {
    const double* x = U + (int64_t)user_row[t] * (k + 1);
    for (int j = tid; j <= k; j += 256) xs[j] = x[j];
    __syncthreads();
  }
  for (int i = tid; i < n; i += 256) {
    double p;
    if constexpr (PRED) {
      const int c = cand[b + i];
      p = NAN;
      if (c >= 0) {
        const double* v = Vc + (int64_t)c * k;
        double s = 0.0;
        for (int j = 0; j < k; ++j) s = add_rn(s, mul_rn(xs[j], v[j]));
        p = add_rn(add_rn(s, xs[k]), med[c]);
      }
      pred[b + i] = p;
    } else {
      p = pred[b + i];
    }
    if (!isnan(p)) {
      const double d = p - actual[b + i];
      e2 = fma(d, d, e2);
      ++np;
    }
  }
  __syncthreads();   // pred visible block-wide
  long long agree = 0, total = 0;
  for (int j0 = 0; j0 < n; j0 += EV_CH) {
    const int nj = min(EV_CH, n - j0);
    for (int j = tid; j < nj; j += 256) {
      const double pv = pred[b + j0 + j];
      aj[j] = isnan(pv) ? NAN : actual[b + j0 + j];   // NaN: never "below" anything
      pj[j] = pv;
    }
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
      const double pi = pred[b + i];
      if (isnan(pi)) continue;
      const double ai = actual[b + i];
      for (int j = 0; j < nj; ++j) {
        if (ai > aj[j]) {
          ++total;
          agree += (pi > pj[j]) ? 1 : 0;
        }
      }
    }
    __syncthreads();
  }
  agree = block_sum_t<long long, 256>(agree, shl);
  total = block_sum_t<long long, 256>(total, shl);
  const long long nk = block_sum_t<long long, 256>(np, shl);
  const double s2 = block_sum_t<double, 256>(e2, shd);
  if (tid == 0) {
    // None when at most one prediction (worker_process.py:251) or when the
    // actual ratings are all equal (my_util.py:111-119): no ordered pair
    n_agree[t] = agree;
    n_dis[t] = total - agree;
    agreement[t] = (nk > 1 && total > 0) ? (double)agree / (double)total : NAN;
    if (sse) sse[t] = s2;
    if (n_pred) n_pred[t] = nk;
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
enum { RT_SCORE = 0, RT_EXCL, RT_SELECT, RT_FOLD, RT_SVD, RT_EVAL, RT_N };

struct Rec {
  int device = 0, k = 0, n_als = 0, n_cand = 0;
  hipStream_t stream = nullptr;
  double *V = nullptr, *Vc = nullptr, *med = nullptr;
  int* mid = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  double ms[RT_N] = {0};
  ~Rec() {
    if (stream) {
      (void)hipFree(V);
      (void)hipFree(Vc);
      (void)hipFree(med);
      (void)hipFree(mid);
      (void)hipStreamDestroy(stream);
    }
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

template <typename T>
struct DBuf {   // call-scoped device buffer
  T* p = nullptr;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(int64_t n) {
    MR_HIP(hipMalloc((void**)&p, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
    return 0;
  }
  int upload(const T* h, int64_t n, hipStream_t s) {
    if (alloc(n)) return -1;
    if (n > 0) MR_H2D(p, h, n * sizeof(T), s);
    return 0;
  }
};

// Times one kernel class with events on the context stream (accumulated).
template <typename F>
static int timed(Rec* r, int cls, F&& launch) {
  MR_HIP(hipEventRecord(r->ev[0], r->stream));
  if (launch()) return -1;
  MR_HIP(hipGetLastError());
  MR_HIP(hipEventRecord(r->ev[1], r->stream));
  MR_HIP(hipEventSynchronize(r->ev[1]));
  float ms = 0.f;
  MR_HIP(hipEventElapsedTime(&ms, r->ev[0], r->ev[1]));
  r->ms[cls] += ms;
  return 0;
}

static int rec_init(Rec* r, int device, int k, int n_als, const double* Vh, int n_cand,
                    const int* cand_als, const int* cand_mid, const double* cand_med) {
  MR_CHECK(k >= 1 && k <= kMaxK, "rec: k must be in 1..128");
  MR_CHECK(n_als >= 0 && n_cand >= 0, "rec: negative sizes");
  std::vector<double> vc((size_t)n_cand * k);
  {
    std::vector<int> seen_mid;
    seen_mid.assign(cand_mid, cand_mid + n_cand);
    std::sort(seen_mid.begin(), seen_mid.end());
    MR_CHECK(std::adjacent_find(seen_mid.begin(), seen_mid.end()) == seen_mid.end(),
             "rec: candidate movie ids must be unique");
    MR_CHECK(n_cand == 0 || seen_mid.front() >= 0, "rec: movie ids must be >= 0");
  }
  for (int c = 0; c < n_cand; ++c) {
    MR_CHECK(cand_als[c] >= 0 && cand_als[c] < n_als, "rec: candidate ALS id out of range");
    std::memcpy(&vc[(size_t)c * k], Vh + (size_t)cand_als[c] * k, k * sizeof(double));
  }
  r->device = device;
  r->k = k;
  r->n_als = n_als;
  r->n_cand = n_cand;
  MR_HIP(hipSetDevice(device));
  MR_HIP(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
  MR_HIP(hipEventCreate(&r->ev[0]));
  MR_HIP(hipEventCreate(&r->ev[1]));
  const size_t nv = std::max<size_t>((size_t)n_als * k, 1), nc = std::max(n_cand, 1);
  MR_HIP(hipMalloc((void**)&r->V, nv * sizeof(double)));
  MR_HIP(hipMalloc((void**)&r->Vc, nc * k * sizeof(double)));
  MR_HIP(hipMalloc((void**)&r->med, nc * sizeof(double)));
  MR_HIP(hipMalloc((void**)&r->mid, nc * sizeof(int)));
  if (n_als) MR_H2D(r->V, Vh, (size_t)n_als * k * 8, r->stream);
  if (n_cand) {
    MR_H2D(r->Vc, vc.data(), vc.size() * 8, r->stream);
    MR_H2D(r->med, cand_med, (size_t)n_cand * 8, r->stream);
    MR_H2D(r->mid, cand_mid, (size_t)n_cand * 4, r->stream);
  }
  MR_HIP(hipStreamSynchronize(r->stream));
  return 0;
}

static void reset_ms(Rec* r) {
  for (double& m : r->ms) m = 0.0;
}

// users per score/select launch: bounds the key scratch to ~1 GiB
static int64_t user_chunk(const Rec* r) {
  const int64_t per = std::max<int64_t>(r->n_cand, 1) * 8;
  return std::max<int64_t>(SC_U, std::min<int64_t>(65535LL * SC_U, (1LL << 30) / per));
}

static int rec_scores(Rec* r, int n_users, const double* Xh, double* out) {
  MR_CHECK(n_users >= 0, "rec: negative n_users");
  reset_ms(r);
  if (n_users == 0 || r->n_cand == 0) return 0;
  const int K = r->k + 1;
  const int64_t B = std::min<int64_t>(user_chunk(r), n_users);
  DBuf<double> X, S;
  if (X.alloc(B * K) || S.alloc(B * r->n_cand)) return -1;
  for (int64_t u0 = 0; u0 < n_users; u0 += B) {
    const int nb = (int)std::min<int64_t>(B, n_users - u0);
    MR_H2D(X.p, Xh + u0 * K, (size_t)nb * K * 8, r->stream);
    const dim3 grid((nb + SC_U - 1) / SC_U, (r->n_cand + SC_C - 1) / SC_C);
    MR_CHECK(grid.y <= 65535, "rec: more than 65535 * 256 candidates");
    if (timed(r, RT_SCORE, [&]() {
          rec_score_kernel<false><<<grid, 256, 0, r->stream>>>(nb, r->n_cand, r->k, X.p, r->Vc,
                                                               r->med, S.p, r->n_cand, nullptr,
                                                               nullptr);
          return 0;
        }))
      return -1;
    MR_D2H(out + u0 * r->n_cand, S.p, (size_t)nb * r->n_cand * 8, r->stream);
  }
  MR_HIP(hipStreamSynchronize(r->stream));
  return 0;
}

static int rec_top_n(Rec* r, int n_users, const double* Xh, const long long* excl_off,
                     const int* excl_cand, int N, int* out_mid, double* out_score,
                     int* out_count) {
  MR_CHECK(n_users >= 0, "rec: negative n_users");
  MR_CHECK(N >= 1 && N <= SEL_CAP / 2, "rec: num_results must be in 1..1024");
  reset_ms(r);
  if (n_users == 0) return 0;
  if (r->n_cand == 0) {
    std::fill(out_count, out_count + n_users, 0);
    return 0;
  }
  const int K = r->k + 1;
  const int64_t B = std::min<int64_t>(user_chunk(r), n_users);
  DBuf<double> X, osc;
  DBuf<uint64_t> S;
  DBuf<unsigned long long> kmin, kmax;
  DBuf<int> omid, ocnt, ecand;
  DBuf<int64_t> eoff;
  if (X.alloc(B * K) || S.alloc(B * r->n_cand) || osc.alloc(B * N) || omid.alloc(B * N) ||
      ocnt.alloc(B) || eoff.alloc(B + 1) || kmin.alloc(B) || kmax.alloc(B))
    return -1;
  int64_t max_ex = 0;
  if (excl_off) {
    for (int64_t u0 = 0; u0 < n_users; u0 += B) {
      const int64_t nb = std::min<int64_t>(B, n_users - u0);
      max_ex = std::max<int64_t>(max_ex, excl_off[u0 + nb] - excl_off[u0]);
    }
    for (int64_t i = 0; i < excl_off[n_users]; ++i)
      MR_CHECK(excl_cand[i] >= 0 && excl_cand[i] < r->n_cand, "rec: excluded candidate out of range");
    if (ecand.alloc(max_ex)) return -1;
  }
  std::vector<int64_t> loc;
  for (int64_t u0 = 0; u0 < n_users; u0 += B) {
    const int nb = (int)std::min<int64_t>(B, n_users - u0);
    MR_H2D(X.p, Xh + u0 * K, (size_t)nb * K * 8, r->stream);
    const dim3 grid((nb + SC_U - 1) / SC_U, (r->n_cand + SC_C - 1) / SC_C);
    MR_CHECK(grid.y <= 65535, "rec: more than 65535 * 256 candidates");
    if (timed(r, RT_SCORE, [&]() {
          rec_range_init_kernel<<<(nb + 255) / 256, 256, 0, r->stream>>>(nb, kmin.p, kmax.p);
          rec_score_kernel<true><<<grid, 256, 0, r->stream>>>(nb, r->n_cand, r->k, X.p, r->Vc,
                                                              r->med, S.p, r->n_cand, kmin.p,
                                                              kmax.p);
          return 0;
        }))
      return -1;
    if (excl_off) {
      loc.assign(nb + 1, 0);
      for (int i = 0; i <= nb; ++i) loc[i] = excl_off[u0 + i] - excl_off[u0];
      MR_H2D(eoff.p, loc.data(), (nb + 1) * 8, r->stream);
      if (loc[nb] > 0)
        MR_H2D(ecand.p, excl_cand + excl_off[u0], loc[nb] * 4, r->stream);
      if (timed(r, RT_EXCL, [&]() {
            rec_exclude_kernel<<<nb, 256, 0, r->stream>>>(S.p, r->n_cand, eoff.p, ecand.p);
            return 0;
          }))
        return -1;
    }
    if (timed(r, RT_SELECT, [&]() {
          rec_select_kernel<<<nb, SEL_NT, 0, r->stream>>>(S.p, r->n_cand, r->n_cand, r->mid,
                                                          kmin.p, kmax.p, N, omid.p, osc.p,
                                                          ocnt.p);
          return 0;
        }))
      return -1;
    MR_D2H(out_mid + u0 * N, omid.p, (size_t)nb * N * 4, r->stream);
    MR_D2H(out_score + u0 * N, osc.p, (size_t)nb * N * 8, r->stream);
    MR_D2H(out_count + u0, ocnt.p, (size_t)nb * 4, r->stream);
  }
  MR_HIP(hipStreamSynchronize(r->stream));
  for (int u = 0; u < n_users; ++u)
    MR_CHECK(out_count[u] >= 0, "rec: top-N candidate buffer overflow (internal)");
  return 0;
}

static int rec_fold_in(Rec* r, int n_users, const long long* off, const int* als_idx,
                       const double* rating, double* Xout, int* method_out) {
  MR_CHECK(n_users >= 0, "rec: negative n_users");
  reset_ms(r);
  if (n_users == 0) return 0;
  const int k = r->k, K = k + 1;
  const int64_t nnz = off[n_users];
  for (int u = 0; u < n_users; ++u)
    MR_CHECK(off[u + 1] - off[u] >= K, "rec: fold-in needs at least k+1 rows per user");
  for (int64_t i = 0; i < nnz; ++i)
    MR_CHECK(als_idx[i] >= 0 && als_idx[i] < r->n_als, "rec: fold-in movie id out of range");
  DBuf<int64_t> doff;
  DBuf<int> didx, dmeth;
  DBuf<double> drat, dX;
  if (doff.upload(reinterpret_cast<const int64_t*>(off), n_users + 1, r->stream) ||
      didx.upload(als_idx, nnz, r->stream) || drat.upload(rating, nnz, r->stream) ||
      dX.alloc((int64_t)n_users * K) || dmeth.alloc(n_users))
    return -1;
  // LDS: G [K][K+1] plus a row stage of up to 32 rows (fewer at k = 128)
  const size_t gbytes = (size_t)K * (K + 1) * sizeof(double);
  const size_t budget = 150 * 1024;
  MR_CHECK(gbytes + 8 * (K + 1) * sizeof(double) <= budget, "rec: fold-in k too large");
  const int rows = (int)std::min<size_t>(32, (budget - gbytes) / ((K + 1) * sizeof(double)));
  const size_t lds = gbytes + (size_t)rows * (K + 1) * sizeof(double);
  const double cond_limit = 1e-8;
  if (lds > 64 * 1024)
    MR_HIP(hipFuncSetAttribute((const void*)fold_in_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (timed(r, RT_FOLD, [&]() {
        fold_in_kernel<<<n_users, 256, lds, r->stream>>>(k, rows, doff.p, didx.p, drat.p, r->V,
                                                         dX.p, dmeth.p, cond_limit);
        return 0;
      }))
    return -1;
  std::vector<int> meth(n_users);
  MR_D2H(meth.data(), dmeth.p, n_users * 4, r->stream);
  MR_HIP(hipStreamSynchronize(r->stream));
  std::vector<int> flagged;
  std::vector<int64_t> soff(1, 0);
  for (int u = 0; u < n_users; ++u)
    if (meth[u] == 2) {
      flagged.push_back(u);
      soff.push_back(soff.back() + (int64_t)(K + 1) * (off[u + 1] - off[u]) + 2 * K);
    }
  if (!flagged.empty()) {
    DBuf<int> dfl;
    DBuf<int64_t> dso;
    DBuf<double> scr;
    if (dfl.upload(flagged.data(), flagged.size(), r->stream) ||
        dso.upload(soff.data(), flagged.size(), r->stream) || scr.alloc(soff.back()))
      return -1;
    const size_t lds2 = (size_t)K * K * sizeof(double);
    if (lds2 > 64 * 1024)
      MR_HIP(hipFuncSetAttribute((const void*)fold_in_svd_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
    if (timed(r, RT_SVD, [&]() {
          fold_in_svd_kernel<<<(unsigned)flagged.size(), 256, lds2, r->stream>>>(
              dfl.p, k, doff.p, didx.p, drat.p, r->V, scr.p, dso.p, dX.p);
          return 0;
        }))
      return -1;
  }
  MR_D2H(Xout, dX.p, (size_t)n_users * K * 8, r->stream);
  MR_HIP(hipStreamSynchronize(r->stream));
  if (method_out) std::copy(meth.begin(), meth.end(), method_out);
  return 0;
}

static int rec_evaluate(Rec* r, int n_rows, const double* Uh, int n_test, const int* user_row,
                        const long long* off, const int* cand, const double* actual,
                        double* agreement, long long* n_agree, long long* n_dis, double* pred,
                        double* sse, long long* n_pred) {
  MR_CHECK(n_rows >= 0 && n_test >= 0, "rec: negative sizes");
  reset_ms(r);
  if (n_test == 0) return 0;
  const int K = r->k + 1;
  const int64_t nnz = off[n_test];
  for (int t = 0; t < n_test; ++t)
    MR_CHECK(user_row[t] >= 0 && user_row[t] < n_rows, "rec: evaluation user row out of range");
  for (int64_t i = 0; i < nnz; ++i)
    MR_CHECK(cand[i] >= -1 && cand[i] < r->n_cand, "rec: evaluation candidate out of range");
  DBuf<double> dU, dact, dpred, dagr, dsse;
  DBuf<int> drow, dcand;
  DBuf<int64_t> doff;
  DBuf<long long> dag, ddis, dnp;
  if (dU.upload(Uh, (int64_t)n_rows * K, r->stream) || drow.upload(user_row, n_test, r->stream) ||
      doff.upload(reinterpret_cast<const int64_t*>(off), n_test + 1, r->stream) ||
      dcand.upload(cand, nnz, r->stream) || dact.upload(actual, nnz, r->stream) ||
      dpred.alloc(nnz) || dagr.alloc(n_test) || dsse.alloc(n_test) || dag.alloc(n_test) ||
      ddis.alloc(n_test) || dnp.alloc(n_test))
    return -1;
  if (timed(r, RT_EVAL, [&]() {
        rec_eval_kernel<true><<<n_test, 256, 0, r->stream>>>(r->k, dU.p, drow.p, doff.p, dcand.p,
                                                       dact.p, r->Vc, r->med, dpred.p, dagr.p,
                                                       dag.p, ddis.p, dsse.p, dnp.p);
        return 0;
      }))
    return -1;
  MR_D2H(agreement, dagr.p, n_test * 8, r->stream);
  MR_D2H(n_agree, dag.p, n_test * 8, r->stream);
  MR_D2H(n_dis, ddis.p, n_test * 8, r->stream);
  if (pred) MR_D2H(pred, dpred.p, nnz * 8, r->stream);
  if (sse) MR_D2H(sse, dsse.p, n_test * 8, r->stream);
  if (n_pred) MR_D2H(n_pred, dnp.p, n_test * 8, r->stream);
  MR_HIP(hipStreamSynchronize(r->stream));
  return 0;
}

static int rank_agreement(int device, int n_users, const long long* off, const double* actual,
                          const double* predicted, double* agreement, long long* n_agree,
                          long long* n_dis) {
  MR_CHECK(n_users >= 0, "rank_agreement: negative n_users");
  if (n_users == 0) return 0;
  MR_HIP(hipSetDevice(device));
  hipStream_t s = nullptr;
  MR_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } guard{s};
  const int64_t nnz = off[n_users];
  DBuf<int64_t> doff;
  DBuf<double> dact, dpred, dagr;
  DBuf<long long> dag, ddis;
  if (doff.upload(reinterpret_cast<const int64_t*>(off), n_users + 1, s) ||
      dact.upload(actual, nnz, s) || dpred.upload(predicted, nnz, s) || dagr.alloc(n_users) ||
      dag.alloc(n_users) || ddis.alloc(n_users))
    return -1;
  rec_eval_kernel<false><<<n_users, 256, 0, s>>>(0, nullptr, nullptr, doff.p, nullptr, dact.p,
                                                 nullptr, nullptr, dpred.p, dagr.p, dag.p,
                                                 ddis.p, nullptr, nullptr);
  MR_HIP(hipGetLastError());
  MR_D2H(agreement, dagr.p, n_users * 8, s);
  if (n_agree) MR_D2H(n_agree, dag.p, n_users * 8, s);
  if (n_dis) MR_D2H(n_dis, ddis.p, n_users * 8, s);
  MR_HIP(hipStreamSynchronize(s));
  return 0;
}

}  // namespace mr

// ---------------------------------------------------------------------------
// C ABI (include/mr_serving.h)
// ---------------------------------------------------------------------------
struct mr_rec {
  mr::Rec r;
};

namespace {
template <typename F>
int rec_guard(F&& f) {
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

mr_rec* mr_rec_create(int device, int k, int n_als, const double* als_movie_factors,
                      int n_cand, const int* cand_als, const int* cand_mid,
                      const double* cand_med) {
  mr_rec* ctx = nullptr;
  const int rc = rec_guard([&]() -> int {
    ctx = new mr_rec();
    return mr::rec_init(&ctx->r, device, k, n_als, als_movie_factors, n_cand, cand_als, cand_mid,
                        cand_med);
  });
  if (rc) {
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void mr_rec_destroy(mr_rec* ctx) { delete ctx; }

int mr_rec_num_candidates(const mr_rec* ctx) { return ctx ? ctx->r.n_cand : -1; }

int mr_rec_fold_in(mr_rec* ctx, int n_users, const long long* off, const int* als_idx,
                   const double* ratings, double* x_out, int* method_out) {
  if (!ctx) return -1;
  return rec_guard([&]() {
    return mr::rec_fold_in(&ctx->r, n_users, off, als_idx, ratings, x_out, method_out);
  });
}

int mr_rec_scores(mr_rec* ctx, int n_users, const double* x, double* out) {
  if (!ctx) return -1;
  return rec_guard([&]() { return mr::rec_scores(&ctx->r, n_users, x, out); });
}

int mr_rec_top_n(mr_rec* ctx, int n_users, const double* x, const long long* excl_off,
                 const int* excl_cand, int num_results, int* out_mid, double* out_score,
                 int* out_count) {
  if (!ctx) return -1;
  return rec_guard([&]() {
    return mr::rec_top_n(&ctx->r, n_users, x, excl_off, excl_cand, num_results, out_mid,
                         out_score, out_count);
  });
}

int mr_rec_evaluate(mr_rec* ctx, int n_rows, const double* U, int n_test, const int* user_row,
                    const long long* off, const int* cand, const double* actual,
                    double* agreement, long long* n_agree, long long* n_disagree, double* pred,
                    double* sse, long long* n_pred) {
  if (!ctx) return -1;
  return rec_guard([&]() {
    return mr::rec_evaluate(&ctx->r, n_rows, U, n_test, user_row, off, cand, actual, agreement,
                            n_agree, n_disagree, pred, sse, n_pred);
  });
}

int mr_rank_agreement(int device, int n_users, const long long* off, const double* actual,
                      const double* predicted, double* agreement, long long* n_agree,
                      long long* n_disagree) {
  return rec_guard([&]() {
    return mr::rank_agreement(device, n_users, off, actual, predicted, agreement, n_agree,
                              n_disagree);
  });
}

int mr_rec_last_kernel_ms(const mr_rec* ctx, double* ms6) {
  if (!ctx || !ms6) return -1;
  for (int i = 0; i < mr::RT_N; ++i) ms6[i] = ctx->r.ms[i];
  return 0;
}

}  // extern "C"
