// Probe (tools only, not shipped): rec_score_kernel's time split, round 3.
// P0: the product loop (register-prefetched staging, order-preserving keys
// and the per-user key range); P1: P0 without the key stores; P2: P0 with the
// next j's LDS operands read into registers while j is multiplied; P3: P2
// without the stores.  Scores of U x C x k = 65536 x 48859 x 64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
constexpr int SC_U = 32, SC_C = 256, SC_KC = 16;
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ uint64_t score_key(double s) {
  if (s == 0.0) s = 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(s);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
template <bool STORE, bool PIPE>
__global__ __launch_bounds__(256) void k_score(int n_users, int n_cand, int k, const double* __restrict__ X,
                                               const double* __restrict__ Vc, const double* __restrict__ med,
                                               uint64_t* __restrict__ out, unsigned long long* kmin,
                                               unsigned long long* kmax) {
  __shared__ double xs[SC_U][SC_KC];
  __shared__ double vs[SC_C][SC_KC + 1];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
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
    for (int i = 0; i < SC_C / 16; ++i) vs[rr + 16 * i][jj] = vreg[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) xs[rr + 16 * i][jj] = xreg[i];
    __syncthreads();
    if (j0 + SC_KC < k) load_chunk(j0 + SC_KC);
    if constexpr (!PIPE) {
      for (int j = 0; j < kc; ++j) {
        double xv[8], vv[4];
#pragma unroll
        for (int p = 0; p < 8; ++p) xv[p] = xs[ty * 8 + p][j];
#pragma unroll
        for (int q = 0; q < 4; ++q) vv[q] = vs[tx + 64 * q][j];
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
    } else {
      double xv[8], vv[4];
#pragma unroll
      for (int p = 0; p < 8; ++p) xv[p] = xs[ty * 8 + p][0];
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = vs[tx + 64 * q][0];
      for (int j = 0; j < kc; ++j) {
        const int jn = j + 1 < kc ? j + 1 : j;
        double xn[8], vn[4];
#pragma unroll
        for (int p = 0; p < 8; ++p) xn[p] = xs[ty * 8 + p][jn];
#pragma unroll
        for (int q = 0; q < 4; ++q) vn[q] = vs[tx + 64 * q][jn];
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
#pragma unroll
        for (int p = 0; p < 8; ++p) xv[p] = xn[p];
#pragma unroll
        for (int q = 0; q < 4; ++q) vv[q] = vn[q];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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
// P4 / P5: the user operands as wave-uniform SCALAR loads instead of LDS
// broadcasts.  Xt[g][j][8]: the 8 users of wave group g, factor j
// contiguous, so one s_load_dwordx16 fetches one j's 8 user values; the
// multiply takes them as SGPR operands.  LDS then carries only the
// candidates' 4 values per lane and j.
template <bool STORE>
__global__ __launch_bounds__(256) void k_score_s(int n_users, int n_cand, int k, const double* __restrict__ Xt,
                                                 const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ double vs[SC_C][SC_KC + 1];
  const int tid = threadIdx.x, tx = tid & 63;
  const int ty = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  const double* __restrict__ xg = Xt + (int64_t)(blockIdx.y * 4 + ty) * k * 8;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
  double vreg[SC_C / 16];
  auto load_chunk = [&](int j0) {
    const int kc = min(SC_KC, k - j0);
    const bool jok = jj < kc;
    const double* src = Vc + (int64_t)(c0 + rr) * k + j0 + jj;
#pragma unroll
    for (int i = 0; i < SC_C / 16; ++i) {
      const bool ok = jok && (c0 + rr + 16 * i) < n_cand;
      vreg[i] = ok ? src[(int64_t)16 * i * k] : 0.0;
    }
  };
  load_chunk(0);
  for (int j0 = 0; j0 < k; j0 += SC_KC) {
#pragma unroll
    for (int i = 0; i < SC_C / 16; ++i) vs[rr + 16 * i][jj] = vreg[i];
    __syncthreads();
    if (j0 + SC_KC < k) load_chunk(j0 + SC_KC);
#pragma unroll
    for (int j = 0; j < SC_KC; ++j) {
      double xv[8], vv[4];
#pragma unroll
      for (int p = 0; p < 8; ++p) xv[p] = xg[(j0 + j) * 8 + p];
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = vs[tx + 64 * q][j];
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
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

// P6 / P7: the user operands broadcast by DPP row_newbcast from registers.
// Per 16-factor chunk, lane i of every 16-lane row holds user (i & 7)'s
// factors j0 + 2t + (i >> 3), t < 8 (8 doubles); factor j of user p is then
// row_newbcast:(p + 8 (j & 1)) of register t = j >> 1 -- no LDS traffic for
// the users (an LDS broadcast still moves 64 lanes x 8 B per value).
template <int T>
__device__ __forceinline__ double bcast64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int2, v).x, 0x150 + T, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int2, v).y, 0x150 + T, 0xF, 0xF, false);
  return __builtin_bit_cast(double, make_int2(lo, hi));
}
template <int H>
__device__ __forceinline__ void xv_of(double (&xv)[8], double xr) {
  xv[0] = bcast64<0 + 8 * H>(xr); xv[1] = bcast64<1 + 8 * H>(xr);
  xv[2] = bcast64<2 + 8 * H>(xr); xv[3] = bcast64<3 + 8 * H>(xr);
  xv[4] = bcast64<4 + 8 * H>(xr); xv[5] = bcast64<5 + 8 * H>(xr);
  xv[6] = bcast64<6 + 8 * H>(xr); xv[7] = bcast64<7 + 8 * H>(xr);
}
template <bool STORE>
__global__ __launch_bounds__(256) void k_score_d(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ double vs[SC_C][SC_KC + 1];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
  const int up = u0 + ty * 8 + (tx & 7), uh = (tx >> 3) & 1;   // this lane's user and j parity
  double vreg[SC_C / 16], xreg[8];
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
    for (int t = 0; t < 8; ++t) {
      const int j = j0 + 2 * t + uh;
      xreg[t] = (j < k && up < n_users) ? X[(int64_t)up * (k + 1) + j] : 0.0;
    }
  };
  load_chunk(0);
  for (int j0 = 0; j0 < k; j0 += SC_KC) {
#pragma unroll
    for (int i = 0; i < SC_C / 16; ++i) vs[rr + 16 * i][jj] = vreg[i];
    double xr[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) xr[t] = xreg[t];
    __syncthreads();
    if (j0 + SC_KC < k) load_chunk(j0 + SC_KC);
#pragma unroll
    for (int j = 0; j < SC_KC; ++j) {
      double xv[8], vv[4];
      if (j & 1) xv_of<1>(xv, xr[j >> 1]); else xv_of<0>(xv, xr[j >> 1]);
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = vs[tx + 64 * q][j];
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
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

// P8 / P9: 8 users x 8 candidates per lane (block: 32 users x 512
// candidates): half the LDS bytes per multiply-add of the 8 x 4 tile.
constexpr int W_C = 512;
template <bool STORE>
__global__ __launch_bounds__(256) void k_score_w(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ double xs[SC_U][SC_KC];
  __shared__ double vs[W_C][SC_KC + 1];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * W_C, u0 = blockIdx.y * SC_U;
  double acc[8][8];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
  for (int j0 = 0; j0 < k; j0 += SC_KC) {
    const int kc = min(SC_KC, k - j0);
    const bool jok = jj < kc;
    const double* src = Vc + (int64_t)(c0 + rr) * k + j0 + jj;
#pragma unroll
    for (int i = 0; i < W_C / 16; ++i) {
      const bool ok = jok && (c0 + rr + 16 * i) < n_cand;
      vs[rr + 16 * i][jj] = ok ? src[(int64_t)16 * i * k] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = rr + 16 * i, u = u0 + r;
      xs[r][jj] = (jok && u < n_users) ? X[(int64_t)u * (k + 1) + j0 + jj] : 0.0;
    }
    __syncthreads();
    for (int j = 0; j < kc; ++j) {
      double xv[8], vv[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) xv[p] = xs[ty * 8 + p][j];
#pragma unroll
      for (int q = 0; q < 8; ++q) vv[q] = vs[tx + 64 * q][j];
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        double pr[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pr[q] = mul_rn(xv[p], vv[q]);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[p][q] = add_rn(acc[p][q], pr[q]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

// P10 / P11: P0 with the LDS tiles transposed to [j][user] / [j][candidate]
// so the j-loop reads are ds_read_b128 broadcasts (the 8 users' values of one
// j, 64 contiguous bytes: 4 x 4 LDS cycles) and conflict-free ds_read_b64
// (4 candidates: 4 x 2 cycles) instead of ds_read2_b64 pairs (8 cycles each):
// 24 instead of 48 LDS cycles per j and wave.  Rows padded by one double so
// the staging writes (16 lanes, one per j) fall in distinct banks.
constexpr int T_XP = SC_U + 2, T_VP = SC_C + 1;
template <bool STORE>
__global__ __launch_bounds__(256) void k_score_t(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ __attribute__((aligned(16))) double xs[SC_KC][T_XP];
  __shared__ double vs[SC_KC][T_VP];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
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
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

template <bool STORE, int DIAG>
__global__ __launch_bounds__(256) void k_score_x(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ __attribute__((aligned(16))) double xs[SC_KC][T_XP];
  __shared__ double vs[SC_KC][T_VP];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
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
    if (DIAG != 1 || j0 == 0) {
#pragma unroll
    for (int i = 0; i < SC_C / 16; ++i) vs[jj][rr + 16 * i] = vreg[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) xs[jj][rr + 16 * i] = xreg[i];
    }
    __syncthreads();
    if (DIAG != 1 && j0 + SC_KC < k) load_chunk(j0 + SC_KC);
    double xv0[8], vv0[4];
    if (DIAG == 2) {
      const double2* xp = reinterpret_cast<const double2*>(&xs[0][ty * 8]);
#pragma unroll
      for (int p = 0; p < 4; ++p) { const double2 t = xp[p]; xv0[2 * p] = t.x; xv0[2 * p + 1] = t.y; }
#pragma unroll
      for (int q = 0; q < 4; ++q) vv0[q] = vs[0][tx + 64 * q];
    }
    for (int j = 0; j < kc; ++j) {
      double xv[8], vv[4];
      if (DIAG == 2) {
#pragma unroll
        for (int p = 0; p < 8; ++p) xv[p] = xv0[p] + (double)j;
#pragma unroll
        for (int q = 0; q < 4; ++q) vv[q] = vv0[q];
      } else {
      const double2* xp = reinterpret_cast<const double2*>(&xs[j][ty * 8]);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const double2 t = xp[p];
        xv[2 * p] = t.x;
        xv[2 * p + 1] = t.y;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = vs[j][tx + 64 * q];
      }
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
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

template <bool STORE>
__global__ __launch_bounds__(256) void k_score_g(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ __attribute__((aligned(16))) double xs[SC_KC][T_XP];
  __shared__ double vs[SC_KC][T_VP];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  // user tile fastest: the blocks in flight share a few candidate tiles
  // (one 128 KB V tile per XCD L2) instead of streaming all of V
  const int c0 = blockIdx.y * SC_C, u0 = blockIdx.x * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
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
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

template <bool STORE>
__global__ __launch_bounds__(256) void k_score_e(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                 const double* __restrict__ Vc, const double* __restrict__ med,
                                                 uint64_t* __restrict__ out, unsigned long long* kmin,
                                                 unsigned long long* kmax) {
  __shared__ __attribute__((aligned(16))) double xs[SC_KC][T_XP];
  __shared__ double vs[SC_KC][T_VP];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
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
  // epilogue: the 8 users' key ranges reduced together (8 independent
  // butterflies per level instead of 8 dependent chains one after another)
  unsigned long long lo[8], hi[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    const double bias = u < n_users ? X[(int64_t)u * (k + 1) + k] : 0.0;
    lo[p] = ~0ull;
    hi[p] = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand || u >= n_users) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo[p] = min(lo[p], (unsigned long long)key);
      hi[p] = max(hi[p], (unsigned long long)key);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      lo[p] = min(lo[p], (unsigned long long)__shfl_xor(lo[p], o, 64));
      hi[p] = max(hi[p], (unsigned long long)__shfl_xor(hi[p], o, 64));
    }
  }
  if (tx == 0) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int u = u0 + ty * 8 + p;
      if (u < n_users) {
        atomicMin(&kmin[u], lo[p]);
        atomicMax(&kmax[u], hi[p]);
      }
    }
  }
}

// P16 / P17: transposed LDS tiles, double-buffered in chunks of 8 factors:
// the chunk c+1 (prefetched into registers during c-1) is written into the
// other buffer before chunk c is multiplied, so one barrier per chunk.
constexpr int DB_KC = 8;
template <bool STORE>
__global__ __launch_bounds__(256) void k_score_db(int n_users, int n_cand, int k, const double* __restrict__ X,
                                                  const double* __restrict__ Vc, const double* __restrict__ med,
                                                  uint64_t* __restrict__ out, unsigned long long* kmin,
                                                  unsigned long long* kmax) {
  __shared__ __attribute__((aligned(16))) double xs[2][DB_KC][T_XP];
  __shared__ double vs[2][DB_KC][T_VP];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  // staging map: 8 factors x 256 candidates = 2048 doubles, 8 per thread:
  // thread (jj = tid & 7, rr = tid >> 3) loads candidates rr + 32 i
  const int jj = tid & 7, rr = tid >> 3;
  double vreg[SC_C / 32], xreg;
  auto load_chunk = [&](int j0) {
    const bool jok = j0 + jj < k;
    const double* src = Vc + (int64_t)(c0 + rr) * k + j0 + jj;
#pragma unroll
    for (int i = 0; i < SC_C / 32; ++i) {
      const bool ok = jok && (c0 + rr + 32 * i) < n_cand;
      vreg[i] = ok ? src[(int64_t)32 * i * k] : 0.0;
    }
    const int u = u0 + rr;   // rr < 32: one user per thread
    xreg = (jok && u < n_users) ? X[(int64_t)u * (k + 1) + j0 + jj] : 0.0;
  };
  auto store_chunk = [&](int b) {
#pragma unroll
    for (int i = 0; i < SC_C / 32; ++i) vs[b][jj][rr + 32 * i] = vreg[i];
    xs[b][jj][rr] = xreg;
  };
  load_chunk(0);
  store_chunk(0);
  if (DB_KC < k) load_chunk(DB_KC);
  __syncthreads();
  int b = 0;
  for (int j0 = 0; j0 < k; j0 += DB_KC) {
    const int kc = min(DB_KC, k - j0);
    if (j0 + DB_KC < k) {
      store_chunk(b ^ 1);                       // chunk j0 + 8 into the other buffer
      if (j0 + 2 * DB_KC < k) load_chunk(j0 + 2 * DB_KC);
    }
    for (int j = 0; j < kc; ++j) {
      double xv[8], vv[4];
      const double2* xp = reinterpret_cast<const double2*>(&xs[b][j][ty * 8]);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const double2 t = xp[p];
        xv[2 * p] = t.x;
        xv[2 * p + 1] = t.y;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = vs[b][j][tx + 64 * q];
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
    b ^= 1;
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    const double bias = X[(int64_t)u * (k + 1) + k];
    unsigned long long lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c >= n_cand) continue;
      const double s = add_rn(add_rn(acc[p][q], bias), med[c]);
      const uint64_t key = score_key(s);
      if (STORE || key == 0x123456789ull) out[(int64_t)u * n_cand + c] = key;
      lo = min(lo, (unsigned long long)key);
      hi = max(hi, (unsigned long long)key);
    }
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

// Pure fp64 VALU throughput: 32 independent chains per lane of a separate
// multiply and add (what the exact score order needs), and the same with FMA.
template <bool FMA>
__global__ __launch_bounds__(256) void k_alu(double* out, double a, double b, int iters) {
  extern __shared__ double occ_lds[];   // dynamic size only limits blocks per CU
  if (iters < 0) occ_lds[threadIdx.x] = a;
  double acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = FMA ? fma(acc[i], a, b) : add_rn(mul_rn(acc[i], a), b);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 32; ++i) s += acc[i];
  if (s == 123.456) out[threadIdx.x] = s;
}

int main() {
  const int U = 65536, C = 48859, k = 64;
  std::vector<double> h((size_t)C * k), hx((size_t)U * (k + 1)), hm(C, 3.0);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.001 * (double)(i % 997) - 0.4;
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = 0.002 * (double)(i % 751) - 0.7;
  double *X, *V, *M;
  uint64_t* O;
  unsigned long long *lo, *hi;
  hipMalloc(&X, hx.size() * 8); hipMalloc(&V, h.size() * 8); hipMalloc(&M, C * 8);
  hipMalloc(&O, (size_t)U * C * 8); hipMalloc(&lo, U * 8); hipMalloc(&hi, U * 8);
  hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(V, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(M, hm.data(), C * 8, hipMemcpyHostToDevice);
  dim3 grid((C + SC_C - 1) / SC_C, U / SC_U);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  // Xt: users in groups of 8, [group][j][8]
  std::vector<double> hxt((size_t)U * k);
  for (int g = 0; g < U / 8; ++g)
    for (int j = 0; j < k; ++j)
      for (int p = 0; p < 8; ++p) hxt[((size_t)g * k + j) * 8 + p] = hx[(size_t)(g * 8 + p) * (k + 1) + j];
  double* XT;
  hipMalloc(&XT, hxt.size() * 8);
  hipMemcpy(XT, hxt.data(), hxt.size() * 8, hipMemcpyHostToDevice);
  const char* names[] = {"P0 product", "P1 no store", "P2 lds-pipe", "P3 pipe nostore", "P4 sgpr users",
                         "P5 sgpr nostore", "P6 dpp users", "P7 dpp nostore", "P8 8x8 tile", "P9 8x8 nostore",
                         "P10 lds [j][.]", "P11 [j][.] nostore",
                         "P12 + epilogue", "P13 + epi nostore", "P14 no restage", "P15 no lds in j",
                         "P16 dbuf kc8", "P17 dbuf nostore", "P18 user-fast grid", "P19 ufast nostore"};
  dim3 gridu(U / SC_U, (C + SC_C - 1) / SC_C);
  dim3 gridw((C + W_C - 1) / W_C, U / SC_U);
  for (int mode = 0; mode < 20; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (mode == 0) k_score<true, false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 1) k_score<false, false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 2) k_score<true, true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 3) k_score<false, true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 4) k_score_s<true><<<grid, 256>>>(U, C, k, XT, X, V, M, O, lo, hi);
      if (mode == 5) k_score_s<false><<<grid, 256>>>(U, C, k, XT, X, V, M, O, lo, hi);
      if (mode == 6) k_score_d<true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 7) k_score_d<false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 8) k_score_w<true><<<gridw, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 9) k_score_w<false><<<gridw, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 10) k_score_t<true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 11) k_score_t<false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 12) k_score_e<true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 13) k_score_e<false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 14) k_score_x<false, 1><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 15) k_score_x<false, 2><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 16) k_score_db<true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 17) k_score_db<false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 18) k_score_g<true><<<gridu, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 19) k_score_g<false><<<gridu, 256>>>(U, C, k, X, V, M, O, lo, hi);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2) {
        const double fl = (double)U * C * (2.0 * k + 2);
        printf("%-16s %8.3f ms  %6.2f TF/s  (%.3f of the 39.3 TF no-FMA ceiling)\n", names[mode], ms,
               fl / ms / 1e9, fl / ms / 1e9 / 39.3);
      }
    }
  }
  {   // P6 must produce P0's keys bit for bit
    uint64_t *O2;
    hipMalloc(&O2, (size_t)U * C * 8);
    k_score<true, false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
    k_score_g<true><<<dim3(U / SC_U, (C + SC_C - 1) / SC_C), 256>>>(U, C, k, X, V, M, O2, lo, hi);
    hipDeviceSynchronize();
    std::vector<uint64_t> a1((size_t)C * 64), a2((size_t)C * 64);
    size_t bad = 0;
    for (int u0 = 0; u0 < U; u0 += U / 8) {
      hipMemcpy(a1.data(), O + (size_t)u0 * C, a1.size() * 8, hipMemcpyDeviceToHost);
      hipMemcpy(a2.data(), O2 + (size_t)u0 * C, a2.size() * 8, hipMemcpyDeviceToHost);
      for (size_t i = 0; i < a1.size(); ++i) bad += a1[i] != a2[i];
    }
    printf("P18 vs P0 keys: %zu mismatches in %zu sampled\n", bad, (size_t)8 * a1.size());
    hipFree(O2);
  }
  hipFuncSetAttribute((const void*)k_alu<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  for (int bpc : {1, 2, 3, 4, 8}) {   // blocks (of 4 waves) per CU -> waves per SIMD
    const size_t lds = bpc == 8 ? 0 : (size_t)(150 * 1024) / bpc;
    const int iters = 2048, blocks = 256 * bpc * 4;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      k_alu<false><<<blocks, 256, lds>>>(M, 1.0000001, 1e-9, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2)
        printf("ALU mul+add, %d wave(s)/SIMD: %6.2f T lane-ops/s\n", bpc,
               (double)blocks * 256 * iters * 64 / ms / 1e9);
    }
  }
  for (int f = 0; f < 2; ++f) {
    const int iters = 4096, blocks = 256 * 8;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (f == 0) k_alu<false><<<blocks, 256>>>(M, 1.0000001, 1e-9, iters);
      else k_alu<true><<<blocks, 256>>>(M, 1.0000001, 1e-9, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2) {
        const double ins = (double)blocks * 256 * iters * 32 * (f == 0 ? 2 : 1);   // lane-ops
        printf("%-16s %8.3f ms  %6.2f T lane-ops/s (%s)\n", f == 0 ? "ALU mul+add" : "ALU fma", ms,
               ins / ms / 1e9, f == 0 ? "v_mul_f64 + v_add_f64" : "v_fma_f64");
      }
    }
  }
  return hipDeviceSynchronize() != hipSuccess;
}
