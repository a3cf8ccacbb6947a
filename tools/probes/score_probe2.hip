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
  const char* names[] = {"P0 product", "P1 no store", "P2 lds-pipe", "P3 pipe nostore"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (mode == 0) k_score<true, false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 1) k_score<false, false><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 2) k_score<true, true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      if (mode == 3) k_score<false, true><<<grid, 256>>>(U, C, k, X, V, M, O, lo, hi);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2) {
        const double fl = (double)U * C * (2.0 * k + 2);
        printf("%-16s %8.3f ms  %6.2f TF/s  (%.3f of the 39.3 TF no-FMA ceiling)\n", names[mode], ms,
               fl / ms / 1e9, fl / ms / 1e9 / 39.3);
      }
    }
  }
  return hipDeviceSynchronize() != hipSuccess;
}
