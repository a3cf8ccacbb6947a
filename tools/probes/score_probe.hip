// Probe: where does rec_score_kernel's time go?  Variants of the same tile
// loop with staging and/or arithmetic switched off (tools only, not shipped).
#include <hip/hip_runtime.h>
#include <cstdio>
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
template <int MODE>  // 0 full, 1 no global staging, 2 no arithmetic, 3 fma
__global__ __launch_bounds__(256) void k_score(int n_users, int n_cand, int k, const double* X,
                                               const double* Vc, const double* med, double* out) {
  __shared__ double xs[SC_U][SC_KC];
  __shared__ double vs[SC_C][SC_KC + 1];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int c0 = blockIdx.x * SC_C, u0 = blockIdx.y * SC_U;
  double acc[8][4];
  for (int p = 0; p < 8; ++p)
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int jj = tid & 15, rr = tid >> 4;
  for (int j0 = 0; j0 < k; j0 += SC_KC) {
    const int kc = min(SC_KC, k - j0);
    if (MODE != 1 || j0 == 0) {
      const double* src = Vc + (int64_t)(c0 + rr) * k + j0 + jj;
#pragma unroll 4
      for (int i = 0; i < SC_C / 16; ++i) {
        const bool ok = (c0 + rr + 16 * i) < n_cand;
        vs[rr + 16 * i][jj] = ok ? src[(int64_t)16 * i * k] : 0.0;
      }
      if (tid < SC_U * SC_KC / 2)
        for (int i = 0; i < 2; ++i) {
          const int r = rr + 16 * i, u = u0 + r;
          xs[r][jj] = (u < n_users) ? X[(int64_t)u * (k + 1) + j0 + jj] : 0.0;
        }
    }
    __syncthreads();
    if (MODE != 2) {
      for (int j = 0; j < kc; ++j) {
        double xv[8], vv[4];
#pragma unroll
        for (int p = 0; p < 8; ++p) xv[p] = xs[ty * 8 + p][j];
#pragma unroll
        for (int q = 0; q < 4; ++q) vv[q] = vs[tx + 64 * q][j];
#pragma unroll
        for (int p = 0; p < 8; ++p)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[p][q] = MODE == 3 ? fma(xv[p], vv[q], acc[p][q]) : add_rn(acc[p][q], mul_rn(xv[p], vv[q]));
      }
    } else {
      acc[0][0] += vs[tx][0] + xs[ty][1];
    }
    __syncthreads();
  }
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + tx + 64 * q;
      if (c < n_cand) out[(int64_t)u * n_cand + c] = acc[p][q] + med[c];
    }
  }
}

// Wider tile: 128 users x 256 candidates per 512-thread block, thread owns
// 8 users x 8 candidates; PF: register prefetch of the next chunk.
template <bool PF>
__global__ __launch_bounds__(512) void k_score2(int n_users, int n_cand, int k, const double* X,
                                                const double* Vc, const double* med, double* out) {
  constexpr int TU = 128, TC = 256, KC = 16;
  __shared__ double xs[2][KC][TU + 2];
  __shared__ double vs[2][KC][TC + 2];
  const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
  const int c0 = blockIdx.x * TC, u0 = blockIdx.y * TU;
  double acc[8][8];
  for (int p = 0; p < 8; ++p)
    for (int q = 0; q < 8; ++q) acc[p][q] = 0.0;
  // staging map: Vc: 256 rows x 16 cols -> thread: col jj = tid & 15, rows (tid>>4) + 32 i, i<8
  //              X : 128 rows x 16 cols -> rows (tid>>4) + 32 i, i<4
  const int jj = tid & 15, rr = tid >> 4;
  double pv[8], px[4];
  auto load = [&](int j0) {
    const bool jok = j0 + jj < k;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = c0 + rr + 32 * i;
      pv[i] = (jok && c < n_cand) ? Vc[(int64_t)c * k + j0 + jj] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = u0 + rr + 32 * i;
      px[i] = (jok && u < n_users) ? X[(int64_t)u * (k + 1) + j0 + jj] : 0.0;
    }
  };
  auto store = [&](int b) {
#pragma unroll
    for (int i = 0; i < 8; ++i) vs[b][jj][rr + 32 * i] = pv[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) xs[b][jj][rr + 32 * i] = px[i];
  };
  load(0);
  store(0);
  __syncthreads();
  int b = 0;
  for (int j0 = 0; j0 < k; j0 += KC) {
    const int kc = min(KC, k - j0);
    if (PF && j0 + KC < k) load(j0 + KC);
    for (int j = 0; j < kc; ++j) {
      double xv[8], vv[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) xv[p] = xs[b][j][ty * 8 + p];
#pragma unroll
      for (int q = 0; q < 8; ++q) vv[q] = vs[b][j][tx + 32 * q];
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        double pr[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pr[q] = mul_rn(xv[p], vv[q]);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[p][q] = add_rn(acc[p][q], pr[q]);
      }
    }
    if (j0 + KC < k) {
      if (!PF) load(j0 + KC);
      store(b ^ 1);
    }
    __syncthreads();
    b ^= 1;
  }
  for (int p = 0; p < 8; ++p) {
    const int u = u0 + ty * 8 + p;
    if (u >= n_users) continue;
    for (int q = 0; q < 8; ++q) {
      const int c = c0 + tx + 32 * q;
      if (c < n_cand) out[(int64_t)u * n_cand + c] = acc[p][q] + med[c];
    }
  }
}
int main() {
  const int U = 8192, C = 48859, k = 64;
  std::vector<double> h((size_t)C * k, 0.25), hx((size_t)U * (k + 1), 0.5), hm(C, 3.0);
  double *X, *V, *M, *O;
  hipMalloc(&X, hx.size() * 8); hipMalloc(&V, h.size() * 8); hipMalloc(&M, C * 8);
  hipMalloc(&O, (size_t)U * C * 8);
  hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(V, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(M, hm.data(), C * 8, hipMemcpyHostToDevice);
  dim3 grid((C + SC_C - 1) / SC_C, U / SC_U);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"full (mul+add)", "no staging", "no arithmetic", "fma", "wide", "wide+pf"};
  for (int mode = 0; mode < 6; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (mode == 0) k_score<0><<<grid, 256>>>(U, C, k, X, V, M, O);
      if (mode == 1) k_score<1><<<grid, 256>>>(U, C, k, X, V, M, O);
      if (mode == 2) k_score<2><<<grid, 256>>>(U, C, k, X, V, M, O);
      if (mode == 3) k_score<3><<<grid, 256>>>(U, C, k, X, V, M, O);
      dim3 g2((C + 255) / 256, U / 128);
      if (mode == 4) k_score2<false><<<g2, 512>>>(U, C, k, X, V, M, O);
      if (mode == 5) k_score2<true><<<g2, 512>>>(U, C, k, X, V, M, O);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2) {
        double ops = (double)U * C * 2.0 * k;
        printf("%-16s %8.3f ms  %6.2f Tops/s (scores %.2e)\n", names[mode], ms, ops / ms / 1e9, (double)U * C);
      }
    }
  }
  return 0;
}
