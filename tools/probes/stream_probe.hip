// Read-stream probe for the general-CG SpMV's access shape (fp64 values +
// int32 column ids, 270 M non-zeros = 3.24 GB): what read rate do different
// stream structures reach?  Each variant sums what it reads (so nothing is
// optimised away) and writes one double per thread.
//   blk  : K1's shape -- a workgroup takes 2048-entry blocks b, b + G, ...;
//          thread t loads entry pairs 256 u + t (16-byte values, 8-byte ids),
//          u = 0..3, the next block's loads issued before this block's use
//   gs<U>: plain grid-stride, U (16-byte value, 8-byte id) pairs per thread
//          per trip, all issued before any use
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double double2_t __attribute__((ext_vector_type(2)));
typedef int int2_t __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void blk_kernel(const double* __restrict__ v, const int* __restrict__ ci,
                                                  long nblk, double* out) {
  const int t = threadIdx.x;
  double s = 0.0;
  double2_t cv[4], nv[4];
  int2_t cc[4], nc[4];
  long b = blockIdx.x;
  auto ld = [&](long bb, double2_t (&w)[4], int2_t (&c)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long m = bb * 1024 + 256 * u + t;
      w[u] = reinterpret_cast<const double2_t*>(v)[m];
      c[u] = reinterpret_cast<const int2_t*>(ci)[m];
    }
  };
  if (b < nblk) ld(b, cv, cc);
  for (; b < nblk; b += gridDim.x) {
    const bool nx = b + gridDim.x < nblk;
    if (nx) ld(b + gridDim.x, nv, nc);
#pragma unroll
    for (int u = 0; u < 4; ++u) s += cv[u].x * (double)cc[u].x + cv[u].y * (double)cc[u].y;
#pragma unroll
    for (int u = 0; u < 4; ++u) { cv[u] = nv[u]; cc[u] = nc[u]; }
  }
  out[blockIdx.x * 256 + t] = s;
}

template <int U>
__global__ __launch_bounds__(256) void gs_kernel(const double* __restrict__ v, const int* __restrict__ ci,
                                                 long npairs, double* out) {
  const long gt = (long)blockIdx.x * 256 + threadIdx.x, G = (long)gridDim.x * 256;
  double s = 0.0;
  for (long m0 = gt; m0 < npairs; m0 += G * U) {
    double2_t w[U];
    int2_t c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = m0 + u * G;
      const long ms = m < npairs ? m : 0;
      w[u] = reinterpret_cast<const double2_t*>(v)[ms];
      c[u] = reinterpret_cast<const int2_t*>(ci)[ms];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (m0 + u * G < npairs) s += w[u].x * (double)c[u].x + w[u].y * (double)c[u].y;
  }
  out[gt] = s;
}

int main() {
  const long nnz = 270L * 1000 * 1000 / 2048 * 2048;
  double* v; int* ci; double* out;
  CK(hipMalloc(&v, nnz * 8));
  CK(hipMalloc(&ci, nnz * 4));
  CK(hipMalloc(&out, 64L << 20));
  CK(hipMemset(v, 0, nnz * 8));
  CK(hipMemset(ci, 0, nnz * 4));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = nnz * 12.0;
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    printf("{\"variant\": \"%s\", \"us\": %.1f, \"TBps\": %.3f}\n", name, best * 1e3, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
  const long nblk = nnz / 2048;
  for (int w : {4, 5, 8, 12}) {
    char nm[64];
    snprintf(nm, sizeof nm, "blk grid=%dxCU", w);
    const int g = w * cus;
    run(nm, [&] { blk_kernel<<<g, 256>>>(v, ci, nblk, out); });
  }
  const long npairs = nnz / 2;
  for (int w : {4, 8, 16}) {
    char nm[64];
    const int g = w * cus;
    snprintf(nm, sizeof nm, "gs4 grid=%dxCU", w);
    run(nm, [&] { gs_kernel<4><<<g, 256>>>(v, ci, npairs, out); });
    snprintf(nm, sizeof nm, "gs8 grid=%dxCU", w);
    run(nm, [&] { gs_kernel<8><<<g, 256>>>(v, ci, npairs, out); });
  }
  CK(hipFree(v));
  CK(hipFree(ci));
  CK(hipFree(out));
  return 0;
}
