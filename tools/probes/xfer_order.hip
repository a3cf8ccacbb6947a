// Probe: is a hipMemcpyAsync H2D from PAGEABLE host memory ordered after the
// kernels enqueued before it on the same stream (write-after-read on the
// device buffer)?  The engine's old set_factors reused one device staging
// buffer for U and V: copy U -> unpack kernel -> copy V -> unpack kernel.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/xfer_order.hip -o tools/probes/xfer_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(2);                                                             \
    }                                                                      \
  } while (0)

// Reads buf after a delay (so the following copy has time to overtake it).
__global__ void slow_copy(const float* buf, float* out, long n, long spin) {
  long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = buf[i];
}

static long count_not(const std::vector<float>& v, float x) {
  long c = 0;
  for (float a : v) c += (a != x);
  return c;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : (8l << 20);   // floats per transfer
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const long spin = 2000000;                               // ~1 ms of clock64 ticks
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *buf, *out1, *out2;
  CK(hipMalloc(&buf, n * 4));
  CK(hipMalloc(&out1, n * 4));
  CK(hipMalloc(&out2, n * 4));
  for (int pinned = 0; pinned < 2; ++pinned) {
    float *A, *B;
    std::vector<float> pa, pb;
    if (pinned) {
      CK(hipHostMalloc((void**)&A, n * 4, hipHostMallocDefault));
      CK(hipHostMalloc((void**)&B, n * 4, hipHostMallocDefault));
    } else {
      pa.assign(n, 0.f);
      pb.assign(n, 0.f);
      A = pa.data();
      B = pb.data();
    }
    for (long i = 0; i < n; ++i) {
      A[i] = 1.f;
      B[i] = 2.f;
    }
    long bad1 = 0, bad2 = 0;
    std::vector<float> h1(n), h2(n);
    for (int r = 0; r < reps; ++r) {
      CK(hipMemcpyAsync(buf, A, n * 4, hipMemcpyHostToDevice, s));
      slow_copy<<<1024, 256, 0, s>>>(buf, out1, n, spin);
      CK(hipMemcpyAsync(buf, B, n * 4, hipMemcpyHostToDevice, s));
      slow_copy<<<1024, 256, 0, s>>>(buf, out2, n, 0);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(h1.data(), out1, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), out2, n * 4, hipMemcpyDeviceToHost));
      bad1 += count_not(h1, 1.f);
      bad2 += count_not(h2, 2.f);
    }
    printf("%s H2D, %ld floats x %d reps: first kernel saw %ld wrong values, second %ld\n",
           pinned ? "pinned  " : "pageable", n, reps, bad1, bad2);
    if (pinned) {
      CK(hipHostFree(A));
      CK(hipHostFree(B));
    }
  }
  // The engine's old set_factors / get_factors shape, with device buffers
  // from the stream-ordered pool (hipMallocAsync / hipFreeAsync): H2D into a
  // pool buffer, a slow kernel reads it, a second H2D into the SAME buffer, a
  // kernel reads it, free; then a slow kernel writes a fresh pool buffer and a
  // D2H reads it.  Host side pageable or pinned.  Counts: first reader saw the
  // second copy's data (H2D overtook a kernel), D2H returned stale data.
  for (int pinned = 0; pinned < 2; ++pinned) {
    long bad_h2d = 0, bad_d2h = 0, bad_plain = 0;
    float *src, *dummy, *back;
    std::vector<float> vs, vd, vb;
    if (pinned) {
      CK(hipHostMalloc((void**)&src, n * 4, hipHostMallocDefault));
      CK(hipHostMalloc((void**)&dummy, n * 4, hipHostMallocDefault));
      CK(hipHostMalloc((void**)&back, n * 4, hipHostMallocDefault));
    } else {
      vs.resize(n); vd.resize(n); vb.resize(n);
      src = vs.data(); dummy = vd.data(); back = vb.data();
    }
    std::vector<float> h(n);
    for (long i = 0; i < n; ++i) dummy[i] = -7.f;
    for (int r = 0; r < reps; ++r) {
      const float val = 3.f + r;
      for (long i = 0; i < n; ++i) src[i] = val + (float)(i & 1023);
      // plain hipMalloc'd buffers: D2H behind a slow producer kernel
      CK(hipMemcpyAsync(out1, src, n * 4, hipMemcpyHostToDevice, s));
      slow_copy<<<1024, 256, 0, s>>>(out1, out2, n, spin);
      CK(hipMemcpyAsync(h.data(), out2, n * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      for (long i = 0; i < n; ++i) bad_plain += (h[i] != src[i]);
      float* tmp;
      CK(hipMallocAsync((void**)&tmp, n * 4, s));
      CK(hipMemcpyAsync(tmp, src, n * 4, hipMemcpyHostToDevice, s));
      slow_copy<<<1024, 256, 0, s>>>(tmp, out1, n, spin);
      CK(hipMemcpyAsync(tmp, dummy, n * 4, hipMemcpyHostToDevice, s));
      slow_copy<<<1024, 256, 0, s>>>(tmp, out2, n, 0);
      CK(hipStreamSynchronize(s));
      CK(hipFreeAsync(tmp, s));
      CK(hipMemcpy(h.data(), out1, n * 4, hipMemcpyDeviceToHost));
      for (long i = 0; i < n; ++i) bad_h2d += (h[i] != src[i]);
      float* tmp2;
      CK(hipMallocAsync((void**)&tmp2, n * 4, s));
      slow_copy<<<1024, 256, 0, s>>>(out1, tmp2, n, spin);
      CK(hipMemcpyAsync(back, tmp2, n * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      CK(hipFreeAsync(tmp2, s));
      for (long i = 0; i < n; ++i) bad_d2h += (back[i] != h[i]);
    }
    printf("%s host: D2H behind a slow kernel (hipMalloc) %ld wrong; pool buffer: H2D overtook "
           "its reader %ld, D2H stale %ld\n", pinned ? "pinned  " : "pageable", bad_plain,
           bad_h2d, bad_d2h);
    if (pinned) {
      CK(hipHostFree(src));
      CK(hipHostFree(dummy));
      CK(hipHostFree(back));
    }
  }
  CK(hipFree(buf));
  CK(hipFree(out1));
  CK(hipFree(out2));
  return 0;
}
