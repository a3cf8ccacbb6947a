// Device CSR construction for the ALS hot path (one-time setup per context).
//
// Replaces the reference's host-side design-matrix construction
// (fill_user_A / fill_item_A first fill, cpp/ls_lib/matrix.cpp:904-936,
// 963-991) and its parallel CSR transpose (sparse_matrix_transpose,
// :617-692): COO triples are stably radix-sorted by entity id on the GPU
// (rocPRIM onesweep), then the opposite ids and values are gathered and the
// row offsets are derived from the sorted keys.  Stability keeps every
// entity's ratings in input order, so runs are reproducible.
#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "mr_internal.h"

namespace mr {

template <typename TV, typename TIn>
__global__ void gather_kernel(int64_t n, const int32_t* __restrict__ perm,
                              const int32_t* __restrict__ other,
                              const TIn* __restrict__ in_val,
                              int32_t* __restrict__ idx, TV* __restrict__ val) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = perm[j];
    idx[j] = other[p];
    val[j] = (TV)in_val[p];
  }
}

__global__ void iota_kernel(int64_t n, int32_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x)
    out[j] = (int32_t)j;
}

// off[e] = first position of key e in the sorted keys; empty entities get
// the position of the next non-empty one.
__global__ void offsets_kernel(int64_t n, int64_t E, const uint32_t* __restrict__ keys,
                               int64_t* __restrict__ off) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t kj = keys[j];
    const int64_t kp = (j == 0) ? -1 : (int64_t)keys[j - 1];
    for (int64_t e = kp + 1; e <= kj; ++e) off[e] = j;
    if (j == n - 1)
      for (int64_t e = kj + 1; e <= E; ++e) off[e] = n;
  }
}

__global__ void shift_keys_kernel(int64_t n, const int32_t* __restrict__ in,
                                  int32_t base, uint32_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x)
    out[j] = (uint32_t)(in[j] - base);
}

static unsigned grid_of(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 16384) g = 16384;
  return (unsigned)g;
}

template <typename TV, typename TIn>
int build_csr(hipStream_t s, int64_t n, int64_t E, const int32_t* d_key,
              int32_t key_base, const int32_t* d_other, const TIn* d_val, int64_t* off,
              int32_t* idx, TV* val) {
  MR_CHECK(n < ((int64_t)1 << 31), "build_csr: more than 2^31-1 ratings in one context");
  if (n == 0) {
    MR_HIP(hipMemsetAsync(off, 0, (E + 1) * sizeof(int64_t), s));
    return 0;
  }
  int bits = 1;
  while (((int64_t)1 << bits) < E) ++bits;
  uint32_t *k0 = nullptr, *k1 = nullptr;
  int32_t *v0 = nullptr, *v1 = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  int rc = -1;
  do {
    if (hipMalloc((void**)&k0, n * 4) != hipSuccess) break;
    if (hipMalloc((void**)&k1, n * 4) != hipSuccess) break;
    if (hipMalloc((void**)&v0, n * 4) != hipSuccess) break;
    if (hipMalloc((void**)&v1, n * 4) != hipSuccess) break;
    shift_keys_kernel<<<grid_of(n), 256, 0, s>>>(n, d_key, key_base, k0);
    iota_kernel<<<grid_of(n), 256, 0, s>>>(n, v0);
    if (rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, (size_t)n, 0, bits, s) !=
        hipSuccess) break;
    if (hipMalloc(&tmp, tb) != hipSuccess) break;
    if (rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, (size_t)n, 0, bits, s) !=
        hipSuccess) break;
    gather_kernel<TV, TIn><<<grid_of(n), 256, 0, s>>>(n, v1, d_other, d_val, idx, val);
    offsets_kernel<<<grid_of(n), 256, 0, s>>>(n, E, k1, off);
    if (hipGetLastError() != hipSuccess) break;
    rc = 0;
  } while (0);
  // temporaries from hipMalloc, not the stream-ordered pool (engine.hip dalloc)
  (void)hipStreamSynchronize(s);
  if (tmp) (void)hipFree(tmp);
  if (k0) (void)hipFree(k0);
  if (k1) (void)hipFree(k1);
  if (v0) (void)hipFree(v0);
  if (v1) (void)hipFree(v1);
  if (rc != 0) set_error("build_csr: device sort failed (out of memory?)");
  return rc;
}

// ---------------------------------------------------------------------------
// Row locality for the general least squares (cgls.hip): rows of a CSR
// matrix stably sorted by their first column id (empty rows last), and the
// matrix rebuilt in that row order.  A^T's rows (the columns of A) then list
// runs of consecutive permuted rows, so the A^T SpMV reads t in order instead
// of gathering it at random; a row permutation leaves the least-squares
// solution and every row sum unchanged (only A^T's summation order moves).
// ---------------------------------------------------------------------------
__global__ void first_col_kernel(int64_t rows, int64_t cols, const int64_t* __restrict__ rp,
                                 const int32_t* __restrict__ ci, uint32_t* __restrict__ key,
                                 int32_t* __restrict__ id) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    key[r] = rp[r + 1] > rp[r] ? (uint32_t)ci[rp[r]] : (uint32_t)cols;
    id[r] = (int32_t)r;
  }
}

__global__ void perm_len_kernel(int64_t rows, const int32_t* __restrict__ perm,
                                const int64_t* __restrict__ rp, int64_t* __restrict__ len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = perm[i];
    len[i] = rp[r + 1] - rp[r];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) len[rows] = 0;
}

// 8 lanes per row copy its non-zeros to the row's new position
__global__ void perm_copy_kernel(int64_t rows, const int32_t* __restrict__ perm,
                                 const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                 const double* __restrict__ v, const int64_t* __restrict__ rp2,
                                 int32_t* __restrict__ ci2, double* __restrict__ v2) {
  const int sub = threadIdx.x & 7;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; i < rows;
       i += ((int64_t)gridDim.x * blockDim.x) >> 3) {
    const int64_t r = perm[i], a = rp[r], n = rp[r + 1] - a, d = rp2[i];
    for (int64_t j = sub; j < n; j += 8) {
      ci2[d + j] = ci[a + j];
      v2[d + j] = v[a + j];
    }
  }
}

int sort_rows_by_first_col(hipStream_t s, int64_t rows, int64_t cols, const int64_t* rp,
                           const int32_t* ci, const double* v, int32_t* perm, int64_t* rp2,
                           int32_t* ci2, double* v2) {
  MR_CHECK(rows < ((int64_t)1 << 31) && cols < ((int64_t)1 << 31), "matrix too large");
  if (rows == 0) {
    MR_HIP(hipMemsetAsync(rp2, 0, sizeof(int64_t), s));
    return 0;
  }
  int bits = 1;
  while (((int64_t)1 << bits) <= cols) ++bits;
  uint32_t *k0 = nullptr, *k1 = nullptr;
  int32_t* v0 = nullptr;
  int64_t* len = nullptr;
  void* tmp = nullptr;
  size_t tb = 0, tb2 = 0;
  int rc = -1;
  do {
    if (hipMalloc((void**)&k0, rows * 4) != hipSuccess) break;
    if (hipMalloc((void**)&k1, rows * 4) != hipSuccess) break;
    if (hipMalloc((void**)&v0, rows * 4) != hipSuccess) break;
    if (hipMalloc((void**)&len, (rows + 1) * 8) != hipSuccess) break;
    first_col_kernel<<<grid_of(rows), 256, 0, s>>>(rows, cols, rp, ci, k0, v0);
    if (rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, perm, (size_t)rows, 0, bits, s) !=
        hipSuccess) break;
    if (rocprim::exclusive_scan(nullptr, tb2, len, rp2, (int64_t)0, (size_t)rows + 1,
                                rocprim::plus<int64_t>(), s) != hipSuccess) break;
    if (hipMalloc(&tmp, std::max(tb, tb2)) != hipSuccess) break;
    if (rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, perm, (size_t)rows, 0, bits, s) !=
        hipSuccess) break;
    perm_len_kernel<<<grid_of(rows), 256, 0, s>>>(rows, perm, rp, len);
    if (rocprim::exclusive_scan(tmp, tb2, len, rp2, (int64_t)0, (size_t)rows + 1,
                                rocprim::plus<int64_t>(), s) != hipSuccess) break;
    perm_copy_kernel<<<grid_of(rows * 8), 256, 0, s>>>(rows, perm, rp, ci, v, rp2, ci2, v2);
    if (hipGetLastError() != hipSuccess) break;
    rc = 0;
  } while (0);
  (void)hipStreamSynchronize(s);
  if (tmp) (void)hipFree(tmp);
  if (k0) (void)hipFree(k0);
  if (k1) (void)hipFree(k1);
  if (v0) (void)hipFree(v0);
  if (len) (void)hipFree(len);
  if (rc != 0) set_error("sort_rows_by_first_col: device sort failed (out of memory?)");
  return rc;
}

template int build_csr<float, double>(hipStream_t, int64_t, int64_t, const int32_t*,
                                      int32_t, const int32_t*, const double*, int64_t*,
                                      int32_t*, float*);
template int build_csr<double, double>(hipStream_t, int64_t, int64_t, const int32_t*,
                                       int32_t, const int32_t*, const double*, int64_t*,
                                       int32_t*, double*);

}  // namespace mr
