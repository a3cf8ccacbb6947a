// HIP kernels of the ALS hot path for MI355X (gfx950, CDNA4).
//
// Replaces the CPU loops of the reference (louisyang2015/movie_recommender,
// cpp/ls_lib/matrix.cpp):
//   gram_kernel      fill_user_A / fill_item_A / fill_ratings_minus_bias
//                    (:898-1031) + the A^T A and A^T b products inside
//                    cg_least_squares (:465-470), in block-diagonal form:
//                    per entity G_e = sum a a^T, c_e = sum a w  (MFMA f32)
//   cg_matvec        SpMV + SpMV^T of a CG iteration (:493-494) = batched
//                    block GEMV G_e p_e, fused with p = -r + beta p (:521)
//                    and the p.Ap partial dot (:497)
//   cg_update        x += alpha p, r += alpha Ap, r.r partials (:501-507)
//   cg_control       global scalars + stop rules (:488-525)
//   solve_kernel     exact per-entity Cholesky (north-star "exact" mode)
// Wave = 64 lanes throughout; no CUDA idioms.
#include "mr_internal.h"

namespace mr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Fixed-order block reduction of one double per thread (deterministic).
template <int NT>
__device__ __forceinline__ double block_sum_f64(double v, double* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum_f64(v);
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += sh[w];
  }
  return t;  // valid on thread 0
}

// ---------------------------------------------------------------------------
// K1: gather-Gram.  One wave per WorkItem (entity or chunk of a heavy
// entity).  Rows a_r are gathered from the opposite factor table
// (row stride ldk floats) and accumulated with v_mfma_f32_32x32x2_f32:
// lane l supplies a_{r0+(l>>5)}[32b + (l&31)], which is both the A operand
// (A[i][kk], i = l&31, kk = l>>5) and the B operand (B[kk][j], j = l&31) of
// the 32x32 block (bi, bj): D += A_bi^T A_bj over 2 ratings per MFMA.  Only
// the KB(KB+1)/2 upper blocks are computed; the epilogue mirrors them
// through LDS.  The rhs and (user side) row sums / counts ride along on
// VALU.  Item side: w = r - U[u][k] (fill_ratings_minus_bias, :1021-1030).
// ---------------------------------------------------------------------------
constexpr int GRAM_WAVES = 4;
constexpr int GRAM_UNR = 4;

template <int KB, bool USER>
__global__ __launch_bounds__(256) void gram_kernel(
    const WorkItem* __restrict__ work, int64_t n_work,
    const int32_t* __restrict__ idx, const float* __restrict__ val,
    const float* __restrict__ F, const float* __restrict__ bias, int k, int ldk,
    GramDst direct, GramDst slab) {
  constexpr int T = KB * (KB + 1) / 2;
  __shared__ float lds_t[GRAM_WAVES][32][33];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t wi = (int64_t)blockIdx.x * GRAM_WAVES + wid;
  if (wi >= n_work) return;  // waves are independent: no block barriers below
  const WorkItem w = work[wi];
  const int half = lane >> 5, col = lane & 31;
  const int64_t end = w.begin + w.len;

  floatx16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float cacc[KB], sacc[KB];
#pragma unroll
  for (int b = 0; b < KB; ++b) { cacc[b] = 0.f; sacc[b] = 0.f; }
  float wsum = 0.f;

  for (int64_t j = w.begin; j < end; j += 64) {
    const int64_t jj = j + lane;
    const bool okr = jj < end;
    int my_idx = okr ? idx[jj] : -1;
    float my_w = okr ? val[jj] : 0.f;
    if (!USER) {
      const float b = bias[okr ? my_idx : 0];
      my_w = okr ? my_w - b : 0.f;
    }
    const int rem = (int)((end - j) < 64 ? (end - j) : 64);
    const int nsteps = (rem + 1) >> 1;
    for (int s0 = 0; s0 < nsteps; s0 += GRAM_UNR) {
      float a[GRAM_UNR][KB];
      float ww[GRAM_UNR];
#pragma unroll
      for (int u = 0; u < GRAM_UNR; ++u) {
        const int s = s0 + u;
        const int src = (2 * s + half) & 63;
        const int ri = __shfl(my_idx, src, 64);
        const float wv = __shfl(my_w, src, 64);
        const bool ok = (s < nsteps) && (ri >= 0);
        ww[u] = ok ? wv : 0.f;
        const int64_t rowb = (int64_t)(ok ? ri : 0) * ldk;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
          const int c = 32 * b + col;
          const bool okc = ok && (c < k);
          const float v = F[okc ? rowb + c : 0];
          a[u][b] = okc ? v : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < GRAM_UNR; ++u) {
        int t = 0;
#pragma unroll
        for (int bi = 0; bi < KB; ++bi)
#pragma unroll
          for (int bj = bi; bj < KB; ++bj) {
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][bi], a[u][bj],
                                                          acc[t], 0, 0, 0);
            ++t;
          }
#pragma unroll
        for (int b = 0; b < KB; ++b) {
          cacc[b] = fmaf(a[u][b], ww[u], cacc[b]);
          if (USER) sacc[b] += a[u][b];
        }
        if (USER) wsum += ww[u];
      }
    }
  }

  // ---- epilogue -----------------------------------------------------------
#pragma unroll
  for (int b = 0; b < KB; ++b) {
    cacc[b] += __shfl_xor(cacc[b], 32, 64);
    if (USER) sacc[b] += __shfl_xor(sacc[b], 32, 64);
  }
  const bool to_slab = w.slab >= 0;
  const int64_t di = to_slab ? (int64_t)w.slab : (int64_t)w.entity;
  const GramDst& D = to_slab ? slab : direct;
  float* __restrict__ Gd = D.G + di * D.sG;
  float* __restrict__ Cd = D.C + di * D.sV;
  if (half == 0) {
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      const int c = 32 * b + col;
      if (c < ldk) {
        Cd[c] = (c < k) ? cacc[b] : 0.f;
        if (USER) D.Gs[di * D.sV + c] = (c < k) ? sacc[b] : 0.f;
      }
    }
  }
  if (USER) {
    const float wt = __shfl(wsum, 0, 64) + __shfl(wsum, 32, 64);
    if (lane == 0) {
      D.Cb[di * D.sS] = wt;
      D.Gn[di * D.sS] = (float)w.len;
    }
  }
  int t = 0;
#pragma unroll
  for (int bi = 0; bi < KB; ++bi) {
#pragma unroll
    for (int bj = bi; bj < KB; ++bj) {
      // direct block (bi, bj): row = 32bi + (r&3) + 8(r>>2) + 4half, col = 32bj + col
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * bi + (r & 3) + 8 * (r >> 2) + 4 * half;
        const int cg = 32 * bj + col;
        if (row < k && cg < ldk) Gd[(int64_t)row * ldk + cg] = acc[t][r];
      }
      if (bi != bj) {
        // mirrored block (bj, bi) through an LDS transpose (stride 33: no
        // bank conflicts on the column read)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          lds_t[wid][(r & 3) + 8 * (r >> 2) + 4 * half][col] = acc[t][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) {
          const int trow = 2 * r2 + half;
          const float v = lds_t[wid][col][trow];
          const int row = 32 * bj + trow;
          const int cg = 32 * bi + col;
          if (row < k && cg < ldk) Gd[(int64_t)row * ldk + cg] = v;
        }
        __builtin_amdgcn_wave_barrier();
      }
      ++t;
    }
  }
}

template <int KB>
static int launch_gram_kb(hipStream_t s, bool user_side, int k,
                          const WorkItem* work, int64_t n_work,
                          const int32_t* idx, const float* val, const float* F,
                          const float* bias, GramDst direct, GramDst slab) {
  if (n_work <= 0) return 0;
  const int64_t grid = (n_work + GRAM_WAVES - 1) / GRAM_WAVES;
  if (user_side)
    gram_kernel<KB, true><<<dim3((unsigned)grid), dim3(256), 0, s>>>(
        work, n_work, idx, val, F, bias, k, ldk_of(k), direct, slab);
  else
    gram_kernel<KB, false><<<dim3((unsigned)grid), dim3(256), 0, s>>>(
        work, n_work, idx, val, F, bias, k, ldk_of(k), direct, slab);
  MR_HIP(hipGetLastError());
  return 0;
}

int launch_gram(hipStream_t s, bool user_side, int k, const WorkItem* work,
                int64_t n_work, const int32_t* idx, const float* val,
                const float* F, const float* bias, GramDst direct,
                GramDst slab) {
  const int kb = (k + 31) / 32;
  switch (kb) {
    case 1: return launch_gram_kb<1>(s, user_side, k, work, n_work, idx, val, F, bias, direct, slab);
    case 2: return launch_gram_kb<2>(s, user_side, k, work, n_work, idx, val, F, bias, direct, slab);
    case 3: return launch_gram_kb<3>(s, user_side, k, work, n_work, idx, val, F, bias, direct, slab);
    case 4: return launch_gram_kb<4>(s, user_side, k, work, n_work, idx, val, F, bias, direct, slab);
    default: set_error("k > 128 not supported by the Gram kernel"); return -1;
  }
}

// ---------------------------------------------------------------------------
// Combine partial records of split entities, in slab order (deterministic).
// Record layout: [k*ldk G][ldk Gs][ldk C][Cb][Gn] (+pad).
// ---------------------------------------------------------------------------
template <bool USER>
__global__ __launch_bounds__(256) void slab_reduce_kernel(
    const SplitItem* __restrict__ split, const float* __restrict__ slab,
    int64_t rec, int k, int ldk, GramDst direct) {
  const SplitItem sp = split[blockIdx.x];
  const int64_t nG = (int64_t)k * ldk;
  const int64_t used = nG + 2 * ldk + 2;
  for (int64_t t = threadIdx.x; t < used; t += blockDim.x) {
    const bool isGs = t >= nG && t < nG + ldk;
    const bool isCb = t == nG + 2 * ldk;
    const bool isGn = t == nG + 2 * ldk + 1;
    if (!USER && (isGs || isCb || isGn)) continue;
    float sum = 0.f;
    for (int q = 0; q < sp.nslab; ++q) sum += slab[(int64_t)(sp.slab0 + q) * rec + t];
    const int64_t e = sp.entity;
    if (t < nG) direct.G[e * direct.sG + t] = sum;
    else if (isGs) direct.Gs[e * direct.sV + (t - nG)] = sum;
    else if (t < nG + 2 * ldk) direct.C[e * direct.sV + (t - nG - ldk)] = sum;
    else if (isCb) direct.Cb[e * direct.sS] = sum;
    else direct.Gn[e * direct.sS] = sum;
  }
}

int launch_slab_reduce(hipStream_t s, bool user_side, int k,
                       const SplitItem* split, int64_t n_split,
                       const float* slab, int64_t rec, GramDst direct) {
  if (n_split <= 0) return 0;
  if (user_side)
    slab_reduce_kernel<true><<<dim3((unsigned)n_split), dim3(256), 0, s>>>(
        split, slab, rec, k, ldk_of(k), direct);
  else
    slab_reduce_kernel<false><<<dim3((unsigned)n_split), dim3(256), 0, s>>>(
        split, slab, rec, k, ldk_of(k), direct);
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// K2: batched block GEMV y_e = G_e v_e (+ bias row/col on the user side),
// with the CG direction update v = -r + beta v fused in front (matrix.cpp:521
// of the previous iteration) and the v.y partial dot behind (:497).
// One wave per entity, grid-stride over entities with a fixed grid so the
// partial sums are reproducible.  G_e rows are read as float4: lane l owns
// columns 4(l % LPR) .. +3 of row ro = l / LPR, LPR = ldk/4, RPI = 64/LPR
// rows per wave-instruction (k=64: 16 lanes per row, 1 KiB per load).
// G is symmetric, so row j of G_e equals column j: y = sum_j G[j][:] v_j.
// ---------------------------------------------------------------------------
constexpr int MV_WAVES = 4;

template <bool USER>
__global__ __launch_bounds__(256) void cg_matvec_kernel(
    const CgState* __restrict__ st, int update_p, int64_t E, int k, int ldk,
    const float* __restrict__ G, const float* __restrict__ Gs,
    const float* __restrict__ Gn, float* __restrict__ v, float* __restrict__ vb,
    const float* __restrict__ r, const float* __restrict__ rb,
    float* __restrict__ y, float* __restrict__ yb, double* __restrict__ partials) {
  if (st->done) return;
  __shared__ float pv[MV_WAVES][kMaxK];
  __shared__ float4 red[MV_WAVES][64];
  __shared__ double sh[MV_WAVES];
  const float beta = (float)st->beta;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int LPR = ldk >> 2;
  const int RPI = 64 / LPR;
  const int ro = lane / LPR, cgp = lane - ro * LPR;
  const bool act = ro < RPI;
  double dsum = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * MV_WAVES + wid; e < E;
       e += (int64_t)gridDim.x * MV_WAVES) {
    float* ve = v + e * ldk;
    for (int i = lane; i < ldk; i += 64) {
      float vi = ve[i];
      if (update_p) {
        vi = fmaf(beta, vi, -r[e * ldk + i]);
        ve[i] = vi;
      }
      pv[wid][i] = vi;
    }
    float vbias = 0.f;
    if (USER) {
      vbias = vb[e];
      if (update_p) {
        vbias = fmaf(beta, vbias, -rb[e]);
        if (lane == 0) vb[e] = vbias;
      }
    }
    __builtin_amdgcn_wave_barrier();
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* __restrict__ Ge = reinterpret_cast<const float4*>(G + e * (int64_t)k * ldk);
    if (act) {
      int j = ro;
#pragma unroll 4
      for (; j < k; j += RPI) {
        const float4 g = Ge[(int64_t)j * LPR + cgp];
        const float pj = pv[wid][j];
        acc.x = fmaf(g.x, pj, acc.x);
        acc.y = fmaf(g.y, pj, acc.y);
        acc.z = fmaf(g.z, pj, acc.z);
        acc.w = fmaf(g.w, pj, acc.w);
      }
    }
    red[wid][lane] = acc;
    __builtin_amdgcn_wave_barrier();
    double d = 0.0;
    float ybp = 0.f;
    if (lane < LPR) {
      float4 s = red[wid][lane];
      for (int q = 1; q < RPI; ++q) {
        const float4 t = red[wid][q * LPR + lane];
        s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
      }
      const int c0 = 4 * lane;
      if (USER) {
        const float4 g4 = reinterpret_cast<const float4*>(Gs + e * ldk)[lane];
        s.x = fmaf(g4.x, vbias, s.x);
        s.y = fmaf(g4.y, vbias, s.y);
        s.z = fmaf(g4.z, vbias, s.z);
        s.w = fmaf(g4.w, vbias, s.w);
        ybp = g4.x * pv[wid][c0] + g4.y * pv[wid][c0 + 1] + g4.z * pv[wid][c0 + 2] +
              g4.w * pv[wid][c0 + 3];
      }
      reinterpret_cast<float4*>(y + e * ldk)[lane] = s;
      d = (double)s.x * pv[wid][c0] + (double)s.y * pv[wid][c0 + 1] +
          (double)s.z * pv[wid][c0 + 2] + (double)s.w * pv[wid][c0 + 3];
    }
    if (USER) {
      const float yb_s = wave_sum_f32(ybp);
      const float ybv = fmaf(Gn[e], vbias, yb_s);
      if (lane == 0) yb[e] = ybv;
      if (lane == 0) d += (double)ybv * vbias;
    }
    dsum += wave_sum_f64(d);
    __builtin_amdgcn_wave_barrier();
  }
  const double tot = block_sum_f64<256>(lane == 0 ? dsum : 0.0, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

int launch_cg_matvec(hipStream_t s, bool user_side, const CgState* st,
                     int update_p, int64_t E, int k, const float* G,
                     const float* Gs, const float* Gn, float* v, float* vb,
                     const float* r, const float* rb, float* y, float* yb,
                     double* partials, int n_part) {
  if (n_part <= 0) return 0;
  if (user_side)
    cg_matvec_kernel<true><<<dim3(n_part), dim3(256), 0, s>>>(
        st, update_p, E, k, ldk_of(k), G, Gs, Gn, v, vb, r, rb, y, yb, partials);
  else
    cg_matvec_kernel<false><<<dim3(n_part), dim3(256), 0, s>>>(
        st, update_p, E, k, ldk_of(k), G, Gs, Gn, v, vb, r, rb, y, yb, partials);
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// CG vector update (matrix.cpp:468-476 init, :501-507 step) + r.r partials.
// Fixed grid, grid-stride, float4: reproducible partial sums.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cg_update_kernel(
    const CgState* __restrict__ st, int mode, int64_t n4, int64_t nb,
    float* __restrict__ x, float* __restrict__ r, float* __restrict__ p,
    const float* __restrict__ q, const float* __restrict__ c,
    float* __restrict__ xb, float* __restrict__ rb, float* __restrict__ pb,
    const float* __restrict__ qb, const float* __restrict__ cb,
    double* __restrict__ partials) {
  if (st->done) return;
  __shared__ double sh[4];
  const float alpha = (float)st->alpha;
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float4* r4 = reinterpret_cast<float4*>(r);
  const float4* q4 = reinterpret_cast<const float4*>(q);
  if (mode == UPD_INIT) {
    const float4* c4 = reinterpret_cast<const float4*>(c);
    float4* p4 = reinterpret_cast<float4*>(p);
    for (int64_t i = tid; i < n4; i += stride) {
      const float4 a = q4[i], b = c4[i];
      const float4 rr = make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
      r4[i] = rr;
      p4[i] = make_float4(-rr.x, -rr.y, -rr.z, -rr.w);
      acc += (double)rr.x * rr.x + (double)rr.y * rr.y + (double)rr.z * rr.z +
             (double)rr.w * rr.w;
    }
    for (int64_t i = tid; i < nb; i += stride) {
      const float rr = qb[i] - cb[i];
      rb[i] = rr;
      pb[i] = -rr;
      acc += (double)rr * rr;
    }
  } else {
    float4* x4 = reinterpret_cast<float4*>(x);
    const float4* p4 = reinterpret_cast<const float4*>(p);
    for (int64_t i = tid; i < n4; i += stride) {
      float4 xv = x4[i], rv = r4[i];
      const float4 pv = p4[i], qv = q4[i];
      xv.x = fmaf(alpha, pv.x, xv.x); xv.y = fmaf(alpha, pv.y, xv.y);
      xv.z = fmaf(alpha, pv.z, xv.z); xv.w = fmaf(alpha, pv.w, xv.w);
      rv.x = fmaf(alpha, qv.x, rv.x); rv.y = fmaf(alpha, qv.y, rv.y);
      rv.z = fmaf(alpha, qv.z, rv.z); rv.w = fmaf(alpha, qv.w, rv.w);
      x4[i] = xv;
      r4[i] = rv;
      acc += (double)rv.x * rv.x + (double)rv.y * rv.y + (double)rv.z * rv.z +
             (double)rv.w * rv.w;
    }
    for (int64_t i = tid; i < nb; i += stride) {
      xb[i] = fmaf(alpha, pb[i], xb[i]);
      const float rv = fmaf(alpha, qb[i], rb[i]);
      rb[i] = rv;
      acc += (double)rv * rv;
    }
  }
  const double tot = block_sum_f64<256>(acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

int launch_cg_update(hipStream_t s, const CgState* st, int mode, int64_t n,
                     int64_t nb, float* x, float* r, float* p, const float* q,
                     const float* c, float* xb, float* rb, float* pb,
                     const float* qb, const float* cb, double* partials,
                     int n_part) {
  cg_update_kernel<<<dim3(n_part), dim3(256), 0, s>>>(
      st, mode, n / 4, nb, x, r, p, q, c, xb, rb, pb, qb, cb, partials);
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// CG scalars and stop rules, exactly as cg_least_squares (matrix.cpp:478-528):
//   INIT : rr = r0.r0, final_rr = rr; stop if it >= max_it or rr < 1e-6
//   ALPHA: alpha = rr / (p.Ap)
//   BETA : rr2, final_rr = rr2, beta = rr2/rr, two consecutive
//          beta > 1 - min_dec end the solve (ret = it, x/r already updated);
//          else rr = rr2, it++, then the loop-top checks of the next iteration.
// ctl: CTL_REDUCE sums the local partials into st->comm[0] (sharded runs
// all-reduce that slot next); CTL_FINALIZE applies the rules from comm[0].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cg_control_kernel(
    CgState* __restrict__ st, int phase, int ctl,
    const double* __restrict__ partials, int n_part) {
  if (phase != CG_INIT && st->done) return;
  __shared__ double sh[4];
  if (ctl & CTL_REDUCE) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < n_part; i += blockDim.x) acc += partials[i];
    const double tot = block_sum_f64<256>(acc, sh);
    if (threadIdx.x == 0) st->comm[0] = tot;
  }
  if (threadIdx.x != 0 || !(ctl & CTL_FINALIZE)) return;
  const double s = st->comm[0];
  if (phase == CG_INIT) {
    st->rr = s;
    st->final_rr = s;
    st->it = 0;
    st->fails = 0;
    st->done = 0;
    st->ret = 0;
    if (st->max_it <= 0 || s < 1e-6) st->done = 1;
  } else if (phase == CG_ALPHA) {
    st->alpha = st->rr / s;
    st->n_matvec += 1;
  } else {
    const double rr2 = s;
    st->final_rr = rr2;
    const double beta = rr2 / st->rr;
    st->beta = beta;
    if (beta > 1.0 - st->min_dec) st->fails += 1;
    else st->fails = 0;
    if (st->fails >= 2) {
      st->done = 1;
      st->ret = st->it;
      return;
    }
    st->rr = rr2;
    st->it += 1;
    if (st->it >= st->max_it || rr2 < 1e-6) {
      st->done = 1;
      st->ret = st->it;
    }
  }
}

int launch_cg_control(hipStream_t s, CgState* st, int phase, int ctl,
                      const double* partials, int n_part) {
  cg_control_kernel<<<dim3(1), dim3(256), 0, s>>>(st, phase, ctl, partials, n_part);
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// Exact mode: per-entity (G_e + ridge I) x_e = c_e by Cholesky in fp64 LDS.
// One 256-thread workgroup per entity; K = k+1 on the user side (bias row /
// column from Gs, Gn, Cb), K = k on the item side.  Non-PD blocks keep their
// previous x_e and are counted.
// ---------------------------------------------------------------------------
template <bool USER>
__global__ __launch_bounds__(256) void solve_kernel(
    int64_t E, int k, int ldk, double ridge, const float* __restrict__ G,
    const float* __restrict__ Gs, const float* __restrict__ Gn,
    const float* __restrict__ C, const float* __restrict__ Cb,
    float* __restrict__ x, float* __restrict__ xb, int* __restrict__ nonpd) {
  extern __shared__ double sm[];
  const int K = USER ? k + 1 : k;
  double* M = sm;            // K*K
  double* b = sm + K * K;    // K
  __shared__ int bad;
  const int64_t e = blockIdx.x;
  const float* Ge = G + e * (int64_t)k * ldk;
  for (int t = threadIdx.x; t < K * K; t += blockDim.x) {
    const int i = t / K, j = t - (t / K) * K;
    double v;
    if (i < k && j < k) v = Ge[(int64_t)i * ldk + j];
    else if (i < k) v = Gs[e * ldk + i];           // j == k
    else if (j < k) v = Gs[e * ldk + j];           // i == k
    else v = Gn[e];
    if (i == j) v += ridge;
    M[t] = v;
  }
  for (int t = threadIdx.x; t < K; t += blockDim.x)
    b[t] = (t < k) ? (double)C[e * ldk + t] : (double)Cb[e];
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  // right-looking Cholesky, lower triangle
  for (int j = 0; j < K; ++j) {
    if (threadIdx.x == 0) {
      const double d = M[j * K + j];
      if (!(d > 0.0)) bad = 1;
      M[j * K + j] = d > 0.0 ? sqrt(d) : 1.0;
    }
    __syncthreads();
    const double djj = M[j * K + j];
    for (int i = j + 1 + threadIdx.x; i < K; i += blockDim.x) M[i * K + j] /= djj;
    __syncthreads();
    const int m = K - j - 1;
    for (int t = threadIdx.x; t < m * m; t += blockDim.x) {
      const int i = j + 1 + t / m, l = j + 1 + (t - (t / m) * m);
      if (l <= i) M[i * K + l] -= M[i * K + j] * M[l * K + j];
    }
    __syncthreads();
  }
  if (bad) {
    if (threadIdx.x == 0) atomicAdd(nonpd, 1);
    return;
  }
  // forward L z = b, then back L^T x = z (column-oriented, parallel over rows)
  for (int j = 0; j < K; ++j) {
    if (threadIdx.x == 0) b[j] /= M[j * K + j];
    __syncthreads();
    const double bj = b[j];
    for (int i = j + 1 + threadIdx.x; i < K; i += blockDim.x) b[i] -= M[i * K + j] * bj;
    __syncthreads();
  }
  for (int j = K - 1; j >= 0; --j) {
    if (threadIdx.x == 0) b[j] /= M[j * K + j];
    __syncthreads();
    const double bj = b[j];
    for (int i = threadIdx.x; i < j; i += blockDim.x) b[i] -= M[j * K + i] * bj;
    __syncthreads();
  }
  for (int t = threadIdx.x; t < K; t += blockDim.x) {
    if (t < k) x[e * ldk + t] = (float)b[t];
    else xb[e] = (float)b[t];
  }
}

int launch_solve(hipStream_t s, bool user_side, int64_t E, int k, double ridge,
                 const float* G, const float* Gs, const float* Gn,
                 const float* C, const float* Cb, float* x, float* xb,
                 int* nonpd) {
  if (E <= 0) return 0;
  const int K = user_side ? k + 1 : k;
  const size_t lds = (size_t)(K * K + K) * sizeof(double);
  if (user_side) {
    MR_HIP(hipFuncSetAttribute((const void*)solve_kernel<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    solve_kernel<true><<<dim3((unsigned)E), dim3(256), lds, s>>>(
        E, k, ldk_of(k), ridge, G, Gs, Gn, C, Cb, x, xb, nonpd);
  } else {
    MR_HIP(hipFuncSetAttribute((const void*)solve_kernel<false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    solve_kernel<false><<<dim3((unsigned)E), dim3(256), lds, s>>>(
        E, k, ldk_of(k), ridge, G, Gs, Gn, C, Cb, x, xb, nonpd);
  }
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// Layout conversion: reference fp64 rows of `width` (k+1 for users, k for
// items) <-> fp32 device rows of ldk floats (+ separate bias column).
// ---------------------------------------------------------------------------
__global__ void unpack_kernel(int64_t rows, int width, int k, int ldk,
                              const double* __restrict__ src,
                              float* __restrict__ fac, float* __restrict__ bias) {
  const int64_t n = rows * ldk;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / ldk;
    const int c = (int)(t - r * ldk);
    fac[t] = (c < k) ? (float)src[r * width + c] : 0.f;
    if (bias && c == 0) bias[r] = (float)src[r * width + k];
  }
}

__global__ void pack_kernel(int64_t rows, int width, int k, int ldk,
                            const float* __restrict__ fac,
                            const float* __restrict__ bias, double* __restrict__ dst) {
  const int64_t n = rows * width;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / width;
    const int c = (int)(t - r * width);
    dst[t] = (c < k) ? (double)fac[r * ldk + c] : (double)bias[r];
  }
}

static unsigned grid_for(int64_t n, int bs = 256, int64_t cap = 8192) {
  int64_t g = (n + bs - 1) / bs;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

int launch_unpack_factors(hipStream_t s, int64_t rows, int width, int k,
                          int ldk, const double* src, float* fac, float* bias) {
  if (rows <= 0) return 0;
  unpack_kernel<<<grid_for(rows * ldk), 256, 0, s>>>(rows, width, k, ldk, src, fac, bias);
  MR_HIP(hipGetLastError());
  return 0;
}

int launch_pack_factors(hipStream_t s, int64_t rows, int width, int k, int ldk,
                        const float* fac, const float* bias, double* dst) {
  if (rows <= 0) return 0;
  pack_kernel<<<grid_for(rows * width), 256, 0, s>>>(rows, width, k, ldk, fac, bias, dst);
  MR_HIP(hipGetLastError());
  return 0;
}

// ŷ = u[:k].v + u[k]  (matrix.cpp:1035-1053), one thread per pair.
__global__ void predict_kernel(int64_t n, int k, int ldk, const int* __restrict__ uid,
                               const int* __restrict__ iid,
                               const float* __restrict__ Uf,
                               const float* __restrict__ Ub,
                               const float* __restrict__ Vf, double* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = uid[t], i = iid[t];
    double s = 0.0;
    for (int j = 0; j < k; ++j) s += (double)Uf[u * ldk + j] * Vf[i * ldk + j];
    out[t] = s + Ub[u];
  }
}

int launch_predict(hipStream_t s, int64_t n, int k, int ldk, const int* uid,
                   const int* iid, const float* Ufac, const float* Ubias,
                   const float* Vfac, double* out) {
  if (n <= 0) return 0;
  predict_kernel<<<grid_for(n), 256, 0, s>>>(n, k, ldk, uid, iid, Ufac, Ubias, Vfac, out);
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// General CSR least squares in fp64 (cg_least_squares_from_python path):
// SpMV with 16 lanes per row, dot / update partials with a fixed grid.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void spmv_f64_kernel(
    int64_t rows, const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
    const double* __restrict__ v, const double* __restrict__ x, double* __restrict__ y) {
  const int sub = threadIdx.x & 15;
  for (int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4; row < rows;
       row += ((int64_t)gridDim.x * blockDim.x) >> 4) {
    double s = 0.0;
    for (int64_t j = rp[row] + sub; j < rp[row + 1]; j += 16) s += v[j] * x[ci[j]];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
    if (sub == 0) y[row] = s;
  }
}

int launch_spmv_f64(hipStream_t s, int64_t rows, const int64_t* rp,
                    const int32_t* ci, const double* v, const double* x, double* y) {
  if (rows <= 0) return 0;
  spmv_f64_kernel<<<grid_for(rows * 16), 256, 0, s>>>(rows, rp, ci, v, x, y);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ __launch_bounds__(256) void dot_f64_kernel(const CgState* st, int64_t n,
                                                      const double* __restrict__ a,
                                                      const double* __restrict__ b,
                                                      double* __restrict__ partials) {
  if (st && st->done) return;
  __shared__ double sh[4];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    acc += a[i] * b[i];
  const double tot = block_sum_f64<256>(acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

int launch_dot_f64(hipStream_t s, const CgState* st, int64_t n, const double* a,
                   const double* b, double* partials, int n_part) {
  dot_f64_kernel<<<dim3(n_part), 256, 0, s>>>(st, n, a, b, partials);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ __launch_bounds__(256) void update_f64_kernel(
    const CgState* __restrict__ st, int mode, int64_t n, double* __restrict__ x,
    double* __restrict__ r, double* __restrict__ p, const double* __restrict__ q,
    const double* __restrict__ c, double* __restrict__ partials) {
  if (st->done) return;
  __shared__ double sh[4];
  const double alpha = st->alpha;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double rv;
    if (mode == UPD_INIT) {
      rv = q[i] - c[i];
      p[i] = -rv;
    } else {
      x[i] = x[i] + alpha * p[i];
      rv = r[i] + alpha * q[i];
    }
    r[i] = rv;
    acc += rv * rv;
  }
  const double tot = block_sum_f64<256>(acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

int launch_update_f64(hipStream_t s, const CgState* st, int mode, int64_t n,
                      double* x, double* r, double* p, const double* q,
                      const double* c, double* partials, int n_part) {
  update_f64_kernel<<<dim3(n_part), 256, 0, s>>>(st, mode, n, x, r, p, q, c, partials);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ void p_update_f64_kernel(const CgState* __restrict__ st, int64_t n,
                                    double* __restrict__ p, const double* __restrict__ r) {
  if (st->done) return;
  const double beta = st->beta;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = -r[i] + beta * p[i];
}

int launch_p_update_f64(hipStream_t s, const CgState* st, int64_t n, double* p,
                        const double* r) {
  if (n <= 0) return 0;
  p_update_f64_kernel<<<grid_for(n), 256, 0, s>>>(st, n, p, r);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ void rows_of_kernel(int64_t rows, const int64_t* __restrict__ rp,
                               int32_t* __restrict__ row_of) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x)
    for (int64_t j = rp[r]; j < rp[r + 1]; ++j) row_of[j] = (int32_t)r;
}

int launch_rows_of(hipStream_t s, int64_t rows, const int64_t* rp, int32_t* row_of) {
  if (rows <= 0) return 0;
  rows_of_kernel<<<grid_for(rows), 256, 0, s>>>(rows, rp, row_of);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ void i32_to_i64_kernel(int64_t n, const int32_t* __restrict__ in,
                                  int64_t* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    out[t] = in[t];
}

int launch_i32_to_i64(hipStream_t s, int64_t n, const int32_t* in, int64_t* out) {
  if (n <= 0) return 0;
  i32_to_i64_kernel<<<grid_for(n), 256, 0, s>>>(n, in, out);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ void validate_ids_kernel(int64_t n, const int32_t* __restrict__ ids,
                                    int32_t lo, int32_t hi, int* __restrict__ bad) {
  int local = 0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    local |= (ids[t] < lo || ids[t] >= hi);
  if (local) atomicOr(bad, 1);
}

int launch_validate_ids(hipStream_t s, int64_t n, const int32_t* ids, int32_t lo,
                        int32_t hi, int* bad) {
  if (n <= 0) return 0;
  validate_ids_kernel<<<grid_for(n), 256, 0, s>>>(n, ids, lo, hi, bad);
  MR_HIP(hipGetLastError());
  return 0;
}

}  // namespace mr
