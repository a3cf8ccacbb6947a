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
#include <cstdlib>
#include <utility>

#include "mr_internal.h"


namespace mr {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
// Cross-lane sums without the LDS: v + v[lane ^ 16] and v + v[lane ^ 32] by
// the gfx950 v_permlane16_swap / v_permlane32_swap (called with vdst = vsrc = v
// they return {own rows, partner rows} in one order or the other, and the
// fp add commutes, so every lane gets exactly v + v[lane ^ S]); lane ^ 8 /
// ^ 4 / ^ 2 / ^ 1 by DPP.  Bit-identical to the __shfl_xor butterflies they
// replace (which went through ds_bpermute), one VALU op per 32-bit half.
template <int S>
__device__ __forceinline__ uint32_t xor_swap_u32(uint32_t v, uint32_t& other) {
  if constexpr (S == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    other = p[1];
    return p[0];
  } else {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    other = p[1];
    return p[0];
  }
}
template <int S>
__device__ __forceinline__ double xor_sum_f64(double v) {   // S = 16 or 32
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  uint32_t lo1, hi1;
  const uint32_t lo0 = xor_swap_u32<S>((uint32_t)u, lo1);
  const uint32_t hi0 = xor_swap_u32<S>((uint32_t)(u >> 32), hi1);
  return __builtin_bit_cast(double, ((uint64_t)hi0 << 32) | lo0) +
         __builtin_bit_cast(double, ((uint64_t)hi1 << 32) | lo1);
}
template <int S>
__device__ __forceinline__ float xor_sum_f32(float v) {
  uint32_t o;
  const uint32_t a = xor_swap_u32<S>(__builtin_bit_cast(uint32_t, v), o);
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, o);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v);

// Butterfly over the wave (xor 32, 16, 8, 4, 2, 1): every lane gets the sum,
// in the same bits.  Within a 16-lane row, row_ror:8 is lane ^ 8 and, once
// the values are symmetric under ^ 8, row_ror:4 acts as lane ^ 4.
__device__ __forceinline__ double wave_sum_f64(double v) {
  v = xor_sum_f64<32>(v);
  v = xor_sum_f64<16>(v);
  v += dpp_f64<0x128>(v);
  v += dpp_f64<0x124>(v);
  v += dpp_f64<0x4E>(v);
  return v + dpp_f64<0xB1>(v);
}
// ---------------------------------------------------------------------------
// Order-independent CG sums (round 3; the one-pass CG and its fused start).
// A sum of fp64 terms is kept as an integer: every term is truncated toward
// zero to a multiple of 2^kXLsb and added exactly into kXD 32-bit digits held
// in int64 containers (digit j weighs 2^(32 j + kXLsb); a term adds < 2^32 to
// at most three digits, so 2^31 terms fit without a carry).  Integer
// addition is associative: the value does not depend on which lane, wave,
// block or rank added which term, so a sharded run (or another grid size)
// reproduces the scalars bit for bit.  Digit kXD counts terms that are not
// finite or >= 2^96 in magnitude (the sum is then NaN; the CG's sums are
// far below that).  Lane j < kXD of a wave holds digit j, lane kXD the count.
// ---------------------------------------------------------------------------
constexpr int kXD = 10;
constexpr int kXLsb = -192;
constexpr int kXW = kXD + 1;   // containers per sum (digits + the count)

__device__ __forceinline__ int64_t xterm(double t, int j) {
  const uint64_t bits = (uint64_t)__double_as_longlong(t);
  const int e = (int)((bits >> 52) & 0x7FF);
  uint64_t m = bits & 0xFFFFFFFFFFFFFull;
  int x = -1074;
  if (e != 0) {
    m |= 1ull << 52;
    x = e - 1075;
  }
  if (j == kXD) return (e == 0x7FF || x + 53 > 96) ? 1 : 0;
  if (e == 0x7FF || x + 53 > 96) return 0;
  int p = x - kXLsb;
  if (p < 0) {
    m = p <= -64 ? 0 : (m >> (-p));
    p = 0;
  }
  const int i = p >> 5, o = p & 31;
  const uint64_t lo = m << o, hi = o ? (m >> (64 - o)) : 0;
  int64_t v = 0;
  if (j == i) v = (int64_t)(lo & 0xFFFFFFFFull);
  else if (j == i + 1) v = (int64_t)(lo >> 32);
  else if (j == i + 2) v = (int64_t)hi;
  return (bits >> 63) ? -v : v;
}

// Canonical digits (carries propagated) -> fp64, the same operations in the
// same order everywhere (tests/test_oracle.py restates it): Horner in base
// 2^32 from the top digit, then the exact scaling by 2^kXLsb.
__device__ double xsum_value(const int64_t* c_in) {
  if (c_in[kXD] != 0) return __longlong_as_double(0x7FF8000000000000ll);
  int64_t c[kXD];
#pragma unroll
  for (int j = 0; j < kXD; ++j) c[j] = c_in[j];
#pragma unroll
  for (int j = 0; j < kXD - 1; ++j) {
    const int64_t carry = c[j] >> 32;   // floor division by 2^32
    c[j] -= carry * 4294967296ll;
    c[j + 1] += carry;
  }
  double v = (double)c[kXD - 1];
#pragma unroll
  for (int j = kXD - 2; j >= 0; --j) v = __dadd_rn(__dmul_rn(v, 4294967296.0), (double)c[j]);
  return ldexp(v, kXLsb);
}

// General-CG SpMV (csr_spmv_kernel) timing probes (wrong results; never in the product build), bit mask:
// 1 no gathers, 2 no LDS staging / row sums (each thread sums its own
// entries), 4 no output stores, 8 no row-offset loads; the CG then runs
// to max_iteration (no stagnation or small-residual stop)
#ifndef MR_SP_PROBE
#define MR_SP_PROBE 0
#endif

// Block-level flush of each wave's per-lane containers of NV sums into the
// global bins [kXBins][NV][kXW] (bin = block mod kXBins, agent-scope integer
// atomics: exact, so their order does not matter).
constexpr int kXBins = 16;
// Entities per term of the one-pass CG's sums (a function of the kernel
// variant only, never of the grid or the shard): larger chunks save wave
// sums, smaller ones shorten the last round of a wave's entities.  Shard
// boundaries at multiples of kXAlign (distributed.SUM_CHUNK) keep a sharded
// run's terms those of the single-GPU run.
#ifndef MR_XC_U
#define MR_XC_U 4
#endif
#ifndef MR_XC_I
#define MR_XC_I 2
#endif
constexpr int kXAlign = 4;
constexpr int xchunk_of(int nb, bool user) { return nb > 4 ? 1 : (user ? MR_XC_U : MR_XC_I); }
static_assert(kXAlign % MR_XC_U == 0 && kXAlign % MR_XC_I == 0, "chunks must divide kXAlign");
// The block's containers in LDS, sh[nsh][sum][container] (one set per wave,
// or one per block).
template <int NV>
__device__ __forceinline__ void xsum_flush_lds(int64_t (*sh)[NV][kXW], int64_t* __restrict__ bins,
                                               int nsh) {
  __syncthreads();
  if (threadIdx.x < NV * kXW) {
    const int v = threadIdx.x / kXW, d = threadIdx.x % kXW;
    int64_t t = 0;
    for (int w = 0; w < nsh; ++w) t += sh[w][v][d];
    if (t != 0)
      __hip_atomic_fetch_add(bins + ((int64_t)(blockIdx.x % kXBins) * NV + v) * kXW + d, t,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <int NV>
__device__ __forceinline__ void xsum_flush(const int64_t (&acc)[NV], int64_t* __restrict__ bins) {
  __shared__ int64_t sh[4][NV][kXW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < kXW) {
#pragma unroll
    for (int v = 0; v < NV; ++v) sh[wid][v][lane] = acc[v];
  }
  xsum_flush_lds<NV>(sh, bins, (int)(blockDim.x >> 6));
}

// The consumer, one wave (of the last block / control): lane l < NV * kXW
// returns the bins' total of container l (sum v = l / kXW, digit l % kXW)
// and resets those bins for the next kernel (stream order).
template <int NV>
__device__ __forceinline__ int64_t xsum_collect(int64_t* __restrict__ bins, int lane) {
  int64_t t = 0;
  if (lane < NV * kXW) {
    const int v = lane / kXW, d = lane % kXW;
    // all bin loads in flight at once, then the (exact, order-free) sum,
    // then the clears: a load-add-clear per bin put 16 dependent memory
    // round trips into the serial tail of every CG iteration (~8 us)
    int64_t* a = bins + (int64_t)v * kXW + d;
    int64_t x[kXBins];
#pragma unroll
    for (int b = 0; b < kXBins; ++b)
      x[b] = __hip_atomic_load(a + (int64_t)b * NV * kXW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int b = 0; b < kXBins; ++b) t += x[b];
#pragma unroll
    for (int b = 0; b < kXBins; ++b)
      __hip_atomic_store(a + (int64_t)b * NV * kXW, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return t;
}

__device__ __forceinline__ float wave_sum_f32(float v) {
  v = xor_sum_f32<32>(v);
  v = xor_sum_f32<16>(v);
  v += dpp_f32<0x128>(v);
  v += dpp_f32<0x124>(v);
  v += dpp_f32<0x4E>(v);
  return v + dpp_f32<0xB1>(v);
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

// Cross-lane moves of a double through DPP (two 32-bit halves).  CTRL:
// quad_perm 0xB1 = lane ^ 1, 0x4E = lane ^ 2 (inside a quad); row_ror 0x124
// / 0x128 rotate a 16-lane row by 4 / 8.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {   // declared above
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}
// Sum over the 4 lanes of a quad; every lane of the quad gets the same value.
__device__ __forceinline__ double quad_sum_f64(double v) {
  v += dpp_f64<0xB1>(v);
  return v + dpp_f64<0x4E>(v);
}
// Sum over the 16 lanes of a row; lanes 0..3 of the row hold the same value,
// (Q0 + Q3) + (Q2 + Q1) over the row's quad sums Q (other lanes: other orders).
__device__ __forceinline__ double row_sum_f64(double v) {
  v = quad_sum_f64(v);
  v += dpp_f64<0x124>(v);
  return v + dpp_f64<0x128>(v);
}

constexpr int MV_WAVES = 4;

// Per-wave LDS scratch of the tile GEMV (one entity at a time).  The CG
// vectors are fp64 (a fp32 residual / direction breaks CG's recurrences on
// ill-conditioned blocks: DESIGN.md "Precision"), G is fp32 and every product
// G_ij v_j is accumulated in fp64.
template <int NB>
struct MvScratch {
  static constexpr int NF = NB / 2;
  double pv[16 * NB];              // the vector, virtual order
  double redR[NB][16];             // row sums (quad-reduced in registers)
  double redC[NB][256];            // 16-lane column partials: [b][16 rr + c]
  float dd[NF > 0 ? 16 * NF : 1];  // side-array diagonals of the folded tiles
};

// y = G_e v for ONE entity, by one wave, on tri16 tiles already in registers
// (lane l holds float4 l of every tile: T[l>>2][4(l&3) .. +3]).  Row products
// T v_bj go to y_bi, and for bi < bj column products T^T v_bi to y_bj, all in
// fp64.  Two passes with one block's accumulators live at a time -- block
// rows (summed over the 4 lanes of a row by DPP), then block columns (the
// 16-lane column partials through LDS) -- and a sched_barrier per tile, so the
// fp64 copies of the tiles are not all hoisted: the kernel fits 4 waves per
// SIMD.  Requires sc.pv (v in virtual order) and sc.dd staged.  Returns y at
// virtual index lane + 64 h in yo[h] (0 for padding, n >= k) and, user side,
// the bias row yb = Gs.v + Gn vb (wave-uniform); Gs_e / gn are the entity's
// row sums and count.  The user-side bias column Gs vb is added to every y.
// A diagonal block contributes only its stored triangle (the bf16x3 MFMA sum
// is not bitwise symmetric; mr_internal.h).
template <int NB, bool USER>
__device__ __forceinline__ void tile_matvec_finish(MvScratch<NB>& sc, double vb,
                                                   const float* __restrict__ Gs_e, float gn, int k,
                                                   double (&yo)[(16 * NB + 63) / 64], double& yb);

template <int NB, bool USER, bool OPAQUE = (NB > 4)>
__device__ __forceinline__ void tile_matvec(
    const float4 (&g)[NB * (NB - 1) / 2 + NB / 2 + (NB & 1)], MvScratch<NB>& sc, double vb,
    const float* __restrict__ Gs_e, float gn, int k, double (&yo)[(16 * NB + 63) / 64],
    double& yb) {
  constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2;
  const int lane = threadIdx.x & 63;
  const int rr = lane >> 2, c4 = (lane & 3) * 4;
  auto tile = [&](int t, double (&ge)[4]) {
    float4 gg = g[t];
    // NB > 4: an opaque copy, so the two passes convert each tile afresh
    // instead of keeping every tile's fp64 copy live between them (GVN would
    // merge the conversions: 352 -> 256 VGPRs, 2 waves/SIMD at k = 128; the
    // values are the same, so the results are bit-identical).  At NB <= 4 the
    // merged form fits 4 waves/SIMD and measured faster.
    if constexpr (OPAQUE) asm volatile("" : "+v"(gg.x), "+v"(gg.y), "+v"(gg.z), "+v"(gg.w));
    ge[0] = gg.x; ge[1] = gg.y; ge[2] = gg.z; ge[3] = gg.w;
  };
  // diagonal tile of block b and whether its stored triangle is the lower one
  auto diag_tile = [&](int b, bool& lower) {
    lower = (b & 1) && b < 2 * NF;
    return (b < 2 * NF) ? NO + (b >> 1) : NO + NF;
  };
  // pass 1: block rows, y_bi[rr] = sum_bj T(bi,bj)[rr][:] v_bj
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
    double s0 = 0.0;
#pragma unroll
    for (int bj = bi + 1; bj < NB; ++bj) {
      double ge[4];
      tile(off_index(bi, bj, NB), ge);
#pragma unroll
      for (int x = 0; x < 4; ++x) s0 = fma(ge[x], sc.pv[16 * bj + c4 + x], s0);
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      bool lower;
      const int t = diag_tile(bi, lower);
      double ge[4];
      tile(t, ge);
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int c = c4 + x;
        const bool use = lower ? (c < rr) : (c >= rr);   // lower: diagonal from dd
        s0 = fma(use ? ge[x] : 0.0, sc.pv[16 * bi + c], s0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const double rs = quad_sum_f64(s0);
    if ((lane & 3) == 0) sc.redR[bi][rr] = rs;
  }
  // pass 2: block columns, y_bj[c] += sum_{bi <= bj} T(bi,bj)[:][c] v_bi
  // (16-lane partials per column through LDS)
#pragma unroll
  for (int bj = 0; bj < NB; ++bj) {
    double cc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int bi = 0; bi < bj; ++bi) {
      double ge[4];
      tile(off_index(bi, bj, NB), ge);
      const double pi = sc.pv[16 * bi + rr];
#pragma unroll
      for (int x = 0; x < 4; ++x) cc[x] = fma(ge[x], pi, cc[x]);
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      bool lower;
      const int t = diag_tile(bj, lower);
      double ge[4];
      tile(t, ge);
      const double pr = sc.pv[16 * bj + rr];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int c = c4 + x;
        const bool use = lower ? (c < rr) : (c > rr);
        cc[x] = fma(use ? ge[x] : 0.0, pr, cc[x]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    double2* dst = reinterpret_cast<double2*>(&sc.redC[bj][4 * lane]);
    dst[0] = make_double2(cc[0], cc[1]);
    dst[1] = make_double2(cc[2], cc[3]);
  }
  tile_matvec_finish<NB, USER>(sc, vb, Gs_e, gn, k, yo, yb);
}

// The end of the tile GEMV, after the row sums (sc.redR) and the 16-lane
// column partials (sc.redC) of every block are in LDS: y in the fixed order
// redR + ((C0 + C1) + (C2 + C3)) over the column partials, the folded
// diagonals and, user side, the bias column / row.
template <int NB, bool USER>
__device__ __forceinline__ void tile_matvec_finish(MvScratch<NB>& sc, double vb,
                                                   const float* __restrict__ Gs_e, float gn, int k,
                                                   double (&yo)[(16 * NB + 63) / 64], double& yb) {
  constexpr int NF = NB / 2, NP = 16 * NB, NV = (NP + 63) / 64;
  const int lane = threadIdx.x & 63;
  __builtin_amdgcn_wave_barrier();
  double ybp = 0.0;
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;   // virtual index
    yo[h] = 0.0;
    if (o >= NP) continue;
    const int n = nat_of(o, NB);
    if (n >= k) continue;
    const int b = o >> 4, ii = o & 15;
    const double* C = &sc.redC[b][ii];
    double s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      s[j] = (C[16 * (4 * j)] + C[16 * (4 * j + 1)]) + (C[16 * (4 * j + 2)] + C[16 * (4 * j + 3)]);
    double y = sc.redR[b][ii] + ((s[0] + s[1]) + (s[2] + s[3]));
    if (NF > 0 && (b & 1) && b < 2 * NF) y = fma((double)sc.dd[(b >> 1) * 16 + ii], sc.pv[o], y);
    if (USER) {
      const double gs = Gs_e[n];
      y = fma(gs, vb, y);
      ybp = fma(gs, sc.pv[o], ybp);
    }
    yo[h] = y;
  }
  if (USER) yb = fma((double)gn, vb, wave_sum_f64(ybp));
}

// Streamed tile GEMV for NB > 4 (k = 65 ... 128): the same products, sums and
// order as tile_matvec, in ONE pass over the tiles instead of two passes over
// tiles held in registers (32 tiles = 128 VGPRs at k = 128: with the column
// partials and the CG vectors both the matvec and the one-pass kernel spilled).
// The tiles are consumed in block-row order -- row bi's strictly-upper tiles
// (bi, bj > bi), then its diagonal tile -- and each tile feeds both of its
// sums: the row sum of bi (T v_bj, summed over bj ascending and the diagonal
// last, as pass 1) and the column partials of bj (T^T v_bi, summed over bi
// ascending with bj's own diagonal last, as pass 2: every (bi < bj) tile of
// column bj precedes row bj's diagonal in this order).  Row bi's sum and
// column bi's partials are complete after row bi's diagonal and go to LDS
// there, so the live column accumulators shrink row by row.  Loads run
// TD tiles ahead of the tile being multiplied through a register ring:
// ring[] holds the stream's first TD tiles on entry (tile_stream_load), the
// rest are loaded from Ge (this lane's float4 of tile t at Ge[64 t + lane]).
template <int NB>
struct TileStream {   // load order: t[i] = tile index of the i-th tile consumed
  static constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF + (NB & 1);
  int t[NTILE];
  constexpr TileStream() : t() {
    int n = 0;
    for (int bi = 0; bi < NB; ++bi) {
      for (int bj = bi + 1; bj < NB; ++bj) t[n++] = bi * NB - bi * (bi + 1) / 2 + (bj - bi - 1);
      if ((bi & 1) == 0) t[n++] = bi < 2 * NF ? NO + bi / 2 : NO + NF;   // odd rows reuse it
    }
  }
};
// load position of tile (bi, bj > bi) / of row bi's diagonal tile (even bi)
__host__ __device__ constexpr int stream_pos_off(int bi, int bj, int nb) {
  return bi * nb - bi * (bi + 1) / 2 + (bj - bi - 1) + (bi + 1) / 2;
}
__host__ __device__ constexpr int stream_pos_diag(int bi, int nb) {
  return bi * nb - bi * (bi + 1) / 2 + (nb - 1 - bi) + (bi + 1) / 2;
}
template <int NB>
constexpr bool tile_stream_consistent() {
  constexpr TileStream<NB> S{};
  for (int bi = 0; bi < NB; ++bi) {
    for (int bj = bi + 1; bj < NB; ++bj)
      if (S.t[stream_pos_off(bi, bj, NB)] != bi * NB - bi * (bi + 1) / 2 + (bj - bi - 1)) return false;
    if ((bi & 1) == 0 &&
        S.t[stream_pos_diag(bi, NB)] != (bi < 2 * (NB / 2) ? NB * (NB - 1) / 2 + bi / 2
                                                            : NB * (NB - 1) / 2 + NB / 2))
      return false;
  }
  return true;
}
static_assert(tile_stream_consistent<5>() && tile_stream_consistent<6>() &&
                  tile_stream_consistent<7>() && tile_stream_consistent<8>(),
              "stream positions disagree with the load order");
// NB > 4 streams its tiles (MR_TS_STREAM 0: the two-pass register form)
#ifndef MR_TS_STREAM
#define MR_TS_STREAM 1
#endif
#ifndef MR_TS_AHEAD
#define MR_TS_AHEAD 12
#endif
template <int NB>
constexpr int ts_ahead() {
  constexpr int n = NB * (NB - 1) / 2 + NB / 2 + (NB & 1);
  return MR_TS_AHEAD < n ? MR_TS_AHEAD : n;
}
template <bool NT>
__device__ __forceinline__ float4 tile_ld(const floatx4* __restrict__ Ge, int t, int lane) {
  const floatx4 v = NT ? __builtin_nontemporal_load(Ge + t * 64 + lane) : Ge[t * 64 + lane];
  return make_float4(v[0], v[1], v[2], v[3]);
}
template <int NB, bool NT>
__device__ __forceinline__ void tile_stream_load(const floatx4* __restrict__ Ge, int lane,
                                                 float4 (&ring)[ts_ahead<NB>()]) {
  constexpr TileStream<NB> S{};
#pragma unroll
  for (int i = 0; i < ts_ahead<NB>(); ++i) ring[i] = tile_ld<NT>(Ge, S.t[i], lane);
}
template <int NB, bool USER, bool NT>
__device__ __forceinline__ void tile_matvec_stream(
    const floatx4* __restrict__ Ge, float4 (&ring)[ts_ahead<NB>()], MvScratch<NB>& sc, double vb,
    const float* __restrict__ Gs_e, float gn, int k, double (&yo)[(16 * NB + 63) / 64],
    double& yb) {
  constexpr TileStream<NB> S{};
  constexpr int NTILE = TileStream<NB>::NTILE, NF = NB / 2, TD = ts_ahead<NB>();
  const int lane = threadIdx.x & 63;
  const int rr = lane >> 2, c4 = (lane & 3) * 4;
  // take the tile at load position i and refill its ring slot with i + TD
  auto take = [&](int i, double (&ge)[4]) {
    float4 gg = ring[i % TD];
    if (i + TD < NTILE) ring[i % TD] = tile_ld<NT>(Ge, S.t[i + TD], lane);
    ge[0] = gg.x; ge[1] = gg.y; ge[2] = gg.z; ge[3] = gg.w;
  };
  double cc[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) cc[b][0] = cc[b][1] = cc[b][2] = cc[b][3] = 0.0;
  double dge[4] = {0.0, 0.0, 0.0, 0.0};   // the folded diagonal tile, kept for the odd row
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
    double s0 = 0.0;
    const double pi = sc.pv[16 * bi + rr];
#pragma unroll
    for (int bj = bi + 1; bj < NB; ++bj) {
      double ge[4];
      take(stream_pos_off(bi, bj, NB), ge);
#pragma unroll
      for (int x = 0; x < 4; ++x) s0 = fma(ge[x], sc.pv[16 * bj + c4 + x], s0);
#pragma unroll
      for (int x = 0; x < 4; ++x) cc[bj][x] = fma(ge[x], pi, cc[bj][x]);
      // the products happen here, not where their sums are next needed (the
      // compiler otherwise sinks them and keeps the tiles' fp64 copies live)
      asm volatile("" : "+v"(s0), "+v"(cc[bj][0]), "+v"(cc[bj][1]), "+v"(cc[bj][2]), "+v"(cc[bj][3]));
      __builtin_amdgcn_sched_barrier(0);
    }
    if ((bi & 1) == 0) take(stream_pos_diag(bi, NB), dge);
    const bool lower = (bi & 1) && bi < 2 * NF;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int c = c4 + x;
      const bool use = lower ? (c < rr) : (c >= rr);   // lower: diagonal from dd
      s0 = fma(use ? dge[x] : 0.0, sc.pv[16 * bi + c], s0);
    }
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int c = c4 + x;
      const bool use = lower ? (c < rr) : (c > rr);
      cc[bi][x] = fma(use ? dge[x] : 0.0, pi, cc[bi][x]);
    }
    const double rs = quad_sum_f64(s0);
    if ((lane & 3) == 0) sc.redR[bi][rr] = rs;
    double2* dst = reinterpret_cast<double2*>(&sc.redC[bi][4 * lane]);
    dst[0] = make_double2(cc[bi][0], cc[bi][1]);
    dst[1] = make_double2(cc[bi][2], cc[bi][3]);
    __builtin_amdgcn_sched_barrier(0);
  }
  tile_matvec_finish<NB, USER>(sc, vb, Gs_e, gn, k, yo, yb);
}

// CG start for ONE entity, by one wave, in block form (cg_least_squares,
// matrix.cpp:464-476 and the first matvec / dot of its loop, :493-497):
//   r0 = G x - c,  p0 = -r0,  q0 = G p0
// written to the (fp64) CG vectors; this wave's lanes add r0.r0 to drr,
// p0.q0 to dpq and q0.q0 to dqq (callers reduce in a fixed order; the
// one-pass CG derives r1.r1 from them, r0.q0 being exactly -p0.q0).  G / Gs / Gn / C / Cb hold
// the entity's finished normal equations (after slab_reduce for split
// entities).
template <int NB, bool USER>
__device__ __forceinline__ void cg_start_entity(int64_t e, int k, int ldk,
                                                const GramDst& D, const CgStart& cs,
                                                MvScratch<NB>& sc, double& drr, double& dpq,
                                                double& dqq) {
  constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF + (NB & 1);
  constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  const int lane = threadIdx.x & 63;
  // x in natural order (staged to LDS in virtual order); c at the natural
  // column of this lane's y slot h (virtual index lane + 64 h)
  float xv[NV], cn[NV];
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int i = lane + 64 * h;
    xv[h] = (i < NP) ? cs.x[e * ldk + i] : 0.f;
    cn[h] = (i < NP) ? D.C[e * D.sV + nat_of(i, NB)] : 0.f;
  }
  const double xb = USER ? (double)cs.xb[e] : 0.0;
  const double cb = USER ? (double)D.Cb[e * D.sS] : 0.0;
  const float gn = USER ? D.Gn[e * D.sS] : 0.f;
  const float* Gs_e = USER ? D.Gs + e * D.sV : nullptr;
  const float4* __restrict__ Ge = reinterpret_cast<const float4*>(D.G + e * D.sG);
  float4 g[NTILE];
#pragma unroll
  for (int t = 0; t < NTILE; ++t) g[t] = Ge[t * 64 + lane];
  if (NF > 0 && lane < 16 * NF) sc.dd[lane] = D.G[e * D.sG + NTILE * 256 + lane];
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int i = lane + 64 * h;
    if (i < NP) sc.pv[virt_of(i, NB)] = xv[h];
  }
  __builtin_amdgcn_wave_barrier();
  double yo[NV], yb = 0.0;
  tile_matvec<NB, USER>(g, sc, xb, Gs_e, gn, k, yo, yb);
  __builtin_amdgcn_wave_barrier();
  // r0 = G x - c, p0 = -r0 (:468-476); p0 replaces x in LDS
  double d = 0.0;
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;
    if (o < NP) {
      const int n = nat_of(o, NB);
      double pn = 0.0;
      if (n < k) {
        const double rv = yo[h] - (double)cn[h];
        cs.r[e * ldk + n] = rv;
        cs.p[e * ldk + n] = -rv;
        d = fma(rv, rv, d);
        pn = -rv;
      }
      sc.pv[o] = pn;
    }
  }
  double pb = 0.0;
  if (USER) {
    const double rbv = yb - cb;
    pb = -rbv;
    if (lane == 0) {
      cs.rb[e] = rbv;
      cs.pb[e] = pb;
      d = fma(rbv, rbv, d);
    }
  }
  drr += wave_sum_f64(d);
  __builtin_amdgcn_wave_barrier();
  // q0 = G p0 and p0.q0 (:493-497)
  tile_matvec<NB, USER>(g, sc, pb, Gs_e, gn, k, yo, yb);
  d = 0.0;
  double dq = 0.0;
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;
    if (o < NP) {
      const int n = nat_of(o, NB);
      if (n < k) {
        cs.q[e * ldk + n] = yo[h];
        d = fma(yo[h], sc.pv[o], d);
        dq = fma(yo[h], yo[h], dq);
      }
    }
  }
  if (USER && lane == 0) {
    cs.qb[e] = yb;
    d = fma(yb, pb, d);
    dq = fma(yb, yb, dq);
  }
  dpq += wave_sum_f64(d);
  dqq += wave_sum_f64(dq);
  __builtin_amdgcn_wave_barrier();
}

// Fixed-order (r.r, p.Gp, q.q) triple per block: wave partials summed in wave
// order.
__device__ __forceinline__ void store_start_sums(double drr, double dpq, double dqq,
                                                 double* parts) {
  __shared__ double shp[4][3];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    shp[wid][0] = drr;
    shp[wid][1] = dpq;
    shp[wid][2] = dqq;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, c = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      a += shp[w][0];
      b += shp[w][1];
      c += shp[w][2];
    }
    parts[3 * (int64_t)blockIdx.x] = a;
    parts[3 * (int64_t)blockIdx.x + 1] = b;
    parts[3 * (int64_t)blockIdx.x + 2] = c;
  }
}

// NB contiguous floats at p (16-B aligned when NB % 4 == 0).
template <int NB>
__device__ __forceinline__ void load_row_seg(float (&v)[NB], const float* __restrict__ p) {
  if constexpr (NB % 4 == 0) {
#pragma unroll
    for (int h = 0; h < NB / 4; ++h) {
      const float4 t = reinterpret_cast<const float4*>(p)[h];
      v[4 * h] = t.x; v[4 * h + 1] = t.y; v[4 * h + 2] = t.z; v[4 * h + 3] = t.w;
    }
  } else if constexpr (NB % 2 == 0) {
#pragma unroll
    for (int h = 0; h < NB / 2; ++h) {
      const float2 t = reinterpret_cast<const float2*>(p)[h];
      v[2 * h] = t.x; v[2 * h + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int b = 0; b < NB; ++b) v[b] = p[b];
  }
}

// Per-wave LDS of the accumulator-based CG start (start_from_acc).
template <int NB>
struct StartScratch {
  double pv[16 * NB];                // the vector, virtual order
  double partR[4 * NB][64];          // [4 bi + r][lane]: row-product partials
  double yC[16 * NB];                // column-product sums
  float sC[16 * NB];                 // rhs c, virtual order
  float sGs[16 * NB];                // user side: row sums, virtual order
};

// Accumulator tile of upper block (bi, bj), bi <= bj, row-major upper order.
__host__ __device__ constexpr int acc_tile(int bi, int bj, int nb) {
  return bi * nb - bi * (bi - 1) / 2 + (bj - bi);
}

// y = G v straight from the MFMA accumulators of the Gram wave (no memory
// round trip), products accumulated in fp64.  acc[t(bi,bj)] (bi <= bj,
// diagonal blocks FULL) holds B[4q + r][col] in lane (q, col).  Row products
// B v_bj go to y_bi (per-lane partials summed over the 16 lanes of row q
// through LDS -- a DPP tree cost 4x the instructions), column products
// B^T v_bi to y_bj (summed over the 4 rows by lane shuffles), both in a
// fixed order; a diagonal block contributes its stored triangle only.
// One tile's fp64 copy live at a time: this epilogue must fit the main
// loop's register budget (3 waves per SIMD at k = 64), so tile conversions
// are not hoisted (sched_barrier).  v in sc.pv (virtual order).  Returns y at virtual
// o = lane + 64 h in yo[h] (without the bias column) -- 0 for padding.
// TILE(bi, bj) returns the accumulator tile of upper block (bi, bj) (the Gram
// wave's own registers, or -- the NB = 8 pair kernel -- the partner wave's LDS
// dump).
// OWN(bi, bj): whether this wave holds block (bi, bj) (the pair kernel's
// split start: each wave takes its own tiles' products, the two partial
// results are added afterwards); partR / yC: where the row partials and the
// column sums go.
template <int NB, bool SB, class TILE, class OWN>
__device__ __forceinline__ void acc_matvec_g(TILE&& tile, OWN&& own, StartScratch<NB>& sc,
                                             double (*partR)[64], double* yC, int k,
                                             double (&yo)[(16 * NB + 63) / 64]);
template <int NB, bool SB = false, class TILE>
__device__ __forceinline__ void acc_matvec_t(TILE&& tile, StartScratch<NB>& sc, int k,
                                             double (&yo)[(16 * NB + 63) / 64]) {
  acc_matvec_g<NB, SB>(tile, [](int, int) { return true; }, sc, sc.partR, sc.yC, k, yo);
}
template <int NB, bool SB, class TILE, class OWN>
__device__ __forceinline__ void acc_matvec_g(TILE&& tile, OWN&& own, StartScratch<NB>& sc,
                                             double (*partR)[64], double* yC, int k,
                                             double (&yo)[(16 * NB + 63) / 64]) {
  constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  const int lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  // One pass over the upper tiles, block rows in order, each row starting at
  // its diagonal block: every accumulator is converted to fp64 once and feeds
  // both its row product y_bi[4q + r] += B(bi,bj)[4q + r][col] v_bj[col]
  // (lane partials, summed over the 16 lanes of row group q through LDS) and
  // its column product y_bj[col] += B(bi,bj)[4q + r][col] v_bi[4q + r] (a
  // per-lane running sum per block column, contributions in bi order --
  // column bi is complete once row bi is done).
  double cc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) cc[b] = 0.0;
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
    const bool lower = (bi & 1) && !((NB & 1) && bi == NB - 1);
    double R[4] = {0.0, 0.0, 0.0, 0.0};
    const double2 va = *reinterpret_cast<const double2*>(&sc.pv[16 * bi + 4 * q]);
    const double2 vb = *reinterpret_cast<const double2*>(&sc.pv[16 * bi + 4 * q + 2]);
    const double vr[4] = {va.x, va.y, vb.x, vb.y};   // v_bi at rows 4q + r
#pragma unroll
    for (int bj = bi; bj < NB; ++bj) {
      if (!own(bi, bj)) continue;
      const double vj = sc.pv[16 * bj + col];
      const floatx4 at = tile(bi, bj);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        const double a = (double)at[r];
        // diagonal block: the bf16x3 sum is not bitwise symmetric, so use
        // exactly the triangle tri16 stores (upper for even blocks and the
        // odd last block, lower + side diagonal for odd folded blocks); the
        // column product skips the diagonal element the row product used
        const bool use_r = bi != bj || (lower ? (col <= row) : (col >= row));
        const bool use_c = bi != bj || (lower ? (col < row) : (col > row));
        R[r] = fma(use_r ? a : 0.0, vj, R[r]);
        cc[bj] = fma(use_c ? a : 0.0, vr[r], cc[bj]);
      }
#ifdef MR_ACC_SB   // per-tile scheduling barrier (off: Gram users / items -1 %)
      __builtin_amdgcn_sched_barrier(0);
#else
      // SB (the pair kernel, whose tiles partly come from LDS): one tile's
      // loads at a time, not all 36 hoisted
      if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
#endif
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) partR[4 * bi + r][lane] = R[r];
    double c = xor_sum_f64<16>(cc[bi]);
    c = xor_sum_f64<32>(c);   // identical in all 4 rows
    if (q == 0) yC[16 * bi + col] = c;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;
    yo[h] = 0.0;
    if (o >= NP || nat_of(o, NB) >= k) continue;
    // row 4q + r of block b: the 16 lanes (q, 0..15) of partial r
    const int b = o >> 4, i = o & 15;
    const double2* pr = reinterpret_cast<const double2*>(&partR[4 * b + (i & 3)][16 * (i >> 2)]);
    double s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double2 v = pr[j];
      s[j] = v.x + v.y;
    }
    const double rs = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    yo[h] = rs + yC[o];
  }
  __builtin_amdgcn_wave_barrier();
}
template <int NB>
__device__ __forceinline__ void acc_matvec(const floatx4 (&acc)[NB * (NB + 1) / 2],
                                           StartScratch<NB>& sc, int k,
                                           double (&yo)[(16 * NB + 63) / 64]) {
  acc_matvec_t<NB>([&](int bi, int bj) { return acc[acc_tile(bi, bj, NB)]; }, sc, k, yo);
}

// Fused CG start of one unsplit entity from the Gram wave's registers
// (cg_least_squares, matrix.cpp:464-476 and iteration 0's matvec / dot,
// :493-497, in block form): r0 = G x - c, p0 = -r0, q0 = G p0, written to
// the fp64 CG vectors; adds r0.r0 to drr, p0.q0 to dpq and q0.q0 to dqq
// (lane partials summed across the wave).  cacc / sacc: c and the row sums at virtual
// (b, col) in every lane (already reduced over q); wt / gn: user-side
// sum of ratings and count; xv / xb: x at virtual (b, col) and its bias.
// The start's inputs in StartScratch (lanes q == 0): x (virtual order) for
// the NB segments in [b0, b1), and c / the row sums of those segments.
template <int NB, bool USER, int NL>
__device__ __forceinline__ void start_stage(const float (&cacc)[NL], const float (&sacc)[NL],
                                            int b0, int k, StartScratch<NB>& sc) {
  const int lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  if (q == 0) {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int b = b0 + j;
      const bool live = NB * col + b < k;   // natural column of virtual (b, col)
      sc.sC[16 * b + col] = live ? cacc[j] : 0.f;
      if (USER) sc.sGs[16 * b + col] = live ? sacc[j] : 0.f;
    }
  }
}
template <int NB>
__device__ __forceinline__ void start_stage_x(const float (&xv)[NB], StartScratch<NB>& sc) {
  const int lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  if (q == 0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) sc.pv[16 * b + col] = xv[b];
  }
}
// The start itself once its inputs are staged (start_stage / start_stage_x),
// on the accumulator tiles TILE(t).
// The start after y = G x (yo, virtual order): r0 = y - c (+ bias column),
// p0 = -r0 written to the CG vectors, r0.r0 added to drr, p0 into sc.pv
// (and pn / pb for the q0 step).
template <int NB, bool USER>
__device__ __forceinline__ void start_r0(const double (&yo)[(16 * NB + 63) / 64], float wt,
                                         float gn, float xb, int64_t e, int k, int ldk,
                                         const CgStart& cs, StartScratch<NB>& sc, double& drr,
                                         double (&pn)[(16 * NB + 63) / 64], double& pb) {
  constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  const int lane = threadIdx.x & 63;
  const double xbd = xb;
  double d = 0.0, ybp = 0.0;
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;
    pn[h] = 0.0;
    if (o < NP) {
      const int n = nat_of(o, NB);
      if (n < k) {
        double y = yo[h];
        if (USER) {
          const double gs = sc.sGs[o];
          y = fma(gs, xbd, y);
          ybp = fma(gs, sc.pv[o], ybp);
        }
        const double rv = y - (double)sc.sC[o];
        cs.r[e * ldk + n] = rv;
        cs.p[e * ldk + n] = -rv;
        d = fma(rv, rv, d);
        pn[h] = -rv;
      }
    }
  }
  pb = 0.0;
  if (USER) {
    const double rbv = fma((double)gn, xbd, wave_sum_f64(ybp)) - (double)wt;
    pb = -rbv;
    if (lane == 0) {
      cs.rb[e] = rbv;
      cs.pb[e] = pb;
      d = fma(rbv, rbv, d);
    }
  }
  drr += wave_sum_f64(d);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;
    if (o < NP) sc.pv[o] = pn[h];
  }
  __builtin_amdgcn_wave_barrier();
}
// The start after q0 = G p0 (yo): q0 written, p0.q0 and q0.q0 added.
template <int NB, bool USER>
__device__ __forceinline__ void start_q0(const double (&yo)[(16 * NB + 63) / 64], float gn,
                                         double pb, const double (&pn)[(16 * NB + 63) / 64],
                                         int64_t e, int k, int ldk, const CgStart& cs,
                                         StartScratch<NB>& sc, double& dpq, double& dqq) {
  constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  const int lane = threadIdx.x & 63;
  double d = 0.0, ybp = 0.0, dq = 0.0;
#pragma unroll
  for (int h = 0; h < NV; ++h) {
    const int o = lane + 64 * h;
    if (o < NP) {
      const int n = nat_of(o, NB);
      if (n < k) {
        double y = yo[h];
        if (USER) {
          const double gs = sc.sGs[o];
          y = fma(gs, pb, y);
          ybp = fma(gs, pn[h], ybp);
        }
        cs.q[e * ldk + n] = y;
        d = fma(y, pn[h], d);
        dq = fma(y, y, dq);
      }
    }
  }
  if (USER) {
    const double qb = fma((double)gn, pb, wave_sum_f64(ybp));
    if (lane == 0) {
      cs.qb[e] = qb;
      d = fma(qb, pb, d);
      dq = fma(qb, qb, dq);
    }
  }
  dpq += wave_sum_f64(d);
  dqq += wave_sum_f64(dq);
}
// The start itself once its inputs are staged (start_stage / start_stage_x),
// on the accumulator tiles TILE(bi, bj).
template <int NB, bool USER, bool SB = false, class TILE>
__device__ __forceinline__ void start_from_tiles(TILE&& tile, float wt, float gn, float xb,
                                                 int64_t e, int k, int ldk, const CgStart& cs,
                                                 StartScratch<NB>& sc, double& drr, double& dpq,
                                                 double& dqq) {
  constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  __builtin_amdgcn_wave_barrier();
  double yo[NV], pn[NV], pb;
  acc_matvec_t<NB, SB>(tile, sc, k, yo);
  start_r0<NB, USER>(yo, wt, gn, xb, e, k, ldk, cs, sc, drr, pn, pb);
  // q0 = G p0 (+ bias column), p0.q0
  acc_matvec_t<NB, SB>(tile, sc, k, yo);
  start_q0<NB, USER>(yo, gn, pb, pn, e, k, ldk, cs, sc, dpq, dqq);
}
template <int NB, bool USER>
__device__ __forceinline__ void start_from_acc(const floatx4 (&acc)[NB * (NB + 1) / 2],
                                               const float (&cacc)[NB], const float (&sacc)[NB],
                                               float wt, float gn, const float (&xv)[NB],
                                               float xb, int64_t e, int k, int ldk,
                                               const CgStart& cs, StartScratch<NB>& sc,
                                               double& drr, double& dpq, double& dqq) {
  start_stage_x<NB>(xv, sc);
  start_stage<NB, USER, NB>(cacc, sacc, 0, k, sc);
  start_from_tiles<NB, USER>([&](int bi, int bj) { return acc[acc_tile(bi, bj, NB)]; }, wt, gn,
                             xb, e, k, ldk, cs, sc, drr, dpq, dqq);
}

// ---------------------------------------------------------------------------
// K1: gather-Gram.  One wave per WorkItem (an entity, or a chunk of a heavy
// entity).  Rows a_r are gathered from the opposite factor table (row stride
// ldk floats) and accumulated on the matrix cores with
// v_mfma_f32_16x16x32_bf16 in an exact bf16x3 split (below).  Only the
// NB(NB+1)/2 upper 16 x 16 blocks are computed (k = 64: 10 of 16), and the
// accumulators are stored as they stand: D[row = 4(l>>4) + reg][col = l&15]
// is exactly the row-major tile layout of tri16 storage, so the epilogue needs
// no transpose (diagonal blocks are masked into their folded tile / side
// array).  The rhs and (user side) row sums / counts ride along on VALU.
// Item side: w = r - U[u][k] (fill_ratings_minus_bias, :1021-1030).
//
// bf16x3: v_mfma_f32_16x16x32_bf16 takes, in lane (q, col), 8 consecutive K
// values of row / column col.  With K = ratings that is "ratings 8q .. 8q+7
// of virtual column 16b + col", which is what lane (q, col) holds after
// gathering rows 8q + t (t < 8) of a 32-rating half with its NB-float
// segment per row: the operands need no transpose.  Each float is split
// EXACTLY into three bf16 by truncation (h = top 16 bits, m = top 16 bits of
// a - h, l = a - h - m, which has <= 8 significant bits), and each block
// accumulates the six products of weight >= 2^-16 of h h^T: hh + hm + mh +
// hl + lh + mm (the dropped ml, lm, ll are <= 2^-24 relative, below the fp32
// rounding of the sum).
// ---------------------------------------------------------------------------


// Per-lane raw loads of one 32-rating half: opposite id, rating and (item
// side) the opposite bias.  Lanes past the end of the work item load from a
// safe in-range address and are masked (id -> the all-zero row `zrow`,
// weight 0) only when the half becomes current, so no select waits on a load
// that was just issued.
struct ChunkRaw {
  int idx;
  float r;
  float b;
};
struct ChunkRegs {
  int idx;
  float w;
};

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Lane (q, col) gathers rows 8q .. 8q+7 of a 32-rating half, NB contiguous
// floats each from its column base Fc (natural columns NB col .. NB col +
// NB-1 = virtual (b, col)).  Rating 8q + t of the half sits in lane 16q + t
// (and 16q + 8 + t) of the ChunkRegs (half_slot), so its id / weight reach the
// 16 lanes of row q by one DPP row_newbcast:t (no LDS permute).
__device__ __forceinline__ int half_slot(int lane) { return 8 * (lane >> 4) + (lane & 7); }
template <int T>
__device__ __forceinline__ int row_bcast(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + T, 0xF, 0xF, false);
}
// Row source: a 64-bit base (any table size), or (BUF, tables < 2 GiB) a
// buffer resource with a 32-bit byte offset -- one shift-or per row instead
// of 64-bit address arithmetic; out-of-range offsets read 0.
struct RowSrc {
  const char* Fc;                 // 64-bit path: table + this lane's column offset
  __amdgpu_buffer_rsrc_t rsrc;    // BUF path: whole table
  uint32_t colb;                  // BUF path: this lane's column offset, bytes
};
// Timing probes of the Gram's streams (wrong results; never in the product
// build): MR_PROBE_GRAM 1 drops the G stores, 3 sends them all to the first
// 8 entities' G (an L2-resident region: the same stores without their HBM
// writes), 2 the row gathers (each row
// replaced by a value derived from its id, so the id / weight stream stays)
#ifndef MR_PROBE_GRAM
#define MR_PROBE_GRAM 0
#endif
template <int NB, int T, bool BUF>
__device__ __forceinline__ void gather_row(float (&f)[8][NB], float (&w)[8], ChunkRegs cr,
                                           const RowSrc& src, uint32_t row_bytes) {
  const int ri = row_bcast<T>(cr.idx);
  w[T] = __builtin_bit_cast(float, row_bcast<T>(__builtin_bit_cast(int, cr.w)));
  if constexpr (MR_PROBE_GRAM == 2) {
#pragma unroll
    for (int b = 0; b < NB; ++b) f[T][b] = (float)(ri + b) * 1e-6f;
  } else if constexpr (BUF) {
    const uint32_t off = (uint32_t)ri * row_bytes + src.colb;
#pragma unroll
    for (int h = 0; h < NB / 4; ++h) {
      const floatx4 v = __builtin_bit_cast(
          floatx4, __builtin_amdgcn_raw_buffer_load_b128(src.rsrc, (int)(off + 16 * h), 0, 0));
      f[T][4 * h] = v[0]; f[T][4 * h + 1] = v[1]; f[T][4 * h + 2] = v[2]; f[T][4 * h + 3] = v[3];
    }
  } else {
    load_row_seg<NB>(f[T],
                     reinterpret_cast<const float*>(src.Fc + (uint64_t)(uint32_t)ri * row_bytes));
  }
}
template <int NB, bool BUF, int... T>
__device__ __forceinline__ void gather_rows(float (&f)[8][NB], float (&w)[8], ChunkRegs cr,
                                            const RowSrc& src, uint32_t row_bytes,
                                            std::integer_sequence<int, T...>) {
  (gather_row<NB, T, BUF>(f, w, cr, src, row_bytes), ...);
}
template <int NB, bool BUF>
__device__ __forceinline__ void gather_half(float (&f)[8][NB], float (&w)[8], ChunkRegs cr,
                                            const RowSrc& src, uint32_t row_bytes) {
  gather_rows<NB, BUF>(f, w, cr, src, row_bytes, std::make_integer_sequence<int, 8>{});
}

// rhs c = sum a w and (user side) row sums, fp32 on VALU, per lane over its
// 8 ratings (the 4 q-groups are combined in the epilogue); then the exact
// 3-way split, packed 2 ratings per dword (rating 2j in the low half).
template <int NB, bool USER>
__device__ __forceinline__ void bf3_split(u32x4_t (&P)[3][NB], u32x4_t& W, float (&cacc)[NB],
                                          float (&sacc)[NB], float& wsum,
                                          const float (&f)[8][NB], const float (&w)[8],
                                          bool rhs_mfma) {
  if (USER) {
#pragma unroll
    for (int t = 0; t < 8; ++t) wsum += w[t];
  }
  if (rhs_mfma) {
    // user side, every weight exact in bf16: the rhs and the row sums are
    // taken by the matrix cores as a 16-column block W (column 0: the
    // weights, column 1: ones; gram_wave), whose B operand is built here
    const int col = threadIdx.x & 15;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t wv = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, w[2 * j + 1]),
                                                __builtin_bit_cast(uint32_t, w[2 * j]), 0x07060302u);
      W[j] = col == 0 ? wv : (col == 1 ? 0x3F803F80u : 0u);
    }
  } else {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        cacc[b] = fmaf(f[t][b], w[t], cacc[b]);
        if (USER) sacc[b] += f[t][b];
      }
    }
  }
  // a = h + m + l per float: r = a - h, l = r - m (h, m = the value with its
  // low 16 bits cleared), then the bf16 pairs of ratings (2j, 2j+1) packed
  // by v_perm.  Plain f32 subtracts, not v_pk_add_f32: beside MFMAs a packed
  // f32 op costs more issue time than the two single ones it replaces
  // (MI355X_MICROARCH.md), and this file is built with -fno-slp-vectorize so
  // the compiler does not re-pack them.
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      uint32_t R[2], L[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float a = f[2 * j + u][b];
        const float r = a - __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, a) & 0xFFFF0000u);
        R[u] = __builtin_bit_cast(uint32_t, r);
        L[u] = __builtin_bit_cast(uint32_t, r - __builtin_bit_cast(float, R[u] & 0xFFFF0000u));
      }
      P[0][b][j] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, f[2 * j + 1][b]),
                                         __builtin_bit_cast(uint32_t, f[2 * j][b]), 0x07060302u);
      P[1][b][j] = __builtin_amdgcn_perm(R[1], R[0], 0x07060302u);
      P[2][b][j] = __builtin_amdgcn_perm(L[1], L[0], 0x07060302u);
    }
  }
}

// hh, hm, mh, hl, lh, mm over the NB(NB+1)/2 upper blocks, product-major
// (consecutive MFMAs write different accumulators: no dependency stalls).
// Wait states around the inline-asm MFMAs (NB >= 5).  LLVM's hazard
// recognizer sees an asm statement as an opaque instruction, so it inserts
// none of the gfx950 MFMA wait states for it; these guards make them explicit
// instead of relying on the surrounding code's length:
//   * before the first MFMA of a half: VALU writes of P (the split) and of the
//     accumulators (their zeroing) -> MFMA SrcA/B/C reads need <= 2 wait
//     states on gfx940+; s_nop 4 gives 5;
//   * after the last MFMA, before the epilogue reads the accumulators: an
//     8-pass XDL result -> VALU / v_accvgpr_read needs NumPasses + 3 (+1 on
//     gfx950) = 12 wait states; three s_nop give 8 + 8 + 4 = 20.
// sched_barrier(0) on both sides keeps the scheduler from moving any
// instruction across a guard.  A plain nop statement is not enough after the
// last MFMA: the compiler placed its accumulator copies (v_accvgpr_read)
// right behind the MFMA, above the nops, so the exit guard takes every
// accumulator as an operand (below).  tests/test_asm_guards.py disassembles
// the gfx950 code object and counts both gaps on every NB >= 5 instance, so a
// change that shortens them fails the CPU suite.
__device__ __forceinline__ void mfma_entry_guard() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4");
  __builtin_amdgcn_sched_barrier(0);
}
// The exit guard names every accumulator as an in/out AGPR operand (the nop
// statement first, then operand-only statements in groups of four, volatile
// and so kept in order): a read of any accumulator -- including the copies
// the compiler makes for the epilogue -- depends on a statement at or after
// the nops and cannot be scheduled between the last MFMA and them.
template <int T>
__device__ __forceinline__ void acc_tie(floatx4 (&acc)[T], int g0) {
#pragma unroll
  for (int g = g0; g < T; g += 4) {
    __builtin_amdgcn_sched_barrier(0);
    if (g + 3 < T)
      asm volatile("" : "+a"(acc[g]), "+a"(acc[g + 1]), "+a"(acc[g + 2]), "+a"(acc[g + 3]));
    else if (g + 2 < T)
      asm volatile("" : "+a"(acc[g]), "+a"(acc[g + 1]), "+a"(acc[g + 2]));
    else if (g + 1 < T)
      asm volatile("" : "+a"(acc[g]), "+a"(acc[g + 1]));
    else
      asm volatile("" : "+a"(acc[g]));
  }
  __builtin_amdgcn_sched_barrier(0);
}
template <int T, int TW>
__device__ __forceinline__ void mfma_exit_guard(floatx4 (&acc)[T], floatx4 (&accw)[TW], bool w) {
  static_assert(T >= 4, "NB >= 5 only");
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]));
  acc_tie(acc, 4);
  if (w) acc_tie(accw, 0);   // user side: the W block's accumulators too
}

template <int NB, bool USER>
__device__ __forceinline__ void bf3_mfma(floatx4 (&acc)[NB * (NB + 1) / 2], floatx4 (&accw)[NB],
                                         const u32x4_t (&P)[3][NB], const u32x4_t& W,
                                         bool rhs_mfma) {
  if constexpr (NB >= 5) mfma_entry_guard();
#pragma unroll
  for (int sidx = 0; sidx < 6; ++sidx) {
    const int pa = (sidx == 2) ? 1 : (sidx == 4) ? 2 : (sidx == 5) ? 1 : 0;
    const int pb = (sidx == 1) ? 1 : (sidx == 3) ? 2 : (sidx == 5) ? 1 : 0;
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = bi; bj < NB; ++bj) {
        if constexpr (NB >= 5) {
          // the same instruction with the accumulator pinned to AGPRs: with
          // the builtin, the allocator kept part of the NB >= 5 accumulators
          // in VGPRs inside the loop and copied them to / from AGPRs every
          // half (200 v_accvgpr_* per half at NB = 8; loop 984 -> 783
          // instructions; k = 128 Gram users 1313 -> 1255 us, items 1001 ->
          // 960 us same-box, bit-identical).  Hazard wait states: explicit
          // guards (mfma_entry_guard above, mfma_exit_guard after the loop).
          asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
              : "+a"(acc[t]) : "v"(P[pa][bi]), "v"(P[pb][bj]));
        } else {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, P[pa][bi]), __builtin_bit_cast(bf16x8_t, P[pb][bj]),
              acc[t], 0, 0, 0);
        }
        ++t;
      }
  }
  if (USER && rhs_mfma) {
    // W block: D[m][0] += a[16 b + m] w (rhs), D[m][1] += a[16 b + m] (row
    // sums); the weights are exact in bf16, so the three parts of a give
    // every product of weight >= 2^-16 of the fp32 ones
#pragma unroll
    for (int part = 0; part < 3; ++part)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if constexpr (NB >= 5) {
          asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(accw[b]) : "v"(P[part][b]), "v"(W));
        } else {
          accw[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, P[part][b]), __builtin_bit_cast(bf16x8_t, W), accw[b],
              0, 0, 0);
        }
      }
  }
}

// Stores of the Gram's tri16 G (MR_G_NT: non-temporal, so the stream of G
// does not evict the gathered factor table from the Infinity Cache)
#ifndef MR_G_NT
#define MR_G_NT 1
#endif
// MR_G_SC1 (A/B knob): the G stores write-through (`sc1`: the line leaves
// L2 instead of staying there dirty)
#ifndef MR_G_SC1
#define MR_G_SC1 0
#endif
__device__ __forceinline__ void gst(float* p, float v) {
  if (MR_PROBE_GRAM == 1) return;
  if (MR_G_SC1) asm volatile("global_store_dword %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
  else if (MR_G_NT && MR_PROBE_GRAM != 3) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// MR_G_WIDE: a tile leaves as ONE 16-byte store per lane (the whole 1 KiB
// tile contiguous per wave instruction) instead of four 4-byte stores of
// 4 x 64 B.  Lane (q, 4j + i) holds rows 4q .. 4q+3 of column 4j + i; a
// quad-local 4 x 4 transpose (DPP quad_perm: lane ^ 2, then lane ^ 1) gives
// it row 4q + i, columns 4j .. 4j+3.  Same bytes at the same addresses.
#ifndef MR_G_WIDE
#define MR_G_WIDE 0
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_quad(float s) {
  return __builtin_bit_cast(float,
                            __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ floatx4 quad_transpose(floatx4 v, int i) {
  const bool hi = (i & 2) != 0, odd = (i & 1) != 0;
  float r0 = dpp_quad<0x4E>(hi ? v[0] : v[2]);   // quad_perm [2,3,0,1]
  float r1 = dpp_quad<0x4E>(hi ? v[1] : v[3]);
  if (hi) { v[0] = r0; v[1] = r1; } else { v[2] = r0; v[3] = r1; }
  r0 = dpp_quad<0xB1>(odd ? v[0] : v[1]);         // quad_perm [1,0,3,2]
  r1 = dpp_quad<0xB1>(odd ? v[2] : v[3]);
  if (odd) { v[0] = r0; v[2] = r1; } else { v[1] = r0; v[3] = r1; }
  return v;
}
__device__ __forceinline__ void gst4(float* p, floatx4 v) {
  if (MR_PROBE_GRAM == 1) return;
  // s_nop: a store of more than 8 bytes reads its data VGPRs after issue, so
  // a VALU write to them needs wait states the hazard recognizer cannot see
  // through an asm statement
  if (MR_G_SC1)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
  else if (MR_G_NT && MR_PROBE_GRAM != 3) __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p));
  else *reinterpret_cast<floatx4*>(p) = v;
}

template <int NB, bool USER, bool FUSE, bool BUF>
__device__ __forceinline__ void gram_wave(
    int64_t wi, const WorkItem* __restrict__ work,
    const int32_t* __restrict__ idx, const float* __restrict__ val,
    const float* __restrict__ F, const float* __restrict__ bias, int k, int ldk, int zrow,
    const GramDst& direct, const GramDst& slab, const CgStart& cs, StartScratch<NB>* ssc,
    double& drr, double& dpq, double& dqq, bool rhs_mfma) {
  constexpr int T = NB * (NB + 1) / 2;
  const int lane = threadIdx.x & 63;
  // work-item fields in SGPRs: all control flow below is scalar
  const int64_t wbeg = work[wi].begin;
  const int wlen = work[wi].len;
  const int went = work[wi].entity;
  const int wslab = work[wi].slab;
  const int q = lane >> 4, col = lane & 15;
  const int64_t end = wbeg + wlen;
  constexpr uint32_t row_bytes = 64u * NB;     // ldk = 16 NB floats
  RowSrc src;
  src.Fc = reinterpret_cast<const char*>(F) + 4 * NB * col;
  src.colb = 4u * NB * (uint32_t)col;
  if constexpr (BUF)
    src.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(F), (short)0,
                                                 (int)((uint32_t)(zrow + 1) * row_bytes),
                                                 0x00020000);

  // fused CG start: this lane's x entries (virtual (b, col) = natural
  // NB*col + b, contiguous) are fetched now and used after the loop
  float xv[NB];
  float xbv = 0.f;
  if constexpr (FUSE) {
    const int64_t xe = (wslab < 0) ? (int64_t)went : 0;
    load_row_seg<NB>(xv, cs.x + xe * ldk + NB * col);
    if (USER) xbv = cs.xb[xe];
  }

  floatx4 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 accw[NB];   // user side: the W block (rhs, row sums), see bf3_mfma
#pragma unroll
  for (int b = 0; b < NB; ++b) accw[b] = floatx4{0.f, 0.f, 0.f, 0.f};
  float cacc[NB], sacc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) { cacc[b] = 0.f; sacc[b] = 0.f; }
  float wsum = 0.f;
  rhs_mfma = USER && rhs_mfma;

  // Main loop: one iteration = one 32-rating half with its own id / weight
  // registers (lanes 0..31; lanes 32..63 mirror them), so the loop body is
  // uniform: ONE split site and ONE MFMA site (two call sites per iteration
  // made the compiler rotate the accumulators through extra AGPRs every
  // iteration).  The half's rows land in F; once split into P (and the rhs
  // taken), F is refilled with the next half while P's MFMAs run.  Rows past
  // the end are the zero row with weight 0.  F is loaded and consumed inside
  // one iteration and only VALU results (P) cross the back-edge, so no
  // register copy there ever waits on a load in flight.
  const int64_t safe = wlen > 0 ? wbeg : 0;    // an address every wave may read
  const int slot = half_slot(lane);
  auto ld32 = [&](int c) {
    const int64_t jj = wbeg + 32 * (int64_t)c + slot;
    ChunkRaw r;
    const int64_t js = jj < end ? jj : safe;
    r.idx = idx[js];
    r.r = val[js];
    r.b = 0.f;
    return r;
  };
  auto bias32 = [&](ChunkRaw& cr, int c) {
    if (!USER) {
      const bool ok = wbeg + 32 * (int64_t)c + slot < end;
      cr.b = bias[ok ? cr.idx : zrow];
    }
  };
  auto fin32 = [&](const ChunkRaw& cr, int c) {
    const bool ok = wbeg + 32 * (int64_t)c + slot < end;
    ChunkRegs r;
    r.idx = ok ? cr.idx : zrow;
    r.w = ok ? cr.r - cr.b : 0.f;
    return r;
  };
  ChunkRaw h1 = ld32(1), h2 = ld32(2);
  ChunkRaw h0 = ld32(0);
  bias32(h0, 0);
  bias32(h1, 1);
  float Fr[8][NB], w[8];
  u32x4_t P[3][NB], W;
  gather_half<NB, BUF>(Fr, w, fin32(h0, 0), src, row_bytes);
  bf3_split<NB, USER>(P, W, cacc, sacc, wsum, Fr, w, rhs_mfma);
  // the last half is peeled: its iteration would gather and split a half
  // past the end (zero rows, weight 0) that no MFMA uses -- about one half's
  // VALU work per work item (users: ~6 halves each)
  const int nhalves = (wlen + 31) >> 5;
  for (int h = 0; h < nhalves - 1; ++h) {
    const ChunkRaw h3 = ld32(h + 3);
    bias32(h2, h + 2);
    gather_half<NB, BUF>(Fr, w, fin32(h1, h + 1), src, row_bytes);
    bf3_mfma<NB, USER>(acc, accw, P, W, rhs_mfma);
    __builtin_amdgcn_sched_barrier(0);
    bf3_split<NB, USER>(P, W, cacc, sacc, wsum, Fr, w, rhs_mfma);
    h1 = h2;
    h2 = h3;
  }
  if (nhalves > 0) bf3_mfma<NB, USER>(acc, accw, P, W, rhs_mfma);
  if constexpr (NB >= 5) mfma_exit_guard(acc, accw, USER);

  // ---- epilogue -----------------------------------------------------------
  // c and (user side) the row sums at virtual (b, col) in every lane: from
  // the per-lane VALU partials (summed over the 4 rating groups q), or from
  // the W block, whose D[4 q' + r][n] sits in lane (q', n) register r
  // (n = 0: rhs, n = 1: row sums) -- lane (q, col) takes register col & 3
  // of lane 16 (col >> 2) + n
  if (rhs_mfma) {
    const int s0 = 16 * (col >> 2), r = col & 3;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v0[4], v1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v0[j] = __shfl(accw[b][j], s0, 64);
        v1[j] = __shfl(accw[b][j], s0 + 1, 64);
      }
      sacc[b] = r == 0 ? v1[0] : r == 1 ? v1[1] : r == 2 ? v1[2] : v1[3];
      cacc[b] = r == 0 ? v0[0] : r == 1 ? v0[1] : r == 2 ? v0[2] : v0[3];
    }
  } else {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      cacc[b] = xor_sum_f32<16>(cacc[b]);
      cacc[b] = xor_sum_f32<32>(cacc[b]);
      if (USER) {
        sacc[b] = xor_sum_f32<16>(sacc[b]);
        sacc[b] = xor_sum_f32<32>(sacc[b]);
      }
    }
  }
  const bool to_slab = wslab >= 0;
  const int64_t di = to_slab ? (int64_t)wslab : (int64_t)went;
  const GramDst& D = to_slab ? slab : direct;
  float* __restrict__ Gd = D.G + (MR_PROBE_GRAM == 3 ? (di & 7) : di) * D.sG;
  float* __restrict__ Cd = D.C + di * D.sV;
  if (q == 0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c = NB * col + b;   // natural column of virtual (b, col); c < ldk
      Cd[c] = (c < k) ? cacc[b] : 0.f;
      if (USER) D.Gs[di * D.sV + c] = (c < k) ? sacc[b] : 0.f;
    }
  }
  auto lane_f32 = [](float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  };
  const float wt = USER ? (lane_f32(wsum, 0) + lane_f32(wsum, 16)) +
                              (lane_f32(wsum, 32) + lane_f32(wsum, 48))
                        : 0.f;
  if (USER && lane == 0) {
    D.Cb[di * D.sS] = wt;
    D.Gn[di * D.sS] = (float)wlen;
  }
  // tri16 layout (mr_internal.h): off-diagonal blocks as full tiles, diagonal
  // blocks folded pairwise.  Branch-free: every lane stores all 4 rows of
  // every tile (a folded tile takes D_2m or D_2m+1 by a select), so the only
  // masked store is the side array; store offsets are compile-time except the
  // lane's 64 q + col.  (Per-element masked stores cost ~400 instructions of
  // exec-mask branches per wave.)  Plain stores: 4-byte sc1 write-through
  // stores, to keep the gathered rows in L2, made the kernel 4 % slower.
  constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF + (NB & 1);
  if constexpr (MR_G_WIDE) {
    float* __restrict__ Gw = Gd + 64 * q + 16 * (col & 3) + 4 * (col >> 2);
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
#pragma unroll
      for (int bj = bi + 1; bj < NB; ++bj) {
        const int t = acc_tile(bi, bj, NB), o = off_index(bi, bj, NB) * 256;
        gst4(&Gw[o], quad_transpose(acc[t], col & 3));
      }
    }
#pragma unroll
    for (int m = 0; m < NF; ++m) {
      const int te = acc_tile(2 * m, 2 * m, NB), to = acc_tile(2 * m + 1, 2 * m + 1, NB);
      float dg = 0.f;
      floatx4 f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        f[r] = col >= row ? acc[te][r] : acc[to][r];
        if (col - 4 * q == r) dg = acc[to][r];
      }
      gst4(&Gw[(NO + m) * 256], quad_transpose(f, col & 3));
      if ((col >> 2) == q) gst(&Gd[NTILE * 256 + m * 16 + col], dg);   // D_2m+1's diagonal
    }
    if constexpr ((NB & 1) != 0)
      gst4(&Gw[(NO + NF) * 256], quad_transpose(acc[acc_tile(NB - 1, NB - 1, NB)], col & 3));
  } else {
    float* __restrict__ Gl = Gd + 64 * q + col;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
#pragma unroll
      for (int bj = bi + 1; bj < NB; ++bj) {
        const int t = acc_tile(bi, bj, NB), o = off_index(bi, bj, NB) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) gst(&Gl[o + 16 * r], acc[t][r]);
      }
    }
#pragma unroll
    for (int m = 0; m < NF; ++m) {
      const int te = acc_tile(2 * m, 2 * m, NB), to = acc_tile(2 * m + 1, 2 * m + 1, NB);
      float dg = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        gst(&Gl[(NO + m) * 256 + 16 * r], col >= row ? acc[te][r] : acc[to][r]);
        if (col - 4 * q == r) dg = acc[to][r];
      }
      if ((col >> 2) == q) gst(&Gd[NTILE * 256 + m * 16 + col], dg);   // D_2m+1's diagonal
    }
    if constexpr ((NB & 1) != 0) {
      const int t = acc_tile(NB - 1, NB - 1, NB);
#pragma unroll
      for (int r = 0; r < 4; ++r) gst(&Gl[(NO + NF) * 256 + 16 * r], acc[t][r]);
    }
  }
  if constexpr (FUSE) {
    if (!to_slab)
      start_from_acc<NB, USER>(acc, cacc, sacc, wt, (float)wlen, xv, xbv, went, k, ldk, cs,
                               *ssc, drr, dpq, dqq);
  }
}

// Waves are independent: one work item each, no block barriers -- except in
// the FUSE form, whose waves then start the CG solve on their entity
// (start_from_acc; split entities are started after slab_reduce) and meet
// once at the end to store the block's (r.r, p.Gp) pair.
template <int NB, bool USER, bool FUSE, bool BUF, bool RHSM>
__global__ __launch_bounds__(64 * GRAM_WAVES, (NB <= 4 ? 3 : 1)) void gram_kernel(
    const WorkItem* __restrict__ work, int64_t n_work,
    const int32_t* __restrict__ idx, const float* __restrict__ val,
    const float* __restrict__ F, const float* __restrict__ bias, int k, int ldk, int zrow,
    GramDst direct, GramDst slab, CgStart cs) {
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wi = (int64_t)blockIdx.x * GRAM_WAVES + wid;
  double drr = 0.0, dpq = 0.0, dqq = 0.0;
  if constexpr (!FUSE) {
    if (wi >= n_work) return;
    gram_wave<NB, USER, false, BUF>(wi, work, idx, val, F, bias, k, ldk, zrow, direct, slab, cs,
                                    nullptr, drr, dpq, dqq, RHSM);
  } else {
    __shared__ StartScratch<NB> scr[GRAM_WAVES];
    if (wi < n_work)
      gram_wave<NB, USER, true, BUF>(wi, work, idx, val, F, bias, k, ldk, zrow, direct, slab,
                                     cs, &scr[wid], drr, dpq, dqq, RHSM);
    if (cs.xbins) {   // one-pass CG: the entity's start sums, order-independent
      const int lane = threadIdx.x & 63;
      const int64_t t3[3] = {xterm(drr, lane), xterm(dpq, lane), xterm(dqq, lane)};
      xsum_flush<3>(t3, cs.xbins);
    } else {
      store_start_sums(drr, dpq, dqq, cs.parts);
    }
  }
}

// ---------------------------------------------------------------------------
// K1 at NB = 8 (k = 113 ... 128, the C4 / C5 shapes): one work item on a PAIR
// of waves (round 5).  The one-wave form holds all 36 upper blocks (144
// AGPRs) beside the three bf16 parts of 8 segments (96 VGPRs) and the
// gathered rows: one wave per SIMD, issue-bound, the row-gather latency and
// the epilogue exposed.  Here wave r ("role") of a 128-thread block owns
// segments 4r .. 4r+3 of every gathered row (one dwordx4 per row per lane:
// half the gather instructions), splits them, and accumulates 18 blocks:
//   role 0: the 10 blocks inside segments 0-3, and (bi, bj), bi <= 3, bj = 4, 5
//   role 1: the 10 blocks inside segments 4-7, and (bi, bj), bi <= 3, bj = 6, 7
// so role 0 reads the partner's parts of segments 4, 5 and role 1 those of
// segments 0-3 from an LDS stage written once per 32-rating half (two
// barriers per half).  Every block is still accumulated by ONE wave, over the
// same halves with the same six products in the same order, so G is
// bitwise the one-wave kernel's.  Epilogue: each wave stores its own tiles
// (role 0 holds the folded diagonal pairs 0-1 and 2-3, role 1 4-5 and 6-7);
// the fused CG start is split over the pair (each wave takes the products of
// its own tiles, role 1 adds role 0's partials: a summation order of its
// own), or with MR_PAIR_SPLIT_START = 0 runs on role 1 over role 0's tiles
// dumped into the (then free) stage -- the one-wave kernel's acc_matvec
// arithmetic, bitwise its start.  Role 1 fetches x at the wave's start.
// Accumulators in VGPRs (mfma_acc), at most 256 registers per wave: two
// waves per SIMD.
// ---------------------------------------------------------------------------
constexpr int PAIR_T = 18;   // upper blocks per wave
// MR_PAIR_PREFETCH: the next half's rows are gathered while this half's
// MFMAs run (1, default) or after them (0).  MR_PAIR_SPLIT_START: the fused
// CG start split over both waves (1, default) or run by role 1 on a dump of
// role 0's tiles (0, bitwise the one-wave kernel's start).  Same box, fixed
// 10 CG iterations, ML-full k = 128 users / items Gram (profiles/r05/ab_pair):
// one wave 1.230 / 0.957 ms; pair 1.069-1.084 / 0.849-0.868 (both 0);
// prefetch 1.088 / 0.851; split start 1.084 / 0.868; both 1.058 / 0.838 ms.
#ifndef MR_PAIR_PREFETCH
#define MR_PAIR_PREFETCH 1
#endif
#ifndef MR_PAIR_SPLIT_START
#define MR_PAIR_SPLIT_START 1
#endif
__host__ __device__ constexpr int pair_owner(int bi, int bj) { return (bi <= 3 && bj <= 5) ? 0 : 1; }
__host__ __device__ constexpr int pair_local(int bi, int bj) {
  return pair_owner(bi, bj) == 0 ? (bj <= 3 ? acc_tile(bi, bj, 4) : 10 + 4 * (bj - 4) + bi)
                                 : (bi >= 4 ? acc_tile(bi - 4, bj - 4, 4) : 10 + 2 * bi + (bj - 6));
}
constexpr bool pair_partition_ok() {
  int seen[2][PAIR_T] = {};
  for (int bi = 0; bi < 8; ++bi)
    for (int bj = bi; bj < 8; ++bj) {
      const int o = pair_owner(bi, bj), l = pair_local(bi, bj);
      if (l < 0 || l >= PAIR_T || seen[o][l]) return false;
      seen[o][l] = 1;
    }
  return true;
}
static_assert(pair_partition_ok(), "the two waves' block lists must partition the 36 blocks");
// LDS stage of the partner parts: [segment 0..5][part][lane]; the same 1,152
// 16-byte slots hold role 0's 18 accumulator tiles in the epilogue
constexpr int PAIR_STAGE = 6 * 3 * 64;
static_assert(PAIR_STAGE == PAIR_T * 64, "stage and tile dump share the LDS array");

// Accumulators in arch VGPRs ("+v": the VGPR form of the MFMA): a kernel
// that uses no AGPR gets the whole 256-register budget of 2 waves / SIMD as
// VGPRs, where any AGPR use makes the allocator split it 128 / 128.
__device__ __forceinline__ void mfma_acc(floatx4& acc, const u32x4_t& a, const u32x4_t& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// mfma_exit_guard for VGPR accumulators: 20 wait states between the last
// MFMA and any reader of its result, in a statement that takes every
// accumulator as an operand (so no copy or read of one is scheduled above it)
template <int T, int TW>
__device__ __forceinline__ void mfma_exit_guard_v(floatx4 (&acc)[T], floatx4 (&accw)[TW]) {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
#pragma unroll
  for (int g = 4; g < T; g += 2) {
    __builtin_amdgcn_sched_barrier(0);
    if (g + 1 < T) asm volatile("" : "+v"(acc[g]), "+v"(acc[g + 1]));
    else asm volatile("" : "+v"(acc[g]));
  }
#pragma unroll
  for (int g = 0; g < TW; ++g) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" : "+v"(accw[g]));
  }
  __builtin_amdgcn_sched_barrier(0);
}
// s_waitcnt lgkmcnt(0) as the builtin (vmcnt / expcnt left at their maximum),
// so the waitcnt pass sees the partner operands already waited for and puts
// nothing between mfma_entry_guard's nops and the first MFMA
__device__ __forceinline__ void lds_wait() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// One half's MFMAs of a role (products hh, hm, mh, hl, lh, mm per block, in
// that order, as bf3_mfma).  P: this wave's own segments' parts; stg: the
// stage with the partner's.
template <int ROLE, bool USER>
__device__ __forceinline__ void pair_mfma(floatx4 (&acc)[PAIR_T], floatx4 (&accw)[4],
                                          const u32x4_t (&P)[3][4], const u32x4_t& W,
                                          bool rhs_mfma, const u32x4_t* __restrict__ stg,
                                          int lane) {
  auto seg = [&](u32x4_t (&X)[3], int s) {
    X[0] = stg[(3 * s + 0) * 64 + lane];
    X[1] = stg[(3 * s + 1) * 64 + lane];
    X[2] = stg[(3 * s + 2) * 64 + lane];
  };
  u32x4_t X[3], Y[3];
  if constexpr (ROLE == 0) {
    seg(X, 4);
    seg(Y, 5);
    mfma_entry_guard();
#pragma unroll
    for (int sidx = 0; sidx < 6; ++sidx) {
      const int pa = (sidx == 2) ? 1 : (sidx == 4) ? 2 : (sidx == 5) ? 1 : 0;
      const int pb = (sidx == 1) ? 1 : (sidx == 3) ? 2 : (sidx == 5) ? 1 : 0;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = bi; bj < 4; ++bj) mfma_acc(acc[acc_tile(bi, bj, 4)], P[pa][bi], P[pb][bj]);
    }
    lds_wait();
    mfma_entry_guard();
#pragma unroll
    for (int sidx = 0; sidx < 6; ++sidx) {
      const int pa = (sidx == 2) ? 1 : (sidx == 4) ? 2 : (sidx == 5) ? 1 : 0;
      const int pb = (sidx == 1) ? 1 : (sidx == 3) ? 2 : (sidx == 5) ? 1 : 0;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) mfma_acc(acc[10 + bi], P[pa][bi], X[pb]);
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) mfma_acc(acc[14 + bi], P[pa][bi], Y[pb]);
    }
  } else {
    seg(X, 0);
    seg(Y, 1);
    mfma_entry_guard();
#pragma unroll
    for (int sidx = 0; sidx < 6; ++sidx) {
      const int pa = (sidx == 2) ? 1 : (sidx == 4) ? 2 : (sidx == 5) ? 1 : 0;
      const int pb = (sidx == 1) ? 1 : (sidx == 3) ? 2 : (sidx == 5) ? 1 : 0;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = bi; bj < 4; ++bj) mfma_acc(acc[acc_tile(bi, bj, 4)], P[pa][bi], P[pb][bj]);
    }
    lds_wait();
    mfma_entry_guard();
#pragma unroll
    for (int sidx = 0; sidx < 6; ++sidx) {
      const int pa = (sidx == 2) ? 1 : (sidx == 4) ? 2 : (sidx == 5) ? 1 : 0;
      const int pb = (sidx == 1) ? 1 : (sidx == 3) ? 2 : (sidx == 5) ? 1 : 0;
      mfma_acc(acc[10], X[pa], P[pb][2]);
      mfma_acc(acc[11], X[pa], P[pb][3]);
      mfma_acc(acc[12], Y[pa], P[pb][2]);
      mfma_acc(acc[13], Y[pa], P[pb][3]);
    }
    seg(X, 2);
    seg(Y, 3);
    lds_wait();
    mfma_entry_guard();
#pragma unroll
    for (int sidx = 0; sidx < 6; ++sidx) {
      const int pa = (sidx == 2) ? 1 : (sidx == 4) ? 2 : (sidx == 5) ? 1 : 0;
      const int pb = (sidx == 1) ? 1 : (sidx == 3) ? 2 : (sidx == 5) ? 1 : 0;
      mfma_acc(acc[14], X[pa], P[pb][2]);
      mfma_acc(acc[15], X[pa], P[pb][3]);
      mfma_acc(acc[16], Y[pa], P[pb][2]);
      mfma_acc(acc[17], Y[pa], P[pb][3]);
    }
  }
  if (USER && rhs_mfma) {   // the W block of this wave's segments (bf3_mfma)
#pragma unroll
    for (int part = 0; part < 3; ++part)
#pragma unroll
      for (int b = 0; b < 4; ++b) mfma_acc(accw[b], P[part][b], W);
  }
}

// the segments a role writes into the stage for its partner (written out
// statement by statement: as a loop nest the compiler kept P in scratch
// memory and copied it with a runtime-indexed loop)
template <int S0, int PS, int... I>
__device__ __forceinline__ void pair_stage_put(const u32x4_t (&P)[3][4], u32x4_t* __restrict__ stg,
                                               int lane, std::integer_sequence<int, I...>) {
  ((stg[(3 * (S0 + I / 3) + I % 3) * 64 + lane] = P[I % 3][PS + I / 3]), ...);
}
template <int ROLE>
__device__ __forceinline__ void pair_stage_write(const u32x4_t (&P)[3][4],
                                                 u32x4_t* __restrict__ stg, int lane) {
  if constexpr (ROLE == 0) pair_stage_put<0, 0>(P, stg, lane, std::make_integer_sequence<int, 12>{});
  else pair_stage_put<4, 0>(P, stg, lane, std::make_integer_sequence<int, 6>{});
}

// Work-list position of pair block b: the list deals range x's chunks to
// positions p with (p / 4) mod 8 == x (four waves per one-wave Gram block,
// block b on XCD b mod 8); with one work item per block the same XCD holds
// position p = 32 g + 4 x + j for block b = 32 g + 8 j + x (a bijection on
// every full group of 32; the tail keeps p = b).
__device__ __forceinline__ int64_t pair_pos(int64_t b, int64_t n) {
  if (b >= (n & ~(int64_t)31)) return b;
  return 32 * (b >> 5) + 4 * (b & 7) + ((b >> 3) & 3);
}

// One wave of the pair, its role a template parameter: each role's code is
// compiled on its own (a runtime role made the compiler keep P in scratch).
template <int ROLE, bool USER, bool FUSE, bool BUF, bool RHSM>
__device__ __forceinline__ void gram_pair_wave(
    const WorkItem* __restrict__ work, int64_t n_work,
    const int32_t* __restrict__ idx, const float* __restrict__ val,
    const float* __restrict__ F, const float* __restrict__ bias, int k, int ldk, int zrow,
    const GramDst& direct, const GramDst& slab, const CgStart& cs, u32x4_t* __restrict__ stg,
    StartScratch<8>& sc) {
  constexpr int NB = 8;
  constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF;
  constexpr int role = ROLE;
  const int lane = threadIdx.x & 63;
  const int64_t wi = pair_pos(blockIdx.x, n_work);
  const bool rhs_mfma = USER && RHSM;
  double drr = 0.0, dpq = 0.0, dqq = 0.0;
  const int64_t wbeg = work[wi].begin;
  const int wlen = work[wi].len;
  const int went = work[wi].entity;
  const int wslab = work[wi].slab;
  const int q = lane >> 4, col = lane & 15;
  const int64_t end = wbeg + wlen;
  constexpr uint32_t row_bytes = 64u * NB;
  // fused start (role 1): this entity's x segment and bias, fetched now and
  // used after the halves (at the epilogue they were an exposed global load
  // per work item)
  float xpre[NB];
  float xbpre = 0.f;
  if constexpr (FUSE && ROLE == 1) {
    const int64_t xe = wslab < 0 ? (int64_t)went : 0;
    load_row_seg<NB>(xpre, cs.x + xe * ldk + NB * col);
    if (USER) xbpre = cs.xb[xe];
  }
  // this wave's 4 segments: floats 4 role .. 4 role + 3 of the lane's 8
  RowSrc src;
  src.Fc = reinterpret_cast<const char*>(F) + 4 * NB * col + 16 * role;
  src.colb = 4u * NB * (uint32_t)col + 16u * (uint32_t)role;
  if constexpr (BUF)
    src.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(F), (short)0,
                                                 (int)((uint32_t)(zrow + 1) * row_bytes),
                                                 0x00020000);
  floatx4 acc[PAIR_T];
#pragma unroll
  for (int t = 0; t < PAIR_T; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 accw[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) accw[b] = floatx4{0.f, 0.f, 0.f, 0.f};
  float cacc[4], sacc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) { cacc[b] = 0.f; sacc[b] = 0.f; }
  float wsum = 0.f;
  const int64_t safe = wlen > 0 ? wbeg : 0;
  const int slot = half_slot(lane);
  auto ld32 = [&](int c) {
    const int64_t jj = wbeg + 32 * (int64_t)c + slot;
    ChunkRaw r;
    const int64_t js = jj < end ? jj : safe;
    r.idx = idx[js];
    r.r = val[js];
    r.b = 0.f;
    return r;
  };
  auto bias32 = [&](ChunkRaw& cr, int c) {
    if (!USER) {
      const bool ok = wbeg + 32 * (int64_t)c + slot < end;
      cr.b = bias[ok ? cr.idx : zrow];
    }
  };
  auto fin32 = [&](const ChunkRaw& cr, int c) {
    const bool ok = wbeg + 32 * (int64_t)c + slot < end;
    ChunkRegs r;
    r.idx = ok ? cr.idx : zrow;
    r.w = ok ? cr.r - cr.b : 0.f;
    return r;
  };
  ChunkRaw h1 = ld32(1), h2 = ld32(2);
  ChunkRaw h0 = ld32(0);
  bias32(h0, 0);
  bias32(h1, 1);
  float Fr[8][4], w[8];
  u32x4_t P[3][4], W;
  gather_half<4, BUF>(Fr, w, fin32(h0, 0), src, row_bytes);
  bf3_split<4, USER>(P, W, cacc, sacc, wsum, Fr, w, rhs_mfma);
  pair_stage_write<ROLE>(P, stg, lane);
  __syncthreads();
  const int nhalves = (wlen + 31) >> 5;
  for (int h = 0; h < nhalves - 1; ++h) {
    const ChunkRaw h3 = ld32(h + 3);
    bias32(h2, h + 2);
#if MR_PAIR_PREFETCH
    // the next half's rows in flight during this half's MFMAs
    gather_half<4, BUF>(Fr, w, fin32(h1, h + 1), src, row_bytes);
    pair_mfma<ROLE, USER>(acc, accw, P, W, rhs_mfma, stg, lane);
#else
    // the next half's rows gathered after this half's MFMAs are issued (a
    // second wave per SIMD, of another pair, covers the latency)
    pair_mfma<ROLE, USER>(acc, accw, P, W, rhs_mfma, stg, lane);
    __builtin_amdgcn_sched_barrier(0);
    gather_half<4, BUF>(Fr, w, fin32(h1, h + 1), src, row_bytes);
#endif
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();   // both waves done reading this half's stage
    bf3_split<4, USER>(P, W, cacc, sacc, wsum, Fr, w, rhs_mfma);
    pair_stage_write<ROLE>(P, stg, lane);
    __syncthreads();   // the next half's stage complete
    h1 = h2;
    h2 = h3;
  }
  if (nhalves > 0) pair_mfma<ROLE, USER>(acc, accw, P, W, rhs_mfma, stg, lane);
  mfma_exit_guard_v(acc, accw);

  // ---- epilogue (gram_wave's, over this wave's segments and blocks) -------
  if (rhs_mfma) {
    const int s0 = 16 * (col >> 2), r = col & 3;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float v0[4], v1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v0[j] = __shfl(accw[b][j], s0, 64);
        v1[j] = __shfl(accw[b][j], s0 + 1, 64);
      }
      sacc[b] = r == 0 ? v1[0] : r == 1 ? v1[1] : r == 2 ? v1[2] : v1[3];
      cacc[b] = r == 0 ? v0[0] : r == 1 ? v0[1] : r == 2 ? v0[2] : v0[3];
    }
  } else {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      cacc[b] = xor_sum_f32<16>(cacc[b]);
      cacc[b] = xor_sum_f32<32>(cacc[b]);
      if (USER) {
        sacc[b] = xor_sum_f32<16>(sacc[b]);
        sacc[b] = xor_sum_f32<32>(sacc[b]);
      }
    }
  }
  const bool to_slab = wslab >= 0;
  const int64_t di = to_slab ? (int64_t)wslab : (int64_t)went;
  const GramDst& D = to_slab ? slab : direct;
  float* __restrict__ Gd = D.G + (MR_PROBE_GRAM == 3 ? (di & 7) : di) * D.sG;
  float* __restrict__ Cd = D.C + di * D.sV;
  if (q == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = NB * col + 4 * role + j;   // natural column of virtual (4 role + j, col)
      Cd[c] = (c < k) ? cacc[j] : 0.f;
      if (USER) D.Gs[di * D.sV + c] = (c < k) ? sacc[j] : 0.f;
    }
  }
  auto lane_f32 = [](float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  };
  const float wt = USER ? (lane_f32(wsum, 0) + lane_f32(wsum, 16)) +
                              (lane_f32(wsum, 32) + lane_f32(wsum, 48))
                        : 0.f;
  if (USER && role == 0 && lane == 0) {
    D.Cb[di * D.sS] = wt;
    D.Gn[di * D.sS] = (float)wlen;
  }
  float* __restrict__ Gl = Gd + 64 * q + col;
  float* __restrict__ Gw = Gd + 64 * q + 16 * (col & 3) + 4 * (col >> 2);   // MR_G_WIDE
  auto store_tiles = [&](auto own) {
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
#pragma unroll
      for (int bj = bi + 1; bj < NB; ++bj) {
        if (pair_owner(bi, bj) != decltype(own)::value) continue;
        const int t = pair_local(bi, bj), o = off_index(bi, bj, NB) * 256;
        if constexpr (MR_G_WIDE) {
          gst4(&Gw[o], quad_transpose(acc[t], col & 3));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) gst(&Gl[o + 16 * r], acc[t][r]);
        }
      }
    }
#pragma unroll
    for (int m = 2 * decltype(own)::value; m < 2 * decltype(own)::value + 2; ++m) {
      const int te = pair_local(2 * m, 2 * m), to = pair_local(2 * m + 1, 2 * m + 1);
      float dg = 0.f;
      floatx4 f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        f[r] = col >= row ? acc[te][r] : acc[to][r];
        if (!MR_G_WIDE) gst(&Gl[(NO + m) * 256 + 16 * r], f[r]);
        if (col - 4 * q == r) dg = acc[to][r];
      }
      if (MR_G_WIDE) gst4(&Gw[(NO + m) * 256], quad_transpose(f, col & 3));
      if ((col >> 2) == q) gst(&Gd[NTILE * 256 + m * 16 + col], dg);   // D_2m+1's diagonal
    }
  };
  store_tiles(std::integral_constant<int, ROLE>{});
  if constexpr (FUSE) {
    if (!to_slab) {
      // The start runs on role 1 from its own accumulators (registers) and
      // role 0's, dumped into the stage (free once both waves have passed
      // the barrier behind the last half): the same tiles and the same
      // acc_matvec arithmetic as the one-wave kernel, so the start is
      // bitwise its start.  (Reading the tiles back from the stored tri16
      // G instead -- 4 strided loads per tile per pass -- cost 3 x the
      // one-wave kernel's start.)
      start_stage<NB, USER, 4>(cacc, sacc, 4 * role, k, sc);
#if MR_PAIR_SPLIT_START
      // Split start: each wave takes the products of ITS tiles (from its
      // registers) and role 1 adds role 0's partial result to its own
      // (y = y0 + y1): both waves work, no tile dump -- but a summation
      // order of its own, so the start is not bitwise the one-wave kernel's.
      // Role 0's row partials / column sums / partial y live in the stage.
      constexpr int NV = 2;
      double (*partR0)[64] = reinterpret_cast<double (*)[64]>(stg);
      double* yC0 = reinterpret_cast<double*>(stg) + 32 * 64;
      double* Y0 = yC0 + 16 * NB;
      __syncthreads();   // both waves done with the stage
      if constexpr (ROLE == 1) start_stage_x<NB>(xpre, sc);
      __syncthreads();
      auto own = [](int bi, int bj) { return pair_owner(bi, bj) == ROLE; };
      auto mine = [&](int bi, int bj) {
        floatx4 t = acc[pair_local(bi, bj)];
        asm volatile("" : "+v"(t));   // converted afresh in each pass
        return t;
      };
      double yo[NV], pn[NV], pb = 0.0;
      const float xbv = (USER && ROLE == 1) ? xbpre : 0.f;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        acc_matvec_g<NB, true>(mine, own, sc, ROLE == 0 ? partR0 : sc.partR,
                               ROLE == 0 ? yC0 : sc.yC, k, yo);
        if constexpr (ROLE == 0) {
#pragma unroll
          for (int h = 0; h < NV; ++h) Y0[lane + 64 * h] = yo[h];
        }
        __syncthreads();
        if constexpr (ROLE == 1) {
#pragma unroll
          for (int h = 0; h < NV; ++h) yo[h] = Y0[lane + 64 * h] + yo[h];
          if (pass == 0) start_r0<NB, USER>(yo, wt, (float)wlen, xbv, went, k, ldk, cs, sc, drr, pn, pb);
          else start_q0<NB, USER>(yo, (float)wlen, pb, pn, went, k, ldk, cs, sc, dpq, dqq);
        }
        __syncthreads();   // p0 in sc.pv before the second pass
      }
#else
      floatx4* dump = reinterpret_cast<floatx4*>(stg);
      __syncthreads();   // both waves done with the stage
      if constexpr (ROLE == 0) {
#pragma unroll
        for (int t = 0; t < PAIR_T; ++t) dump[t * 64 + lane] = acc[t];
      } else {
        start_stage_x<NB>(xpre, sc);
      }
      __syncthreads();
      if constexpr (ROLE == 1) {
        const float xbv = USER ? xbpre : 0.f;
        start_from_tiles<NB, USER, true>(
            [&](int bi, int bj) {
              floatx4 t = pair_owner(bi, bj) == 1 ? acc[pair_local(bi, bj)]
                                                  : dump[pair_local(bi, bj) * 64 + lane];
              // opaque per call: the two acc_matvec passes convert the tiles
              // afresh instead of the compiler keeping (spilling) the fp64
              // copies of the first pass for the second
              asm volatile("" : "+v"(t));
              return t;
            },
            wt, (float)wlen, xbv, went, k, ldk, cs, sc, drr, dpq, dqq);
      }
#endif
    }
    if (cs.xbins) {   // one-pass CG: the entity's start sums, order-independent
      const int64_t t3[3] = {xterm(drr, lane), xterm(dpq, lane), xterm(dqq, lane)};
      xsum_flush<3>(t3, cs.xbins);
    } else {
      store_start_sums(drr, dpq, dqq, cs.parts);
    }
  }
}

template <bool USER, bool FUSE, bool BUF, bool RHSM>
__global__ __launch_bounds__(128, 2) void gram_pair_kernel(
    const WorkItem* __restrict__ work, int64_t n_work,
    const int32_t* __restrict__ idx, const float* __restrict__ val,
    const float* __restrict__ F, const float* __restrict__ bias, int k, int ldk, int zrow,
    GramDst direct, GramDst slab, CgStart cs) {
  __shared__ u32x4_t stg[PAIR_STAGE];
  __shared__ StartScratch<8> sc;   // role 1's (the start runs on one wave)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0)
    gram_pair_wave<0, USER, FUSE, BUF, RHSM>(work, n_work, idx, val, F, bias, k, ldk, zrow,
                                             direct, slab, cs, stg, sc);
  else
    gram_pair_wave<1, USER, FUSE, BUF, RHSM>(work, n_work, idx, val, F, bias, k, ldk, zrow,
                                             direct, slab, cs, stg, sc);
}

// Split entities: the CG start after slab_reduce (one wave per entity).
// the folded CG_START control, run by wave 0 of cg_start_split's last block
// (defined with the control kernel below)
__device__ void start_fold_finalize(const StartFold& f, int64_t* start_xbins);

template <int NB, bool USER>
__global__ __launch_bounds__(256) void cg_start_split_kernel(const SplitItem* __restrict__ split,
                                                             int64_t n_split, int k, int ldk,
                                                             GramDst direct, CgStart cs,
                                                             double* __restrict__ parts,
                                                             StartFold fold) {
  __shared__ MvScratch<NB> scr[4];
  const int wid = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 4 + wid;
  double drr = 0.0, dpq = 0.0, dqq = 0.0;
  if (i < n_split)
    cg_start_entity<NB, USER>(split[i].entity, k, ldk, direct, cs, scr[wid], drr, dpq, dqq);
  if (cs.xbins) {
    const int lane = threadIdx.x & 63;
    const int64_t t3[3] = {xterm(drr, lane), xterm(dpq, lane), xterm(dqq, lane)};
    xsum_flush<3>(t3, cs.xbins);
    if (fold.st) {
      // last-arriving block: every block's bin atomics are drained (vmcnt)
      // before its arrival add, as in the one-pass kernel's hand-off
      __shared__ int s_last;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's bin atomics
      __syncthreads();
      if (threadIdx.x == 0) {
        s_last = __hip_atomic_fetch_add(&fold.st->arrive_start, 1u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
      }
      __syncthreads();
      if (s_last && wid == 0) start_fold_finalize(fold, cs.xbins);
    }
  } else {
    store_start_sums(drr, dpq, dqq, parts);
  }
}

template <int NB>
static int launch_gram_nb(hipStream_t s, bool user_side, int k, const WorkItem* work,
                          int64_t n_work, const int32_t* idx, const float* val,
                          const float* F, const float* bias, int zrow, GramDst direct,
                          GramDst slab, const CgStart* start, bool rhs_mfma) {
  if (n_work <= 0) return 0;
  const CgStart cs = start ? *start : CgStart{};
  if constexpr (NB == 8 && MR_GRAM_PAIR) {   // one work item per pair of waves
    const bool buf = (int64_t)(zrow + 1) * ldk_of(k) * 4 < ((int64_t)1 << 31);
#define MR_GP(U, FU, B, R)                                                                     \
  MR_LAUNCH((gram_pair_kernel<U, FU, B, R>), dim3((unsigned)n_work), dim3(128), 0, s, work,    \
            n_work, idx, val, F, bias, k, ldk_of(k), zrow, direct, slab, cs)
#define MR_GP_B(U, FU, R) \
  if (buf) MR_GP(U, FU, true, R); else MR_GP(U, FU, false, R);
    if (user_side) {
      if (rhs_mfma) {
        if (start) { MR_GP_B(true, true, true) } else { MR_GP_B(true, false, true) }
      } else {
        if (start) { MR_GP_B(true, true, false) } else { MR_GP_B(true, false, false) }
      }
    } else {
      if (start) { MR_GP_B(false, true, false) } else { MR_GP_B(false, false, false) }
    }
#undef MR_GP_B
#undef MR_GP
    MR_HIP(hipGetLastError());
    return 0;
  }
  const int64_t grid = (n_work + GRAM_WAVES - 1) / GRAM_WAVES;
  // buffer-resource gathers when the whole table (zrow + 1 rows) is < 2 GiB
  // and the row segment is whole dwordx4s (NB = 4, 8)
  constexpr bool BUFOK = NB % 4 == 0;
  const bool buf = BUFOK && (int64_t)(zrow + 1) * ldk_of(k) * 4 < ((int64_t)1 << 31);
#define MR_GRAM_LAUNCH(U, FU, B, R)                                                          \
  MR_LAUNCH((gram_kernel<NB, U, FU, B, R>), dim3((unsigned)grid), dim3(64 * GRAM_WAVES), 0, s, work, n_work, \
            idx, val, F, bias, k, ldk_of(k), zrow, direct, slab, cs)
#define MR_GRAM_USER(FU, B)                                                                 \
  if (rhs_mfma) MR_GRAM_LAUNCH(true, FU, B, true); else MR_GRAM_LAUNCH(true, FU, B, false);
  if (buf) {
    if (user_side) {
      if (start) { MR_GRAM_USER(true, BUFOK) } else { MR_GRAM_USER(false, BUFOK) }
    } else {
      if (start) MR_GRAM_LAUNCH(false, true, BUFOK, false); else MR_GRAM_LAUNCH(false, false, BUFOK, false);
    }
  } else {
    if (user_side) {
      if (start) { MR_GRAM_USER(true, false) } else { MR_GRAM_USER(false, false) }
    } else {
      if (start) MR_GRAM_LAUNCH(false, true, false, false); else MR_GRAM_LAUNCH(false, false, false, false);
    }
  }
#undef MR_GRAM_USER
#undef MR_GRAM_LAUNCH
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// K1 for k < 32 (NB <= 2): the same normal equations on the VALU, fp32 FMAs
// in rating order (north star: matrix cores only for k >= 32; a 16 x 16 MFMA
// tile would waste most of its work on k = 10).  One wave per work item;
// chunks of 64 ratings: lane t gathers rating t's factor row into LDS in
// virtual order (v = 16 b + i <-> n = NB i + b, mr_internal.h), then every
// lane accumulates its entries over the chunk.  Lane l owns virtual rows
// rr + 16 bi (rr = l >> 2) and columns c4 + 16 bj .. + 3 (c4 = 4 (l & 3)) of
// the upper blocks (bi <= bj), diagonal blocks in full, so its 4 entries of a
// block are exactly float4 l of that block's row-major tile: the tri16 stores
// are one float4 per lane per tile.  rhs c (and, user side, the row sums) in
// the lanes' rows; the count / rating sum are wave-uniform.
// ---------------------------------------------------------------------------
template <int NB, bool USER>
__global__ __launch_bounds__(256) void gram_valu_kernel(
    const WorkItem* __restrict__ work, int64_t n_work, const int32_t* __restrict__ idx,
    const float* __restrict__ val, const float* __restrict__ F, const float* __restrict__ bias,
    int k, int zrow, GramDst direct, GramDst slab) {
  static_assert(NB == 1 || NB == 2, "VALU Gram: k < 32");
  constexpr int LD = 16 * NB;                 // ldk, floats per factor row
  constexpr int NBLK = NB * (NB + 1) / 2;     // upper blocks
  __shared__ float rows[4][64][LD + 1];       // +1: rows of a chunk on distinct banks
  __shared__ float wts[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wi = (int64_t)blockIdx.x * 4 + wid;
  if (wi >= n_work) return;
  const int64_t wbeg = work[wi].begin;
  const int wlen = work[wi].len;
  const int went = work[wi].entity, wslab = work[wi].slab;
  const int rr = lane >> 2, c4 = 4 * (lane & 3);
  float acc[NBLK][4];
#pragma unroll
  for (int t = 0; t < NBLK; ++t) acc[t][0] = acc[t][1] = acc[t][2] = acc[t][3] = 0.f;
  float cacc[NB], sacc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) cacc[b] = sacc[b] = 0.f;
  float wsum = 0.f;
  float (&R)[64][LD + 1] = rows[wid];
  for (int base = 0; base < wlen; base += 64) {
    const int n = min(64, wlen - base);
    {
      const bool ok = lane < n;
      const int id = ok ? idx[wbeg + base + lane] : zrow;
      float w = ok ? val[wbeg + base + lane] : 0.f;
      if (!USER) w -= bias[id];              // r - U[u][k] (fill_ratings_minus_bias); 0 - 0 past the end
      const float4* src = reinterpret_cast<const float4*>(F + (int64_t)id * LD);
#pragma unroll
      for (int h = 0; h < LD / 4; ++h) {
        const float4 a = src[h];
        const float e[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const int nn = 4 * h + x;            // natural column
          R[lane][16 * (nn % NB) + nn / NB] = e[x];
        }
      }
      wts[wid][lane] = w;
    }
    __builtin_amdgcn_wave_barrier();
    for (int t = 0; t < n; ++t) {
      const float w = wts[wid][t];
      float ar[NB], ac[NB][4];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        ar[b] = R[t][16 * b + rr];
#pragma unroll
        for (int x = 0; x < 4; ++x) ac[b][x] = R[t][16 * b + c4 + x];
      }
      int blk = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = bi; bj < NB; ++bj, ++blk)
#pragma unroll
          for (int x = 0; x < 4; ++x) acc[blk][x] = fmaf(ar[bi], ac[bj][x], acc[blk][x]);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        cacc[b] = fmaf(ar[b], w, cacc[b]);
        if (USER) sacc[b] += ar[b];
      }
      if (USER) wsum += w;
    }
    __builtin_amdgcn_wave_barrier();
  }
  // epilogue: tri16 tiles (NB = 1: one full tile; NB = 2: tile 0 = block
  // (0,1), tile 1 = D0 upper with D1's strict lower, side array = D1's diagonal)
  const bool to_slab = wslab >= 0;
  const int64_t di = to_slab ? (int64_t)wslab : (int64_t)went;
  const GramDst& D = to_slab ? slab : direct;
  float4* Gt = reinterpret_cast<float4*>(D.G + di * D.sG);
  if constexpr (NB == 1) {
    Gt[lane] = make_float4(acc[0][0], acc[0][1], acc[0][2], acc[0][3]);
  } else {
    Gt[lane] = make_float4(acc[1][0], acc[1][1], acc[1][2], acc[1][3]);   // block (0,1)
    float f[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) f[x] = (c4 + x >= rr) ? acc[0][x] : acc[2][x];
    Gt[64 + lane] = make_float4(f[0], f[1], f[2], f[3]);
    if ((rr >> 2) == (lane & 3)) {   // this lane holds D1[rr][rr]
      const int x = rr - c4;
      const float dv = x == 0 ? acc[2][0] : x == 1 ? acc[2][1] : x == 2 ? acc[2][2] : acc[2][3];
      D.G[di * D.sG + 512 + rr] = dv;
    }
  }
  if ((lane & 3) == 0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int nn = NB * rr + b;   // natural column of virtual (b, rr)
      D.C[di * D.sV + nn] = nn < k ? cacc[b] : 0.f;
      if (USER) D.Gs[di * D.sV + nn] = nn < k ? sacc[b] : 0.f;
    }
  }
  if (USER && lane == 0) {
    D.Cb[di * D.sS] = wsum;
    D.Gn[di * D.sS] = (float)wlen;
  }
}

// ---------------------------------------------------------------------------
// K1 for k > 128 (NB > 8): the reference has no limit on k, but a wave's
// registers cannot hold NB(NB+1)/2 accumulator tiles past NB = 8.  This form
// trades speed for generality: block (work item, group of 16 stored tri16
// tiles); 32-rating chunks of rows are staged in LDS in virtual order and
// every thread accumulates 4 entries (a row segment of 4 columns, one float4
// of the row-major tile) of each of its group's tiles in fp32, rating order.
// The gathers repeat once per tile group (ceil(NTILE / 16) groups).  Group 0
// also forms the rhs, row sums, rating sum and count.
// ---------------------------------------------------------------------------
constexpr int LK_ROWS = 32;     // ratings per staged chunk
constexpr int LK_TILES = 16;    // stored tiles per block: 4 tiles x 64 threads, 4 passes

template <bool USER>
__global__ __launch_bounds__(256) void gram_largek_kernel(
    const WorkItem* __restrict__ work, const int32_t* __restrict__ idx,
    const float* __restrict__ val, const float* __restrict__ F, const float* __restrict__ bias,
    int k, int zrow, GramDst direct, GramDst slab) {
  extern __shared__ float lk_sm[];
  const int NB = nb16_of(k), ldk = 16 * NB;
  const int NO = n_off_of(NB), NF = n_fold_of(NB), NTILE = n_tiles_of(NB);
  float* rows = lk_sm;                           // [LK_ROWS][ldk + 1], virtual order
  float* wts = lk_sm + LK_ROWS * (ldk + 1);      // [LK_ROWS]
  const int ld = ldk + 1;
  const int64_t wi = blockIdx.x;
  const int64_t wbeg = work[wi].begin;
  const int wlen = work[wi].len, went = work[wi].entity, wslab = work[wi].slab;
  const int tid = threadIdx.x, lane = tid & 63, sub = tid >> 6;
  const int rr = lane >> 2, c4 = 4 * (lane & 3);
  const int group = blockIdx.y;
  // this thread's tiles: group * 16 + 4 j + sub; kind 0 = off-diagonal (bi, bj),
  // 1 = fold m (D_2m upper incl. diagonal, D_2m+1 strict lower), 2 = odd last
  int kind[4], ra[4], rb[4], ca[4], cb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = group * LK_TILES + 4 * j + sub;
    kind[j] = -1; ra[j] = rb[j] = ca[j] = cb[j] = 0;
    if (t < NO) {
      int bi = 0, rem = t;
      while (rem >= NB - 1 - bi) { rem -= NB - 1 - bi; ++bi; }
      const int bj = bi + 1 + rem;
      kind[j] = 0; ra[j] = 16 * bi + rr; ca[j] = 16 * bj + c4;
    } else if (t < NO + NF) {
      const int m = t - NO;
      kind[j] = 1; ra[j] = 32 * m + rr; ca[j] = 32 * m + c4;
      rb[j] = 32 * m + 16 + rr; cb[j] = 32 * m + 16 + c4;
    } else if (t < NTILE) {
      kind[j] = 2; ra[j] = 16 * (NB - 1) + rr; ca[j] = 16 * (NB - 1) + c4;
    }
  }
  // fp64 accumulation, one rounding to fp32 at the store (this path has the
  // registers for it; the dense k = 144 golden is ill-conditioned enough that
  // 170-term fp32 sums land at ~8e-5 of the reference)
  double acc[4][4], sd[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sd[j] = 0.0;
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[j][x] = 0.0;
  }
  // group 0: rhs / row sums of virtual columns tid and tid + 256 (ldk <= 512)
  double cv[2] = {0.0, 0.0}, sv[2] = {0.0, 0.0}, wsum = 0.0;
  for (int base = 0; base < wlen; base += LK_ROWS) {
    const int n = min(LK_ROWS, wlen - base);
    __syncthreads();
    // stage: row t, float4 h; natural column nn -> virtual 16 (nn % NB) + nn / NB
    const int q4 = ldk / 4;
    for (int e = tid; e < LK_ROWS * q4; e += 256) {
      const int t = e / q4, h = e - t * q4;
      const int id = t < n ? idx[wbeg + base + t] : zrow;
      const float4 a = reinterpret_cast<const float4*>(F + (int64_t)id * ldk)[h];
      const float v4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int nn = 4 * h + x;
        rows[t * ld + 16 * (nn % NB) + nn / NB] = v4[x];
      }
    }
    if (tid < LK_ROWS) {
      const bool ok = tid < n;
      const int id = ok ? idx[wbeg + base + tid] : zrow;
      float w = ok ? val[wbeg + base + tid] : 0.f;
      if (!USER) w -= bias[id];
      wts[tid] = w;
    }
    __syncthreads();
    for (int t = 0; t < n; ++t) {
      const float* a = rows + t * ld;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kind[j] < 0) continue;
        const double av = a[ra[j]];
        if (kind[j] == 1) {
          const double bv = a[rb[j]];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const bool up = c4 + x >= rr;          // D_2m's stored upper triangle
            acc[j][x] = fma(up ? av : bv, (double)(up ? a[ca[j] + x] : a[cb[j] + x]), acc[j][x]);
          }
          sd[j] = fma(bv, bv, sd[j]);              // D_2m+1's diagonal (side array)
        } else {
#pragma unroll
          for (int x = 0; x < 4; ++x) acc[j][x] = fma(av, (double)a[ca[j] + x], acc[j][x]);
        }
      }
      if (group == 0) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int vc = tid + 256 * hh;
          if (vc < ldk) {
            const double av = a[vc];
            cv[hh] = fma(av, (double)wts[t], cv[hh]);
            if (USER) sv[hh] += av;
          }
        }
      }
      if (USER) wsum += wts[t];
    }
  }
  const bool to_slab = wslab >= 0;
  const int64_t di = to_slab ? (int64_t)wslab : (int64_t)went;
  const GramDst& D = to_slab ? slab : direct;
  float* Ge = D.G + di * D.sG;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (kind[j] < 0) continue;
    const int t = group * LK_TILES + 4 * j + sub;
    reinterpret_cast<float4*>(Ge + (int64_t)t * 256)[lane] =
        make_float4((float)acc[j][0], (float)acc[j][1], (float)acc[j][2], (float)acc[j][3]);
    if (kind[j] == 1 && (rr >> 2) == (lane & 3))   // the thread at (rr, rr)
      Ge[(int64_t)NTILE * 256 + (t - NO) * 16 + rr] = (float)sd[j];
  }
  if (group == 0) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int vc = tid + 256 * hh;
      if (vc < ldk) {
        const int nn = NB * (vc & 15) + (vc >> 4);   // natural column of virtual vc
        D.C[di * D.sV + nn] = nn < k ? (float)cv[hh] : 0.f;
        if (USER) D.Gs[di * D.sV + nn] = nn < k ? (float)sv[hh] : 0.f;
      }
    }
    if (USER && tid == 0) {
      D.Cb[di * D.sS] = (float)wsum;
      D.Gn[di * D.sS] = (float)wlen;
    }
  }
}

int launch_gram(hipStream_t s, bool user_side, int k, const WorkItem* work,
                int64_t n_work, const int32_t* idx, const float* val,
                const float* F, const float* bias, int zrow, GramDst direct,
                GramDst slab, const CgStart* start, bool rhs_mfma) {
  if (k > kMaxK) {
    MR_CHECK(start == nullptr, "k > 128: no fused CG start");
    MR_CHECK(k <= kMaxKLarge, "k > 512 not supported");
    if (n_work <= 0) return 0;
    const int nb = nb16_of(k), ldk = 16 * nb;
    const size_t lds = (size_t)(LK_ROWS * (ldk + 1) + LK_ROWS) * sizeof(float);
    const dim3 grid((unsigned)n_work, (unsigned)((n_tiles_of(nb) + LK_TILES - 1) / LK_TILES));
    if (user_side) {
      MR_HIP(hipFuncSetAttribute((const void*)gram_largek_kernel<true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      MR_LAUNCH(gram_largek_kernel<true>, grid, dim3(256), lds, s, work, idx, val, F, bias, k,
                zrow, direct, slab);
    } else {
      MR_HIP(hipFuncSetAttribute((const void*)gram_largek_kernel<false>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      MR_LAUNCH(gram_largek_kernel<false>, grid, dim3(256), lds, s, work, idx, val, F, bias, k,
                zrow, direct, slab);
    }
    MR_HIP(hipGetLastError());
    return 0;
  }
  if (k < kMfmaMinK) {
    MR_CHECK(start == nullptr, "k < 32: the VALU Gram has no fused CG start");
    if (n_work <= 0) return 0;
    const dim3 grid((unsigned)((n_work + 3) / 4));
#define MR_VG(NB, U) \
  MR_LAUNCH((gram_valu_kernel<NB, U>), grid, dim3(256), 0, s, work, n_work, idx, val, F, bias, k, zrow, direct, slab)
    if (k <= 16) {
      if (user_side) MR_VG(1, true); else MR_VG(1, false);
    } else {
      if (user_side) MR_VG(2, true); else MR_VG(2, false);
    }
#undef MR_VG
    MR_HIP(hipGetLastError());
    return 0;
  }
#define MR_GRAM_CASE(NB) \
  case NB: return launch_gram_nb<NB>(s, user_side, k, work, n_work, idx, val, F, bias, zrow, direct, slab, start, rhs_mfma);
  switch (nb16_of(k)) {
    MR_GRAM_CASE(1) MR_GRAM_CASE(2) MR_GRAM_CASE(3) MR_GRAM_CASE(4)
    MR_GRAM_CASE(5) MR_GRAM_CASE(6) MR_GRAM_CASE(7) MR_GRAM_CASE(8)
    default: set_error("k > 128 not supported by the Gram kernel"); return -1;
  }
#undef MR_GRAM_CASE
}

int launch_cg_start_split(hipStream_t s, bool user_side, int k, const SplitItem* split,
                          int64_t n_split, GramDst direct, const CgStart& cs, double* parts,
                          const StartFold& fold) {
  if (n_split <= 0) return 0;
  const unsigned grid = (unsigned)((n_split + 3) / 4);
  const int ldk = ldk_of(k);
#define MR_SS_CASE(NB)                                                                      \
  case NB:                                                                                  \
    if (user_side)                                                                          \
      MR_LAUNCH((cg_start_split_kernel<NB, true>), dim3(grid), dim3(256), 0, s, split, n_split, \
                k, ldk, direct, cs, parts, fold);                                           \
    else                                                                                    \
      MR_LAUNCH((cg_start_split_kernel<NB, false>), dim3(grid), dim3(256), 0, s, split,     \
                n_split, k, ldk, direct, cs, parts, fold);                                  \
    break;
  switch (nb16_of(k)) {
    MR_SS_CASE(1) MR_SS_CASE(2) MR_SS_CASE(3) MR_SS_CASE(4)
    MR_SS_CASE(5) MR_SS_CASE(6) MR_SS_CASE(7) MR_SS_CASE(8)
    default: set_error("k > 128 not supported"); return -1;
  }
#undef MR_SS_CASE
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// Combine partial records of split entities, in slab order (deterministic).
// Record layout: [gsize G (tri16)][ldk Gs][ldk C][Cb][Gn] (+pad).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void store_rec(const GramDst& d, int64_t e, int64_t t, float v,
                                          int64_t nG, int ldk, bool user) {
  if (t < nG) d.G[e * d.sG + t] = v;
  else if (t < nG + ldk) { if (user) d.Gs[e * d.sV + (t - nG)] = v; }
  else if (t < nG + 2 * ldk) d.C[e * d.sV + (t - nG - ldk)] = v;
  else if (t == nG + 2 * ldk) { if (user) d.Cb[e * d.sS] = v; }
  else if (t == nG + 2 * ldk + 1) { if (user) d.Gn[e * d.sS] = v; }
}

// grid = (split entities, record float4 chunks); each thread sums one float4
// of the record over the entity's slabs with 4 independent accumulators that
// are combined in a fixed order (reproducible).
template <bool USER>
__global__ __launch_bounds__(256) void slab_reduce_kernel(
    const SplitItem* __restrict__ split, const float* __restrict__ slab,
    int64_t rec, int k, int ldk, GramDst direct) {
  const SplitItem sp = split[blockIdx.x];
  const int64_t nG = gsize_of(k);
  const int64_t used = nG + 2 * ldk + 2;
  const int64_t t4 = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
  if (t4 * 4 >= used) return;
  const float4* base = reinterpret_cast<const float4*>(slab + (int64_t)sp.slab0 * rec) + t4;
  const int64_t rs4 = rec / 4;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  int q = 0;
  for (; q + 4 <= sp.nslab; q += 4) {
    const float4 v0 = base[(q + 0) * rs4], v1 = base[(q + 1) * rs4];
    const float4 v2 = base[(q + 2) * rs4], v3 = base[(q + 3) * rs4];
    a0.x += v0.x; a0.y += v0.y; a0.z += v0.z; a0.w += v0.w;
    a1.x += v1.x; a1.y += v1.y; a1.z += v1.z; a1.w += v1.w;
    a2.x += v2.x; a2.y += v2.y; a2.z += v2.z; a2.w += v2.w;
    a3.x += v3.x; a3.y += v3.y; a3.z += v3.z; a3.w += v3.w;
  }
  for (; q < sp.nslab; ++q) {
    const float4 v0 = base[q * rs4];
    a0.x += v0.x; a0.y += v0.y; a0.z += v0.z; a0.w += v0.w;
  }
  const float r[4] = {(a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                      (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w)};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int64_t t = t4 * 4 + c;
    if (t < used) store_rec(direct, sp.entity, t, r[c], nG, ldk, USER);
  }
}

int launch_slab_reduce(hipStream_t s, bool user_side, int k,
                       const SplitItem* split, int64_t n_split,
                       const float* slab, int64_t rec, GramDst direct) {
  if (n_split <= 0) return 0;
  const int ldk = ldk_of(k);
  const int64_t used4 = (gsize_of(k) + 2 * ldk + 2 + 3) / 4;
  const dim3 grid((unsigned)n_split, (unsigned)((used4 + 255) / 256));
  if (user_side)
    MR_LAUNCH(slab_reduce_kernel<true>, grid, dim3(256), 0, s, split, slab, rec, k, ldk, direct);
  else
    MR_LAUNCH(slab_reduce_kernel<false>, grid, dim3(256), 0, s, split, slab, rec, k, ldk, direct);
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// K2: batched block GEMV y_e = G_e v_e on tri16 storage (+ bias row/col on
// the user side), with the CG direction update v = -r + beta v fused in front
// (matrix.cpp:521 of the previous iteration) and the v.y partial dot behind
// (:497).  One wave per entity, grid-stride with a fixed grid so partial sums
// are reproducible.  Each stored 16x16 block T(bi,bj) is ONE float4 load per
// lane (1 KiB per wave-instruction): lane l holds T[l>>2][4(l&3) .. +3] and
// accumulates the row product T v_bj into y_bi and, for bi < bj, the column
// product T^T v_bi into y_bj; the 4-lane row partials and 16-lane column
// partials are combined once per entity through LDS in a fixed order.
// ---------------------------------------------------------------------------
// CG state access.  The state passes between kernels like every other buffer
// (kernel boundaries order it), so plain loads / stores suffice.  Agent-scope
// atomics here cost ~60 us per GEMV launch (the finalizing block's ~30
// dependent round trips) and were not needed: the replay divergence they were
// meant to fix came from the factor snapshot transfers.
template <class T>
__device__ __forceinline__ T ald(const T* p) {
  return *p;
}
template <class T>
__device__ __forceinline__ void ast(T* p, T v) {
  *p = v;
}

struct CgScalars {   // the fields the rules read and write
  double rr, alpha, beta, final_rr, min_dec, comm0, comm1;
  int32_t it, fails, done, ret, max_it, n_matvec, sharded;
};
__device__ __forceinline__ CgScalars load_state(const CgState* st) {
  CgScalars v;
  v.rr = ald(&st->rr);
  v.alpha = ald(&st->alpha);
  v.beta = ald(&st->beta);
  v.final_rr = ald(&st->final_rr);
  v.min_dec = ald(&st->min_dec);
  v.comm0 = ald(&st->comm[0]);
  v.comm1 = ald(&st->comm[1]);
  v.it = ald(&st->it);
  v.fails = ald(&st->fails);
  v.done = ald(&st->done);
  v.ret = ald(&st->ret);
  v.max_it = ald(&st->max_it);
  v.n_matvec = ald(&st->n_matvec);
  v.sharded = ald(&st->sharded);
  return v;
}
__device__ __forceinline__ void store_state(CgState* st, const CgScalars& v) {
  ast(&st->rr, v.rr);
  ast(&st->alpha, v.alpha);
  ast(&st->beta, v.beta);
  ast(&st->final_rr, v.final_rr);
  ast(&st->min_dec, v.min_dec);
  ast(&st->comm[0], v.comm0);
  ast(&st->comm[1], v.comm1);
  ast(&st->it, v.it);
  ast(&st->fails, v.fails);
  ast(&st->done, v.done);
  ast(&st->ret, v.ret);
  ast(&st->max_it, v.max_it);
  ast(&st->n_matvec, v.n_matvec);
  ast(&st->sharded, v.sharded);
}

// Seqlock publish into slot seq % kMirrorSlots of the host-mapped mirror ring
// (Engine::wait_mirror): odd 2 seq - 1 marks a write in progress, the even
// 2 seq (release) its end.
__device__ __forceinline__ void publish(const CgScalars& v, CgMirror* ring, int seq) {
  if (!ring) return;
  CgMirror* m = ring + (seq & (kMirrorSlots - 1));
  __hip_atomic_store(&m->seq, 2 * seq - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  m->done = v.done;
  m->fails = v.fails;
  m->it = v.it;
  m->ret = v.ret;
  m->n_matvec = v.n_matvec;
  m->rr = v.rr;
  m->final_rr = v.final_rr;
  __threadfence_system();
  __hip_atomic_store(&m->seq, 2 * seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// BETA rule (matrix.cpp:507-525) on rr2 = r.r after the update: beta, the
// two-strikes stagnation test, it++ and the loop-top stop tests.
__device__ __forceinline__ void apply_beta(CgScalars& v, double rr2) {
  v.final_rr = rr2;
  const double beta = rr2 / v.rr;
  v.beta = beta;
  if (!MR_SP_PROBE && beta > 1.0 - v.min_dec) v.fails += 1;
  else v.fails = 0;
  if (v.fails >= 2) {
    v.done = 1;
    v.ret = v.it;
  } else {
    v.rr = rr2;
    v.it += 1;
    if (v.it >= v.max_it || (rr2 < 1e-6 && !MR_SP_PROBE)) {
      v.done = 1;
      v.ret = v.it;
    }
  }
}

// Peer all-reduce of `count` (< kPeerRec) doubles by ONE thread (the finalizing
// thread of a kernel whose blocks have all finished): write this rank's
// values into its record of every rank's exchange buffer, tag it with the
// reduction's sequence number (release, system scope), wait for the tags of
// all ranks' records in the own buffer (acquire), sum in rank order.  Every
// rank issues the same reductions in the same order (the exact-state launch
// protocol), so sequence numbers agree; a slot is reused only after every
// rank has passed kPeerSlots - 1 later reductions, each of which needed this
// rank's data, so no record is overwritten before it is read.  A peer that
// does not arrive within pc->timeout_ticks (MR_OPT_PEER_TIMEOUT_S, default
// 30 s) sets `error` and the caller ends the solve with ret = -1 (the host
// reports it) instead of spinning forever.
// Returns false on timeout.
__device__ __forceinline__ void peer_account(PeerComm* pc, uint64_t t0) {
  __hip_atomic_fetch_add(&pc->wait_ticks, (uint64_t)__builtin_amdgcn_s_memrealtime() - t0,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(&pc->n_reduce, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ bool peer_sum(PeerComm* pc, double* vals, int count) {
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  const uint32_t s = __hip_atomic_load(&pc->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __hip_atomic_store(&pc->seq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int world = pc->world, rank = pc->rank;
  const int64_t slot = s % kPeerSlots;
  for (int q = 0; q < world; ++q) {
    double* rec = pc->buf[q] + (slot * world + rank) * kPeerRec;
    for (int c = 0; c < count; ++c)
      __hip_atomic_store(rec + c, vals[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(rec + kPeerRec - 1), (uint64_t)s, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  double acc[kPeerRec - 1] = {};
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
  for (int q = 0; q < world; ++q) {
    const double* rec = pc->buf[rank] + (slot * world + q) * kPeerRec;
    while (__hip_atomic_load(reinterpret_cast<const uint64_t*>(rec + kPeerRec - 1), __ATOMIC_ACQUIRE,
                             __HIP_MEMORY_SCOPE_SYSTEM) != (uint64_t)s) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > pc->timeout_ticks) {
        pc->error = 1;
        return false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    for (int c = 0; c < count; ++c)
      acc[c] += __hip_atomic_load(rec + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (int c = 0; c < count; ++c) vals[c] = acc[c];
  peer_account(pc, t_in);
  return true;
}

// The same exchange for the integer containers of the order-independent
// sums, by a whole wave: lane l < count owns value l (it stores it into its
// slot of every rank's record and sums the ranks' values for l); lane 0
// advances the sequence number, tags after a system-scope release fence for
// the wave's stores, and waits for the peers' tags (acquire).  Integer sums:
// exact, so all ranks get the same containers.  Returns false on timeout
// (every lane).
__device__ bool peer_sum_lanes(PeerComm* pc, int64_t& val, int count) {
  const int lane = threadIdx.x & 63;
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
  if (lane == 0) {
    // sc1: the next reduction may run on another CU (the resident CG's last
    // block changes every iteration)
    s = __hip_atomic_load(&pc->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(&pc->seq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  s = __builtin_amdgcn_readfirstlane(s);
  const int world = pc->world, rank = pc->rank;
  const int64_t slot = s % kPeerSlots;
  for (int q = 0; q < world; ++q) {
    int64_t* rec = reinterpret_cast<int64_t*>(pc->buf[q]) + (slot * world + rank) * kPeerRec;
    if (lane < count) __hip_atomic_store(rec + lane, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
  if (lane == 0) {
    for (int q = 0; q < world; ++q) {
      int64_t* rec = reinterpret_cast<int64_t*>(pc->buf[q]) + (slot * world + rank) * kPeerRec;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(rec + kPeerRec - 1), (uint64_t)s,
                         __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  int ok = 1;
  if (lane == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    for (int q = 0; q < world && ok; ++q) {
      const int64_t* rec = reinterpret_cast<const int64_t*>(pc->buf[rank]) + (slot * world + q) * kPeerRec;
      while (__hip_atomic_load(reinterpret_cast<const uint64_t*>(rec + kPeerRec - 1),
                               __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != (uint64_t)s) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > pc->timeout_ticks) {
          pc->error = 1;
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  ok = __builtin_amdgcn_readfirstlane(ok);
  if (!ok) return false;
  __threadfence_system();
  int64_t acc = 0;
  for (int q = 0; q < world; ++q) {
    const int64_t* rec = reinterpret_cast<const int64_t*>(pc->buf[rank]) + (slot * world + q) * kPeerRec;
    if (lane < count) acc += __hip_atomic_load(rec + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (lane < count) val = acc;
  if (lane == 0) peer_account(pc, t_in);
  return true;
}

// Self-test of a freshly mapped peer exchange: one reduction of
// {rank + 1, 1}; out = {sum, count, ok}.  Run by every rank at attach time.
__global__ void peer_selftest_kernel(PeerComm* pc, double* out) {
  if (threadIdx.x != 0) return;
  double v[2] = {(double)(pc->rank + 1), 1.0};
  const bool ok = peer_sum(pc, v, 2);
  out[0] = v[0];
  out[1] = v[1];
  out[2] = ok ? 1.0 : 0.0;
}

// Test hook (mr_test_xsum): the order-independent sum of n terms dealt to
// the waves of `gridDim.x` blocks (wave-strided), flushed into `bins`, then
// collected and converted by one wave of a second launch.
__global__ __launch_bounds__(256) void xsum_test_kernel(const double* __restrict__ t, int64_t n,
                                                        int64_t* __restrict__ bins) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), W = (int64_t)gridDim.x * 4;
  int64_t acc[1] = {0};
  for (int64_t i = w; i < n; i += W) acc[0] += xterm(t[i], lane);
  xsum_flush<1>(acc, bins);
}
__global__ void xsum_collect_kernel(int64_t* __restrict__ bins, double* __restrict__ out) {
  __shared__ int64_t xs[kXW];
  const int lane = threadIdx.x;
  const int64_t c = xsum_collect<1>(bins, lane);
  if (lane < kXW) xs[lane] = c;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) out[0] = xsum_value(xs);
}
int launch_xsum_test(hipStream_t s, const double* t, int64_t n, int blocks, int64_t* bins,
                     double* out) {
  xsum_test_kernel<<<blocks, 256, 0, s>>>(t, n, bins);
  MR_HIP(hipGetLastError());
  xsum_collect_kernel<<<1, 64, 0, s>>>(bins, out);
  MR_HIP(hipGetLastError());
  return 0;
}

// Latency probe: `iters` back-to-back reductions of one value by one thread
// (the finalizing thread's part of a CG iteration); out = {ok, iters done}.
__global__ void peer_bench_kernel(PeerComm* pc, int iters, double* out) {
  if (threadIdx.x != 0) return;
  const double want = 0.5 * pc->world * (pc->world + 1);
  int ok = 1, n = 0;
  for (; n < iters; ++n) {
    double v = (double)(pc->rank + 1);
    if (!peer_sum(pc, &v, 1)) { ok = 0; break; }
    if (v != want) ok = 0;
  }
  out[0] = ok;
  out[1] = n;
}

int launch_peer_bench(hipStream_t s, PeerComm* pc, int iters, double* out) {
  peer_bench_kernel<<<1, 64, 0, s>>>(pc, iters, out);
  MR_HIP(hipGetLastError());
  return 0;
}

int launch_peer_selftest(hipStream_t s, PeerComm* pc, double* out) {
  peer_selftest_kernel<<<1, 64, 0, s>>>(pc, out);
  MR_HIP(hipGetLastError());
  return 0;
}

// A failed peer exchange ends the solve (every later kernel is a no-op) with
// ret = -1, published so the host's wait returns.
__device__ void peer_fail(CgState* st, CgMirror* mirror, int seq);

// INIT / ALPHA / BETA rules on the reduced sum s (one thread).
__device__ void cg_finalize(CgState* st, int phase, double s, CgMirror* mirror, int seq) {
  if (PeerComm* pc = ald(&st->peer)) {
    if (!peer_sum(pc, &s, 1)) {
      peer_fail(st, mirror, seq);
      return;
    }
  }
  CgScalars v = load_state(st);
  if (phase == CG_INIT) {
    v.rr = s;
    v.final_rr = s;
    v.it = 0;
    v.fails = 0;
    v.done = 0;
    v.ret = 0;
    if (v.max_it <= 0 || (s < 1e-6 && !MR_SP_PROBE)) v.done = 1;
    store_state(st, v);
    publish(v, mirror, seq);
  } else if (phase == CG_ALPHA) {
    v.alpha = v.rr / s;
    v.n_matvec += 1;
    store_state(st, v);
  } else {
    apply_beta(v, s);
    store_state(st, v);
    publish(v, mirror, seq);
  }
}

__device__ void peer_fail(CgState* st, CgMirror* mirror, int seq) {
  CgScalars v = load_state(st);
  v.done = 1;
  v.ret = -1;
  store_state(st, v);
  publish(v, mirror, seq);
}

// Sharded runs: the BETA step of iteration t (its r.r all-reduced into
// comm[0]) is applied by the matvec of iteration t+1 instead of a one-block
// finalize launch.  Every block derives beta and the stop decision from the
// same state and comm[0] (a pure function, so all blocks agree: if it ends
// the solve they skip the products); the last-arriving block -- every other
// block has finished reading the state by then -- stores the new state,
// publishes it under beta_seq and leaves its own p.Ap partial sum in comm[0]
// for the next all-reduce.
__device__ __forceinline__ bool matvec_entry(const CgState* st, int beta_seq, double& beta,
                                             bool& skip) {
  skip = false;
  if (beta_seq > 0) {
    CgScalars v = load_state(st);
    if (v.done) return false;   // ended earlier (and published then)
    apply_beta(v, v.comm0);
    beta = v.beta;
    skip = v.done != 0;
    return true;
  }
  if (ald(&st->done)) return false;
  beta = ald(&st->beta);
  return true;
}

// Fused control: every block stores its partial sum write-through (sc1) and
// drains it, then one lane adds to an agent-scope counter; the block whose add
// returns gridDim.x-1 reduces all partials (sc1 loads, index order -- the
// control kernel's order, so results are identical) and applies the rules.
// No L2 writeback fence: __threadfence() here (buffer_wbl2 per block) cost
// ~90 us per matvec launch.
__device__ __forceinline__ void store_partial(double* partials, double tot) {
  if (threadIdx.x == 0)
    __hip_atomic_store(&partials[blockIdx.x], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last block of a sharded matvec that folds the previous BETA step: apply
// it (the same decision every block took), publish, then leave the local
// p.Ap sum in comm[0].
__device__ void last_block_beta(CgState* st, double* partials, CgMirror* mirror, int seq,
                                double* sh) {
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(&st->arrive, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  double acc = 0.0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x)
    acc += __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const double tot = block_sum_f64<256>(acc, sh);
  if (threadIdx.x == 0) {
    __hip_atomic_store(&st->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CgScalars v = load_state(st);
    apply_beta(v, v.comm0);
    v.comm0 = tot;
    store_state(st, v);
    publish(v, mirror, seq);
  }
}

__device__ void last_block_finalize(CgState* st, int phase, double* partials, CgMirror* mirror,
                                    int seq, double* sh) {
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(&st->arrive, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  double acc = 0.0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x)
    acc += __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const double tot = block_sum_f64<256>(acc, sh);
  if (threadIdx.x == 0) {
    __hip_atomic_store(&st->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ald(&st->sharded)) {
      // local sum for the all-reduce; the update computes alpha itself from
      // the reduced slot, so ALPHA needs no finalize step (only its count)
      ast(&st->comm[0], tot);
      if (phase == CG_BETA) ast(&st->n_matvec, ald(&st->n_matvec) + 1);
    } else {
      cg_finalize(st, phase, tot, mirror, seq);
    }
  }
}


// G streams once per CG iteration and exceeds the Infinity Cache at scale,
// so it is loaded non-temporally (measured on MI355X, k = 64, ML-full shape:
// users 225 -> 195 us, items 103 -> 94 us, and the CG update 28 -> 25 us
// because its vectors stay cached).
template <int NB, bool USER>
__global__ __launch_bounds__(256, (NB <= 4 ? 4 : 2)) void cg_matvec_kernel(
    const CgState* __restrict__ st, int update_p, int64_t E, int k, int ldk,
    const float* __restrict__ G, const float* __restrict__ Gs,
    const float* __restrict__ Gn, double* __restrict__ v, double* __restrict__ vb,
    const double* __restrict__ r, const double* __restrict__ rb,
    double* __restrict__ y, double* __restrict__ yb, double* __restrict__ partials,
    CgState* fst, int phase, CgMirror* mirror, int beta_seq) {
  double beta = 0.0;
  bool skip;
  if (!matvec_entry(st, beta_seq, beta, skip)) return;
  constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF + (NB & 1);
  constexpr int64_t GS = (int64_t)NTILE * 256 + NF * 16;   // == gsize_of(k)
  constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  constexpr bool STREAM = MR_TS_STREAM && NB > 4;
  __shared__ MvScratch<NB> scr[MV_WAVES];
  __shared__ double sh[MV_WAVES];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  MvScratch<NB>& sc = scr[wid];
  double dsum = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * MV_WAVES + wid; e < (skip ? 0 : E);
       e += (int64_t)gridDim.x * MV_WAVES) {
    // issue order matters for the in-order vmcnt: vector loads first, then
    // every G block of this entity, so staging p waits only for the former
    double* ve = v + e * ldk;
    double vi[NV], ri[NV];
#pragma unroll
    for (int h = 0; h < NV; ++h) {
      const int i = lane + 64 * h;
      vi[h] = (i < NP) ? ve[i] : 0.0;                       // NP == ldk
      ri[h] = (update_p && i < NP) ? r[e * ldk + i] : 0.0;
    }
    double vbias = 0.0, rbias = 0.0;
    if (USER) {
      vbias = vb[e];
      if (update_p) rbias = rb[e];
    }
    const floatx4* __restrict__ Ge = reinterpret_cast<const floatx4*>(G + e * GS);
    float4 g[STREAM ? ts_ahead<NB>() : NTILE];
    if constexpr (STREAM) {
      tile_stream_load<NB, true>(Ge, lane, g);
    } else {
#pragma unroll
      for (int t = 0; t < NTILE; ++t) g[t] = tile_ld<true>(Ge, t, lane);
    }
    float d2 = 0.f;   // diagonal of the odd diagonal blocks (side array)
    if (NF > 0 && lane < 16 * NF) d2 = G[e * GS + NTILE * 256 + lane];
    // p = -r + beta p (matrix.cpp:521) for the entity, then stage it
#pragma unroll
    for (int h = 0; h < NV; ++h) {
      const int i = lane + 64 * h;
      if (i < NP) {
        double x = vi[h];
        if (update_p) {
          x = fma(beta, x, -ri[h]);
          ve[i] = x;
        }
        sc.pv[virt_of(i, NB)] = x;
      }
    }
    if (USER && update_p) {
      vbias = fma(beta, vbias, -rbias);
      if (lane == 0) vb[e] = vbias;
    }
    if (NF > 0 && lane < 16 * NF) sc.dd[lane] = d2;
    __builtin_amdgcn_wave_barrier();
    double yo[NV], ybv = 0.0;
    if constexpr (STREAM)
      tile_matvec_stream<NB, USER, true>(Ge, g, sc, vbias, USER ? Gs + e * ldk : nullptr,
                                         USER ? Gn[e] : 0.f, k, yo, ybv);
    else
      tile_matvec<NB, USER>(g, sc, vbias, USER ? Gs + e * ldk : nullptr, USER ? Gn[e] : 0.f, k,
                            yo, ybv);
    double d = 0.0;
#pragma unroll
    for (int h = 0; h < NV; ++h) {
      const int o = lane + 64 * h;
      if (o < NP) {
        const int n = nat_of(o, NB);
        if (n < k) {
          y[e * ldk + n] = yo[h];
          d = fma(yo[h], sc.pv[o], d);
        }
      }
    }
    if (USER && lane == 0) {
      yb[e] = ybv;
      d = fma(ybv, vbias, d);
    }
    dsum += wave_sum_f64(d);
    __builtin_amdgcn_wave_barrier();
  }
  const double tot = block_sum_f64<256>(lane == 0 ? dsum : 0.0, sh);
  if (fst) store_partial(partials, tot);
  else if (threadIdx.x == 0) partials[blockIdx.x] = tot;
  if (fst && phase == CG_ALPHA) {
    if (beta_seq > 0) last_block_beta(fst, partials, mirror, beta_seq, sh);
    else last_block_finalize(fst, CG_ALPHA, partials, nullptr, 0, sh);
  }
}

// One-pass CG iteration (DESIGN.md "One-pass CG iteration"): ONE kernel per
// CG iteration t >= 1 instead of matvec + update.  Each wave first applies,
// for its entity, iteration t-1's deferred update (x += alpha p, r += alpha q:
// matrix.cpp:501-503, the same fp64 expressions as cg_update_kernel), then
// p = -r + beta p (:521), q = G p, and adds p.q, r.q, q.q and the updated
// residual's own r.r to its partials.  The last-arriving block sums them in a
// fixed order and takes iteration t's scalars: alpha = r.r / p.q (:497) with
// the direct r.r and, without a second pass over the vectors, r'.r' = r.r +
// 2 alpha r.q + alpha^2 q.q for the new residual r' = r + alpha q -- the same
// quantity as the reference's direct r'.r' (:507) up to rounding of order
// eps r.r / r'.r' (CG's per-iteration decrease is moderate, see the design
// note) -- then the BETA rule and the publish.  The derived value sets only
// that beta and stop test: kernel t+1 replaces it by the direct dot, so its
// rounding does not accumulate over the solve.
// Iteration t's own update is deferred to kernel t+1 or, after the stop, to
// cg_update_kernel(UPD_FINISH).  `update` = 0 for t = 0 of an unfused start
// (nothing deferred yet).  Per vector entry: read p, r, q, x; write p, r, q, x
// (56 B fp64/fp32) against 72 B for matvec + update, and one kernel boundary
// less per iteration.
// Occupancy: 4 waves / SIMD (<= 128 VGPRs) at NB <= 4.  The tiles' fp64
// copies are made afresh in each of tile_matvec's two passes (OPAQUE, as at
// NB > 4): with the merged copies the user side at NB = 4 needed 140 VGPRs
// (3 waves / SIMD, or 14 spilled registers at 4); now 110.  Same box, fixed
// 20 CG iterations, k = 64: users 215 -> 211 us per iteration.
#ifndef MR_OP_WAVES_U4
#define MR_OP_WAVES_U4 4
#endif
#ifndef MR_OP_OPAQUE
#define MR_OP_OPAQUE 1
#endif
#ifndef MR_OP_WAVES
#define MR_OP_WAVES 4
#endif
// NT: the G tiles are loaded non-temporally (a side whose per-iteration
// stream is far larger than the Infinity Cache: nothing of it survives to the
// next sweep) or with the default policy (a shard small enough to stay
// on-die between sweeps); the engine picks per side (Engine::tile_nt_for)
// Diagnostic timeline of the one-pass kernel (MR_OP_PROF builds only,
// tools/op_timeline.py): per block, s_memrealtime (100 MHz) at entry, after
// its entities, after its bin flush; the last block also after the bin
// collection, after the state update and after the publish.
#ifndef MR_OP_PROF
#define MR_OP_PROF 0
#endif
constexpr int kOpProfBlocks = 4096;
__device__ int64_t g_op_prof[8 + 4 * kOpProfBlocks];
__device__ __forceinline__ void op_prof(int slot) {
  if constexpr (MR_OP_PROF) {
    const int64_t t = (int64_t)__builtin_amdgcn_s_memrealtime();
    if (slot < 8) g_op_prof[slot] = t;
    else if (blockIdx.x < kOpProfBlocks) g_op_prof[8 + 4 * blockIdx.x + (slot - 8)] = t;
  }
}

// One entity's operands of a one-pass CG iteration, loaded into registers:
// the CG vectors' entries of this lane, the bias entries (user side) and the
// G tiles (NB > 4: the first tiles of the stream, tile_matvec_stream loads
// the rest).  Loading entity e + 1's while e is processed (a second register
// set used in alternation, 2 or 3 waves / SIMD) measured 14-32 % (an 8-rank
// shard) and 19-33 % (full size) slower per users CG iteration at k = 64
// (profiles/r04/r04l).
template <int NB>
struct OpEnt {
  static constexpr int NP = 16 * NB, NV = (NP + 63) / 64;
  static constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF + (NB & 1);
  static constexpr bool STREAM = MR_TS_STREAM && NB > 4;
  static constexpr int NHELD = STREAM ? ts_ahead<NB>() : NTILE;   // tiles held per entity
  static constexpr int64_t GS = (int64_t)NTILE * 256 + NF * 16;     // == gsize_of(k)
  double pi[NV], ri[NV], qi[NV];
  float xi[NV];
  double pbias, rbias, qbias;
  float xbias, d2;
  float4 g[NHELD];
};

// One side's normal equations and CG vectors (local rows; x = the factor
// table itself, warm start in place).
struct OpSide {
  int64_t E;
  int k, ldk;
  const float *G, *Gs, *Gn;
  double *p, *pb, *r, *rb, *q, *qb;
  float *x, *xb;
};

template <int NB, bool USER, bool NT>
__device__ __forceinline__ void op_load(const OpSide& A, int64_t e, int update, OpEnt<NB>& E_,
                                        int lane) {
  using T = OpEnt<NB>;
  const double* pe = A.p + e * A.ldk;
  const double* re = A.r + e * A.ldk;
  const double* qe = A.q + e * A.ldk;
  const float* xe = A.x + e * A.ldk;
  // q and x are loaded whether or not this iteration applies the deferred
  // update (only the first iteration of an unfused start does not; their
  // values are then unused): a load under a branch made the compiler wait
  // for it inside the branch, ahead of the G tile loads
  (void)update;
#pragma unroll
  for (int h = 0; h < T::NV; ++h) {
    const int i = lane + 64 * h;
    E_.pi[h] = (i < T::NP) ? pe[i] : 0.0;
    E_.ri[h] = (i < T::NP) ? re[i] : 0.0;
    E_.qi[h] = (i < T::NP) ? qe[i] : 0.0;
    E_.xi[h] = (i < T::NP) ? xe[i] : 0.f;
  }
  E_.pbias = E_.rbias = E_.qbias = 0.0;
  E_.xbias = 0.f;
  if (USER) {
    E_.pbias = A.pb[e];
    E_.rbias = A.rb[e];
    E_.qbias = A.qb[e];
    E_.xbias = A.xb[e];
  }
  const floatx4* __restrict__ Ge = reinterpret_cast<const floatx4*>(A.G + e * T::GS);
  if constexpr (T::STREAM) {
    tile_stream_load<NB, NT>(Ge, lane, E_.g);
  } else {
#pragma unroll
    for (int t = 0; t < T::NTILE; ++t) E_.g[t] = tile_ld<NT>(Ge, t, lane);
  }
  // the folded tiles' side diagonals (lanes < 16 NF use them); every lane
  // loads (a clamped index), so no register is zeroed and then loaded under
  // an exec mask -- that pattern made the wait-count pass drain every load
  // in flight at the next entity's start
  if constexpr (T::NF > 0) E_.d2 = A.G[e * T::GS + T::NTILE * 256 + (lane < 16 * T::NF ? lane : 0)];
  else E_.d2 = 0.f;
}

// Entity e of one CG iteration (matrix.cpp:488-526 in block form): the
// deferred x / r update of the previous iteration (update != 0), p = -r +
// beta p, q = G p (tile GEMV) written back, and this lane's terms of p.q,
// r.q, q.q and the updated r.r added into a, b, c, d in entity order.
template <int NB, bool USER, bool NT>
__device__ __forceinline__ void op_process(const OpSide& A, int64_t e, int update, double alpha,
                                           double beta, OpEnt<NB>& E_, MvScratch<NB>& sc, double* rs,
                                           double& a, double& b, double& c, double& d, int lane) {
  using T = OpEnt<NB>;
  double* pe = A.p + e * A.ldk;
  double* re = A.r + e * A.ldk;
  double* qe = A.q + e * A.ldk;
  float* xe = A.x + e * A.ldk;
  double pbias = E_.pbias, rbias = E_.rbias;
#pragma unroll
  for (int h = 0; h < T::NV; ++h) {
    const int i = lane + 64 * h;
    if (i < T::NP) {
      double rn = E_.ri[h], pn = E_.pi[h];
      if (update) {
        rn = fma(alpha, E_.qi[h], E_.ri[h]);
        re[i] = rn;
        xe[i] = (float)fma(alpha, E_.pi[h], (double)E_.xi[h]);
        pn = fma(beta, E_.pi[h], -rn);
        pe[i] = pn;
        d = fma(rn, rn, d);
      }
      sc.pv[virt_of(i, NB)] = pn;
      rs[virt_of(i, NB)] = rn;
    }
  }
  if (USER && update) {
    const double rbn = fma(alpha, E_.qbias, rbias);
    const double pbn = fma(beta, pbias, -rbn);
    if (lane == 0) {
      A.rb[e] = rbn;
      A.xb[e] = (float)fma(alpha, pbias, (double)E_.xbias);
      A.pb[e] = pbn;
    }
    rbias = rbn;
    pbias = pbn;
    if (lane == 0) d = fma(rbn, rbn, d);
  }
  if (T::NF > 0 && lane < 16 * T::NF) sc.dd[lane] = E_.d2;
  __builtin_amdgcn_wave_barrier();
  double yo[T::NV], ybv = 0.0;
  if constexpr (T::STREAM)
    tile_matvec_stream<NB, USER, NT>(reinterpret_cast<const floatx4*>(A.G + e * T::GS), E_.g, sc,
                                     pbias, USER ? A.Gs + e * A.ldk : nullptr, USER ? A.Gn[e] : 0.f,
                                     A.k, yo, ybv);
  else
    tile_matvec<NB, USER, (NB > 4) || MR_OP_OPAQUE>(E_.g, sc, pbias, USER ? A.Gs + e * A.ldk : nullptr,
                                                    USER ? A.Gn[e] : 0.f, A.k, yo, ybv);
#pragma unroll
  for (int h = 0; h < T::NV; ++h) {
    const int o = lane + 64 * h;
    if (o < T::NP) {
      const int n = nat_of(o, NB);
      if (n < A.k) {
        qe[n] = yo[h];
        a = fma(yo[h], sc.pv[o], a);
        b = fma(yo[h], rs[o], b);
        c = fma(yo[h], yo[h], c);
      }
    }
  }
  if (USER && lane == 0) {
    A.qb[e] = ybv;
    a = fma(ybv, pbias, a);
    b = fma(ybv, rbias, b);
    c = fma(ybv, ybv, c);
  }
  __builtin_amdgcn_wave_barrier();
}

// One chunk's four terms (lane-wise entity-order sums, reduced across the
// wave once) into the block's order-independent containers (LDS atomics).
__device__ __forceinline__ void op_chunk_terms(double a, double b, double c, double d,
                                               int64_t (*xacc)[4][kXW], int lane) {
  a = wave_sum_f64(a);
  b = wave_sum_f64(b);
  c = wave_sum_f64(c);
  d = wave_sum_f64(d);
  if (lane < kXW) {
    atomicAdd((unsigned long long*)&xacc[0][0][lane], (unsigned long long)xterm(a, lane));
    atomicAdd((unsigned long long*)&xacc[0][1][lane], (unsigned long long)xterm(b, lane));
    atomicAdd((unsigned long long*)&xacc[0][2][lane], (unsigned long long)xterm(c, lane));
    atomicAdd((unsigned long long*)&xacc[0][3][lane], (unsigned long long)xterm(d, lane));
  }
}

// The last block's BETA step of one iteration from the collected containers
// (lane 0's v): alpha from the direct r.r (iteration t >= 1: the residual
// just updated, so the derivation's rounding does not accumulate across
// iterations), r'.r' = r.r + 2 alpha r.q + alpha^2 q.q for beta and the stop.
__device__ __forceinline__ void op_beta(CgScalars& v, const double (&sum)[4], int update) {
  if (update) v.rr = sum[3];
  const double al = v.rr / sum[0];
  v.alpha = al;
  v.n_matvec += 1;
  apply_beta(v, fma(al * al, sum[2], fma(2.0 * al, sum[1], v.rr)));
}

template <int NB, bool USER, bool NT>
__global__ __launch_bounds__(256, (NB <= 4 ? (USER && NB == 4 ? MR_OP_WAVES_U4 : MR_OP_WAVES) : 2))
#ifdef MR_OP_WPE
__attribute__((amdgpu_waves_per_eu(MR_OP_WPE, MR_OP_WPE)))
#endif
void cg_onepass_kernel(
    CgState* __restrict__ st, int update, int rev, int64_t E, int k, int ldk,
    const float* __restrict__ G, const float* __restrict__ Gs, const float* __restrict__ Gn,
    double* __restrict__ p, double* __restrict__ pb, double* __restrict__ r,
    double* __restrict__ rb, double* __restrict__ q, double* __restrict__ qb,
    float* __restrict__ x, float* __restrict__ xb, int64_t* __restrict__ xbins,
    CgMirror* mirror, int seq) {
  if (ald(&st->done)) return;
  if (threadIdx.x == 0) op_prof(8);
  const double beta = ald(&st->beta), alpha = ald(&st->alpha);
  constexpr int XC = xchunk_of(NB, USER);
  const OpSide A{E, k, ldk, G, Gs, Gn, p, pb, r, rb, q, qb, x, xb};
  __shared__ MvScratch<NB> scr[MV_WAVES];
  __shared__ double rvs[MV_WAVES][16 * NB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  MvScratch<NB>& sc = scr[wid];
  double* rs = rvs[wid];
  // the wave's p.q, r.q, q.q, r.r as order-independent sums (lane = digit),
  // one term per chunk of XC consecutive entities: the chunk's partial sums
  // run lane-wise in entity order and are reduced across the wave once, so a
  // term depends only on its chunk, never on the grid
  // (the block's containers live in LDS, added to by LDS integer atomics:
  // no registers held across the GEMV)
  __shared__ int64_t xacc[1][4][kXW];
  if (threadIdx.x < 4 * kXW) (&xacc[0][0][0])[threadIdx.x] = 0;
  __syncthreads();
  const int wu = __builtin_amdgcn_readfirstlane(wid);   // wave-uniform: scalar loop state
  // rev: the grid sweeps the chunks from the last to the first (entity order
  // inside a chunk unchanged, so every chunk's term is the same): alternate
  // iterations then start where the previous sweep ended, on the lines it
  // left in the Infinity Cache (DESIGN.md "Sweep direction")
  const int64_t nch = (E + XC - 1) / XC;
  for (int64_t j = (int64_t)blockIdx.x * MV_WAVES + wu; j < nch;
       j += (int64_t)gridDim.x * MV_WAVES) {
    const int64_t c0 = (rev ? nch - 1 - j : j) * XC;
    const int64_t c1 = c0 + XC < E ? c0 + XC : E;
    double a = 0.0, b = 0.0, c = 0.0;
    double d = 0.0;   // r.r of the updated residual (matrix.cpp:507's direct dot)
    for (int64_t e = c0; e < c1; ++e) {
      OpEnt<NB> cur;
      op_load<NB, USER, NT>(A, e, update, cur, lane);
      op_process<NB, USER, NT>(A, e, update, alpha, beta, cur, sc, rs, a, b, c, d, lane);
    }
    op_chunk_terms(a, b, c, d, xacc, lane);
  }
  if (threadIdx.x == 0) op_prof(9);
  xsum_flush_lds<4>(xacc, xbins, 1);
  // last-arriving block: iteration t's scalars (see last_block_finalize for
  // the memory-model basis of this hand-off; the bins' atomics are drained
  // by the same vmcnt wait as a partial store)
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    op_prof(10);
    s_last = __hip_atomic_fetch_add(&st->arrive, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last || wid != 0) return;
  __shared__ int64_t xs[4 * kXW];
  __shared__ double xv[4];
  if (lane == 0) op_prof(0);
  // the state and the peer pointer are loaded before the bins, so their
  // latency overlaps the collection (the serial tail of every iteration)
  PeerComm* pc = ald(&st->peer);
  CgScalars v{};
  if (lane == 0) v = load_state(st);
  int64_t tot = xsum_collect<4>(xbins, lane);
  if (lane == 0) op_prof(1);
  if (lane == 0) __hip_atomic_store(&st->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (pc) {
    if (!peer_sum_lanes(pc, tot, 4 * kXW)) {
      if (lane == 0) peer_fail(st, mirror, seq);
      return;
    }
  }
  if (lane < 4 * kXW) xs[lane] = tot;
  __builtin_amdgcn_wave_barrier();
  if (lane < 4) xv[lane] = xsum_value(&xs[lane * kXW]);   // the four sums in parallel
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    double sum[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sum[j] = xv[j];
    op_beta(v, sum, update);
    store_state(st, v);
    ast(&st->pending, 1);
    op_prof(2);
    publish(v, mirror, seq);
    op_prof(3);
  }
}

// ---------------------------------------------------------------------------
// Resident CG solve (DESIGN.md "Resident CG solve"): the one-pass iteration
// above for EVERY iteration of a solve in ONE launch.  The grid is exactly
// the blocks the chip holds at once, so all blocks are resident; each wave
// OWNS a fixed set of entity chunks for the whole solve (the one-pass deal of
// chunk j to wave j mod (4 x grid), its order reversed on alternate
// iterations instead of the deal), so the CG vectors of an entity are only
// ever touched by one wave: no cross-CU hand-off of the vectors, no kernel
// boundary (launch ramp, dirty-L2 write-back) between iterations.  Per
// iteration, as one pass: chunks -> containers -> bins; arrival; the last
// block takes alpha, r'.r' and the BETA rule (and the peer all-reduce) and
// broadcasts {alpha, beta, done} to every block through a generation word
// (write-through sc1 stores, drained, then the word: MI355X_MICROARCH.md
// "Valid forms", first table row); the others poll it.  While they wait, each
// wave already loads its first entity of the next iteration (G tiles and its
// own vectors).  After the stop the pending x update (the UPD_FINISH pass)
// is applied by every wave to its own entities.  The arithmetic is the
// one-pass kernel's, term for term: every chunk's terms and every vector
// entry are bitwise those of the launch-per-iteration path.
// The state a block reads after the broadcast was written by another
// block (another XCD): in this kernel the state goes through sc1 loads and
// stores only.
// ---------------------------------------------------------------------------
__device__ __forceinline__ CgScalars load_state_sc1(CgState* st) {
  CgScalars v;
  auto ld = [](auto* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  v.rr = ld(&st->rr);
  v.alpha = ld(&st->alpha);
  v.beta = ld(&st->beta);
  v.final_rr = ld(&st->final_rr);
  v.min_dec = ld(&st->min_dec);
  v.comm0 = ld(&st->comm[0]);
  v.comm1 = ld(&st->comm[1]);
  v.it = ld(&st->it);
  v.fails = ld(&st->fails);
  v.done = ld(&st->done);
  v.ret = ld(&st->ret);
  v.max_it = ld(&st->max_it);
  v.n_matvec = ld(&st->n_matvec);
  v.sharded = ld(&st->sharded);
  return v;
}
__device__ __forceinline__ void store_state_sc1(CgState* st, const CgScalars& v) {
  auto s = [](auto* p, auto x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  s(&st->rr, v.rr);
  s(&st->alpha, v.alpha);
  s(&st->beta, v.beta);
  s(&st->final_rr, v.final_rr);
  s(&st->min_dec, v.min_dec);
  s(&st->comm[0], v.comm0);
  s(&st->comm[1], v.comm1);
  s(&st->it, v.it);
  s(&st->fails, v.fails);
  s(&st->done, v.done);
  s(&st->ret, v.ret);
  s(&st->max_it, v.max_it);
  s(&st->n_matvec, v.n_matvec);
  s(&st->sharded, v.sharded);
}

// While a wave waits for iteration t's broadcast, its first entity of
// iteration t + 1 can already be on its way (MR_RS_PREFETCH): 1 loads its
// operands into registers (held across the barrier), 2 "touches" every
// 128-byte line of its G tiles and vectors with one dword load per lane
// (results discarded: the lines come into L2, no operand registers held),
// 3 = registers where they fit (NB > 4: 2 waves per SIMD) and touches
// below; 0 none.
#ifndef MR_RS_PREFETCH
#define MR_RS_PREFETCH 0
#endif
// poll interval of the broadcast wait (s_sleep units of 64 clocks): one
// poller per block, 4 blocks per CU
#ifndef MR_RS_SLEEP
#define MR_RS_SLEEP 1
#endif
__device__ __forceinline__ uint32_t touch_lines(const void* p, int64_t nbytes, int lane) {
  uint32_t s = 0;
  for (int64_t o = (int64_t)lane * 128; o < nbytes; o += 64 * 128)
    s += *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(p) + o);
  return s;
}
template <int NB, bool USER>
__device__ __forceinline__ uint32_t op_touch(const OpSide& A, int64_t e, int lane) {
  using T = OpEnt<NB>;
  uint32_t s = touch_lines(A.G + e * T::GS, T::GS * 4, lane);
  s += touch_lines(A.p + e * A.ldk, A.ldk * 8, lane);
  s += touch_lines(A.r + e * A.ldk, A.ldk * 8, lane);
  s += touch_lines(A.q + e * A.ldk, A.ldk * 8, lane);
  s += touch_lines(A.x + e * A.ldk, A.ldk * 4, lane);
  return s;
}
// The resident solve's control words live in device memory (ResCtl,
// Engine-owned) and are loaded where they are used, through a pointer made
// opaque at each use: kept in SGPRs for the whole kernel, the barrier's
// pointers pushed the one-pass body into SGPR spills (49 SGPRs into VGPR
// lanes, ~110 v_readlane in the loop) and its loads behind vmcnt(0) waits
// (users k = 64 full size: 207 vs 196 us per CG iteration).
template <class P>
__device__ __forceinline__ P* opaque_ptr(P* p) {
  asm volatile("" : "+s"(p));
  return p;
}

#ifndef MR_RS_WAVES
#define MR_RS_WAVES MR_OP_WAVES
#endif
template <int NB, bool USER, bool NT>
__global__ __launch_bounds__(256, (NB <= 4 ? MR_RS_WAVES : 2))
void cg_resident_kernel(const ResCtl* __restrict__ ctl, int t0, int sweep, int seq, OpSide A) {
  constexpr int XC = xchunk_of(NB, USER);
  using T = OpEnt<NB>;
  constexpr int PF = MR_RS_PREFETCH == 3 ? (NB > 4 ? 1 : 2) : MR_RS_PREFETCH;
  __shared__ MvScratch<NB> scr[MV_WAVES];
  __shared__ double rvs[MV_WAVES][16 * NB];
  __shared__ int64_t xacc[1][4][kXW];
  __shared__ double s_ab[2];
  __shared__ int s_flag[2];   // [0]: broadcast done (2: failed), [1]: last block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  // Wave j0 owns chunks j0, j0 + js, j0 + 2 js, ... (the one-pass deal,
  // fixed for the whole solve; its order reversed on alternate sweeps), so
  // at any moment the grid works on one contiguous window of the side.  A
  // deal of contiguous ranges per wave (counts balanced over the CUs) was
  // measured 10 % slower at full size and no better at shard 0/8
  // (profiles/r06/r06g).  Chunk counts fit 32 bits (E < 2^31 entities).
  const int nch = (int)((A.E + XC - 1) / XC);
  const int j0 = (int)blockIdx.x * MV_WAVES + wu, js = (int)gridDim.x * MV_WAVES;
  const int cnt = j0 < nch ? (nch - 1 - j0) / js + 1 : 0;   // chunks this wave owns
  // the i-th chunk of a sweep: ascending, or descending on reversed sweeps
  // (MR_OPT_CG_SWEEP: 1 = iteration 1 backwards, then alternate)
  auto rev_of = [&](int t) { return sweep == 0 ? 0 : ((t & 1) ^ (sweep == 2 ? 1 : 0)); };
  auto chunk0 = [&](int i, int rev) { return (int64_t)(j0 + (rev ? cnt - 1 - i : i) * js) * XC; };
  // the state at entry was written by the previous kernels of the stream
  CgState* st0 = opaque_ptr(ctl)->st;
  double alpha = ald(&st0->alpha), beta = ald(&st0->beta);
  int done = ald(&st0->done);
  if (threadIdx.x < 4 * kXW) (&xacc[0][0][0])[threadIdx.x] = 0;
  if (done) {
    // ended at the start: publish for the host; the start's pending update
    if (blockIdx.x == 0 && threadIdx.x == 0) publish(load_state(st0), ctl->mirror, seq);
    if (!ald(&st0->pending)) return;
  }
  int t = t0;
  OpEnt<NB> cur;
  if (PF == 1 && !done && cnt > 0) op_load<NB, USER, NT>(A, chunk0(0, rev_of(t)), t > 0, cur, lane);
  __syncthreads();
  while (!done) {
    const int update = t > 0, rev = rev_of(t);
    // MR_OP_PROF builds: the timeline of this launch's iteration t0 + 2
    // (tools/op_timeline.py --resident): per block start / chunks done /
    // arrival / broadcast seen; the last block's collect / compute / gen
    const bool prof = MR_OP_PROF && t == t0 + 2;
    if (prof && threadIdx.x == 0) op_prof(8);
    MvScratch<NB>& sc = scr[wid];
    double* rs = rvs[wid];
    for (int i = 0; i < cnt; ++i) {
      const int64_t c0 = chunk0(i, rev);
      const int64_t c1 = c0 + XC < A.E ? c0 + XC : A.E;
      double a = 0.0, b = 0.0, c = 0.0, d = 0.0;
      for (int64_t e = c0; e < c1; ++e) {
        if constexpr (PF == 1) {
          if (i != 0 || e != c0) op_load<NB, USER, NT>(A, e, update, cur, lane);
          op_process<NB, USER, NT>(A, e, update, alpha, beta, cur, sc, rs, a, b, c, d, lane);
        } else {
          OpEnt<NB> en;
          op_load<NB, USER, NT>(A, e, update, en, lane);
          op_process<NB, USER, NT>(A, e, update, alpha, beta, en, sc, rs, a, b, c, d, lane);
        }
      }
      op_chunk_terms(a, b, c, d, xacc, lane);
    }
    // the block's containers into the bins (and cleared for the next
    // iteration by the thread that read them), then the arrival.  Every
    // thread-derived address below comes from a fresh opaque copy of the
    // thread index: hoisted out of the iteration loop, these addresses would
    // stay live across the GEMV (17 VGPRs spilled at NB = 4)
    if (prof && (threadIdx.x & 63) == 0) op_prof(9);   // the block's last wave wins
    __syncthreads();
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const ResCtl* C = opaque_ptr(ctl);
    CgState* st = C->st;
    if (tid < 4 * kXW) {
      const int v = tid / kXW, dd = tid % kXW;
      const int64_t tt = xacc[0][v][dd];
      xacc[0][v][dd] = 0;
      if (tt != 0)
        __hip_atomic_fetch_add(C->xbins + ((int64_t)(blockIdx.x % kXBins) * 4 + v) * kXW + dd, tt,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_flag[1] = __hip_atomic_fetch_add(&st->arrive, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
      if (prof) op_prof(10);
    }
    __syncthreads();
    const bool fin = s_flag[1] && wid == 0;
    const uint64_t want = ((uint64_t)(uint32_t)seq << 32) | (uint32_t)(t + 1);
    uint32_t touched = 0;
    if (PF == 1) {
      // this wave's own stores of the iteration are complete before it
      // re-reads its first entity's vectors for the next one
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!fin && cnt > 0) op_load<NB, USER, NT>(A, chunk0(0, rev_of(t + 1)), 1, cur, lane);
    } else if (PF == 2 && !fin && cnt > 0) {
      touched = op_touch<NB, USER>(A, chunk0(0, rev_of(t + 1)), tid & 63);
    }
#ifndef MR_RSX_NOFIN
    if (fin) {
#else
    if (false) {
#endif
      __shared__ int64_t xs[4 * kXW];
      __shared__ double xv[4];
      const int lane = tid & 63;
      PeerComm* pc = ald(&st->peer);
      CgScalars v{};
      if (lane == 0) v = load_state_sc1(st);
      if (prof && lane == 0) op_prof(0);
      int64_t tot = xsum_collect<4>(C->xbins, lane);
      if (prof && lane == 0) op_prof(1);
      if (lane == 0) __hip_atomic_store(&st->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int flag = 0;
      if (pc && !peer_sum_lanes(pc, tot, 4 * kXW)) {
        if (lane == 0) {
          v.done = 1;
          v.ret = -1;
          store_state_sc1(st, v);
          publish(v, C->mirror, seq);
        }
        flag = 2;
      } else {
        if (lane < 4 * kXW) xs[lane] = tot;
        __builtin_amdgcn_wave_barrier();
        if (lane < 4) xv[lane] = xsum_value(&xs[lane * kXW]);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          double sum[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) sum[j] = xv[j];
          op_beta(v, sum, update);
          store_state_sc1(st, v);
          __hip_atomic_store(&st->pending, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v.done) publish(v, C->mirror, seq);
          flag = v.done;
        }
      }
      if (lane == 0) {
        __hip_atomic_store(&st->res_alpha, v.alpha, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&st->res_beta, v.beta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&st->res_done, flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (prof && lane == 0) op_prof(2);
      // every store above (state, broadcast, the bins' clears) written
      // through and drained before the generation word moves
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane < kResGenCopies)
        __hip_atomic_store(C->gen + lane * kResGenStride, want, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      // (no drain here: this block's own poll below simply repeats until
      // its generation store is visible)
      if (prof && lane == 0) op_prof(3);
      if (PF == 1 && cnt > 0) op_load<NB, USER, NT>(A, chunk0(0, rev_of(t + 1)), 1, cur, lane);
      if (PF == 2 && cnt > 0) touched = op_touch<NB, USER>(A, chunk0(0, rev_of(t + 1)), lane);
    }
    if (threadIdx.x == 0) {
      const uint64_t* g = C->gen + (blockIdx.x % kResGenCopies) * kResGenStride;
      const uint64_t tmo = C->timeout_ticks;
      const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      while (__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
        if (__builtin_amdgcn_s_memrealtime() - t_start > tmo) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(MR_RS_SLEEP);
      }
      if (prof) op_prof(11);
      s_ab[0] = __hip_atomic_load(&st->res_alpha, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_ab[1] = __hip_atomic_load(&st->res_beta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flag[0] = ok ? __hip_atomic_load(&st->res_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 2;
    }
    __syncthreads();
    if (PF == 2) asm volatile("" ::"v"(touched));   // the touches are not dead code
    // wave-uniform values back into scalar registers (LDS loads land in VGPRs)
    alpha = __builtin_bit_cast(double, ((int64_t)__builtin_amdgcn_readfirstlane(
                                            (int)__builtin_bit_cast(int64_t, s_ab[0])) & 0xFFFFFFFFll) |
                                           (int64_t)__builtin_amdgcn_readfirstlane(
                                               (int)(__builtin_bit_cast(int64_t, s_ab[0]) >> 32)) << 32);
    beta = __builtin_bit_cast(double, ((int64_t)__builtin_amdgcn_readfirstlane(
                                           (int)__builtin_bit_cast(int64_t, s_ab[1])) & 0xFFFFFFFFll) |
                                          (int64_t)__builtin_amdgcn_readfirstlane(
                                              (int)(__builtin_bit_cast(int64_t, s_ab[1]) >> 32)) << 32);
    done = __builtin_amdgcn_readfirstlane(s_flag[0]);
    if (done == 2) return;   // failed peer exchange or a broadcast that never came
    ++t;
    __syncthreads();   // s_ab / s_flag are rewritten by the next iteration
  }
  // the stopped iteration's x update (UPD_FINISH), entry by entry on this
  // wave's own entities: x += alpha p (its residual update would be dead)
#ifndef MR_RSX_NOFINISH
  for (int i = 0; i < cnt; ++i) {
    const int64_t c0 = chunk0(i, 0);
    const int64_t c1 = c0 + XC < A.E ? c0 + XC : A.E;
    for (int64_t e = c0; e < c1; ++e) {
#pragma unroll
      for (int h = 0; h < T::NV; ++h) {
        const int ii = lane + 64 * h;
        if (ii < T::NP) {
          float* xe = A.x + e * A.ldk + ii;
          *xe = (float)fma(alpha, A.p[e * A.ldk + ii], (double)*xe);
        }
      }
      if (USER && lane == 0) A.xb[e] = (float)fma(alpha, A.pb[e], (double)A.xb[e]);
    }
  }
#endif
}

// MR_OP_PROF builds: copy the last one-pass launch's timeline out (slots 0-3:
// the last block; then 4 per block: entry, entities done, flushed, unused)
int op_prof_read(int64_t* out, int n) {
  n = n < 8 + 4 * kOpProfBlocks ? n : 8 + 4 * kOpProfBlocks;
  MR_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_op_prof), (size_t)n * sizeof(int64_t)));
  return MR_OP_PROF ? n : 0;
}

int onepass_blocks_per_cu(bool user_side, int k, bool nt) {
  const void* f = nullptr;
#define MR_OP_FN(NB)                                                                        \
  case NB:                                                                                  \
    if (nt) f = user_side ? (const void*)cg_onepass_kernel<NB, true, true>                  \
                          : (const void*)cg_onepass_kernel<NB, false, true>;                \
    else f = user_side ? (const void*)cg_onepass_kernel<NB, true, false>                    \
                       : (const void*)cg_onepass_kernel<NB, false, false>;                  \
    break;
  switch (nb16_of(k)) {
    MR_OP_FN(1) MR_OP_FN(2) MR_OP_FN(3) MR_OP_FN(4)
    MR_OP_FN(5) MR_OP_FN(6) MR_OP_FN(7) MR_OP_FN(8)
    default: return 0;
  }
#undef MR_OP_FN
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess) return 0;
  return n;
}

int launch_cg_onepass(hipStream_t s, bool user_side, CgState* st, int update, int rev, int64_t E, int k,
                      const float* G, const float* Gs, const float* Gn, double* p, double* pb,
                      double* r, double* rb, double* q, double* qb, float* x, float* xb,
                      int64_t* xbins, int n_part, CgMirror* mirror, int seq, bool nt) {
  if (n_part <= 0) return 0;
#define MR_OP_LAUNCH(NB, U, T)                                                              \
  MR_LAUNCH((cg_onepass_kernel<NB, U, T>), dim3(n_part), dim3(256), 0, s, st, update, rev, E, k, \
            ldk_of(k), G, Gs, Gn, p, pb, r, rb, q, qb, x, xb, xbins, mirror, seq)
#define MR_OP_CASE(NB)                                                                      \
  case NB:                                                                                  \
    if (user_side) {                                                                        \
      if (nt) MR_OP_LAUNCH(NB, true, true); else MR_OP_LAUNCH(NB, true, false);             \
    } else {                                                                                \
      if (nt) MR_OP_LAUNCH(NB, false, true); else MR_OP_LAUNCH(NB, false, false);           \
    }                                                                                       \
    break;
  switch (nb16_of(k)) {
    MR_OP_CASE(1) MR_OP_CASE(2) MR_OP_CASE(3) MR_OP_CASE(4)
    MR_OP_CASE(5) MR_OP_CASE(6) MR_OP_CASE(7) MR_OP_CASE(8)
    default: set_error("one-pass CG needs k <= 128"); return -1;
  }
#undef MR_OP_CASE
#undef MR_OP_LAUNCH
  MR_HIP(hipGetLastError());
  return 0;
}

int resident_blocks_per_cu(bool user_side, int k, bool nt) {
  const void* f = nullptr;
#define MR_RS_FN(NB)                                                                        \
  case NB:                                                                                  \
    if (nt) f = user_side ? (const void*)cg_resident_kernel<NB, true, true>                 \
                          : (const void*)cg_resident_kernel<NB, false, true>;               \
    else f = user_side ? (const void*)cg_resident_kernel<NB, true, false>                   \
                       : (const void*)cg_resident_kernel<NB, false, false>;                 \
    break;
  switch (nb16_of(k)) {
    MR_RS_FN(1) MR_RS_FN(2) MR_RS_FN(3) MR_RS_FN(4)
    MR_RS_FN(5) MR_RS_FN(6) MR_RS_FN(7) MR_RS_FN(8)
    default: return 0;
  }
#undef MR_RS_FN
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess) return 0;
  return n;
}

int launch_cg_resident(hipStream_t s, bool user_side, const ResCtl* ctl, int t0, int sweep,
                       int64_t E, int k, const float* G, const float* Gs, const float* Gn, double* p,
                       double* pb, double* r, double* rb, double* q, double* qb, float* x,
                       float* xb, int n_part, int seq, bool nt) {
  if (n_part <= 0) return 0;
  const OpSide A{E, k, ldk_of(k), G, Gs, Gn, p, pb, r, rb, q, qb, x, xb};
#define MR_RS_LAUNCH(NB, U, T)                                                              \
  MR_LAUNCH((cg_resident_kernel<NB, U, T>), dim3(n_part), dim3(256), 0, s, ctl, t0, sweep, seq, A)
#define MR_RS_CASE(NB)                                                                      \
  case NB:                                                                                  \
    if (user_side) {                                                                        \
      if (nt) MR_RS_LAUNCH(NB, true, true); else MR_RS_LAUNCH(NB, true, false);             \
    } else {                                                                                \
      if (nt) MR_RS_LAUNCH(NB, false, true); else MR_RS_LAUNCH(NB, false, false);           \
    }                                                                                       \
    break;
  switch (nb16_of(k)) {
    MR_RS_CASE(1) MR_RS_CASE(2) MR_RS_CASE(3) MR_RS_CASE(4)
    MR_RS_CASE(5) MR_RS_CASE(6) MR_RS_CASE(7) MR_RS_CASE(8)
    default: set_error("resident CG needs k <= 128"); return -1;
  }
#undef MR_RS_CASE
#undef MR_RS_LAUNCH
  MR_HIP(hipGetLastError());
  return 0;
}

// K2 for k > 128: the same block GEMV (fused p update, fp64 products, p.q
// partial, control in the last block) with the tiles streamed from memory
// instead of held in registers: one wave per entity, two passes over the
// entity's tri16 tiles -- block rows (4-lane quad sums into yR), then block
// columns (16-lane column partials summed in a fixed order into yC) -- so G
// is read twice.  Per-wave LDS: p, yR, yC (16 NB doubles each) + 256 doubles.
template <bool USER>
__global__ __launch_bounds__(256) void cg_matvec_largek_kernel(
    const CgState* __restrict__ st, int update_p, int64_t E, int k,
    const float* __restrict__ G, const float* __restrict__ Gs, const float* __restrict__ Gn,
    double* __restrict__ v, double* __restrict__ vb, const double* __restrict__ r,
    const double* __restrict__ rb, double* __restrict__ y, double* __restrict__ yb,
    double* __restrict__ partials, CgState* fst, int phase, CgMirror* mirror, int beta_seq) {
  double beta = 0.0;
  bool skip;
  if (!matvec_entry(st, beta_seq, beta, skip)) return;
  extern __shared__ double lm_sm[];
  __shared__ double sh[MV_WAVES];
  const int NB = nb16_of(k), ldk = 16 * NB, NP = ldk;
  const int NO = n_off_of(NB), NF = n_fold_of(NB), NTILE = n_tiles_of(NB);
  const int64_t GS = gsize_of(k);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double* pv = lm_sm + (int64_t)wid * (3 * NP + 256);
  double* yR = pv + NP;
  double* yC = yR + NP;
  double* red = yC + NP;
  const int rr = lane >> 2, c4 = (lane & 3) * 4;
  double dsum = 0.0;
  auto diag_tile = [&](int b, bool& lower) {
    lower = (b & 1) && b < 2 * NF;
    return (b < 2 * NF) ? NO + (b >> 1) : NO + NF;
  };
  for (int64_t e = (int64_t)blockIdx.x * MV_WAVES + wid; e < (skip ? 0 : E);
       e += (int64_t)gridDim.x * MV_WAVES) {
    const float4* Ge = reinterpret_cast<const float4*>(G + e * GS);
    double* ve = v + e * ldk;
    // p = -r + beta p (matrix.cpp:521), staged in virtual order
    for (int i = lane; i < NP; i += 64) {
      double x = ve[i];
      if (update_p) {
        x = fma(beta, x, -r[e * ldk + i]);
        ve[i] = x;
      }
      pv[virt_of(i, NB)] = x;
    }
    double vbias = USER ? vb[e] : 0.0;
    if (USER && update_p) {
      vbias = fma(beta, vbias, -rb[e]);
      if (lane == 0) vb[e] = vbias;
    }
    __builtin_amdgcn_wave_barrier();
    // pass 1: block rows
    for (int bi = 0; bi < NB; ++bi) {
      double s0 = 0.0;
      for (int bj = bi + 1; bj < NB; ++bj) {
        const float4 g = Ge[(int64_t)off_index(bi, bj, NB) * 64 + lane];
        const double ge[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int x = 0; x < 4; ++x) s0 = fma(ge[x], pv[16 * bj + c4 + x], s0);
      }
      bool lower;
      const float4 g = Ge[(int64_t)diag_tile(bi, lower) * 64 + lane];
      const double ge[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int c = c4 + x;
        const bool use = lower ? (c < rr) : (c >= rr);
        s0 = fma(use ? ge[x] : 0.0, pv[16 * bi + c], s0);
      }
      const double rs = quad_sum_f64(s0);
      if ((lane & 3) == 0) yR[16 * bi + rr] = rs;
    }
    // pass 2: block columns
    for (int bj = 0; bj < NB; ++bj) {
      double cc[4] = {0.0, 0.0, 0.0, 0.0};
      for (int bi = 0; bi < bj; ++bi) {
        const float4 g = Ge[(int64_t)off_index(bi, bj, NB) * 64 + lane];
        const double ge[4] = {g.x, g.y, g.z, g.w};
        const double pi = pv[16 * bi + rr];
#pragma unroll
        for (int x = 0; x < 4; ++x) cc[x] = fma(ge[x], pi, cc[x]);
      }
      bool lower;
      const float4 g = Ge[(int64_t)diag_tile(bj, lower) * 64 + lane];
      const double ge[4] = {g.x, g.y, g.z, g.w};
      const double pr = pv[16 * bj + rr];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int c = c4 + x;
        const bool use = lower ? (c < rr) : (c > rr);
        cc[x] = fma(use ? ge[x] : 0.0, pr, cc[x]);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) red[4 * lane + x] = cc[x];
      __builtin_amdgcn_wave_barrier();
      if (lane < 16) {   // column c = lane: partials of rows rr = 0..15, fixed order
        double sacc = 0.0;
        for (int q = 0; q < 16; ++q) sacc += red[16 * q + lane];
        yC[16 * bj + lane] = sacc;
      }
      __builtin_amdgcn_wave_barrier();
    }
    // y = row + column parts (+ side diagonals of odd folded blocks, + bias column)
    const float* Gse = USER ? Gs + e * ldk : nullptr;
    double d = 0.0, ybp = 0.0;
    for (int o = lane; o < NP; o += 64) {
      const int n = nat_of(o, NB);
      if (n >= k) continue;
      const int b = o >> 4, ii = o & 15;
      double yv = yR[o] + yC[o];
      if ((b & 1) && b < 2 * NF)
        yv = fma((double)G[e * GS + (int64_t)NTILE * 256 + (b >> 1) * 16 + ii], pv[o], yv);
      if (USER) {
        const double gs = Gse[n];
        yv = fma(gs, vbias, yv);
        ybp = fma(gs, pv[o], ybp);
      }
      y[e * ldk + n] = yv;
      d = fma(yv, pv[o], d);
    }
    if (USER) {
      const double ybv = fma((double)Gn[e], vbias, wave_sum_f64(ybp));
      if (lane == 0) {
        yb[e] = ybv;
        d = fma(ybv, vbias, d);
      }
    }
    dsum += wave_sum_f64(d);
    __builtin_amdgcn_wave_barrier();
  }
  const double tot = block_sum_f64<256>(lane == 0 ? dsum : 0.0, sh);
  if (fst) store_partial(partials, tot);
  else if (threadIdx.x == 0) partials[blockIdx.x] = tot;
  if (fst && phase == CG_ALPHA) {
    if (beta_seq > 0) last_block_beta(fst, partials, mirror, beta_seq, sh);
    else last_block_finalize(fst, CG_ALPHA, partials, nullptr, 0, sh);
  }
}

int launch_cg_matvec(hipStream_t s, bool user_side, const CgState* st,
                     int update_p, int64_t E, int k, const float* G,
                     const float* Gs, const float* Gn, double* v, double* vb,
                     const double* r, const double* rb, double* y, double* yb,
                     double* partials, int n_part, CgState* fst, int phase,
                     CgMirror* mirror, int beta_seq) {
  if (n_part <= 0) return 0;
  if (k > kMaxK) {
    const int NP = ldk_of(k);
    const size_t lds = (size_t)MV_WAVES * (3 * NP + 256) * sizeof(double);
    if (user_side) {
      MR_HIP(hipFuncSetAttribute((const void*)cg_matvec_largek_kernel<true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      MR_LAUNCH(cg_matvec_largek_kernel<true>, dim3(n_part), dim3(256), lds, s, st, update_p, E,
                k, G, Gs, Gn, v, vb, r, rb, y, yb, partials, fst, phase, mirror, beta_seq);
    } else {
      MR_HIP(hipFuncSetAttribute((const void*)cg_matvec_largek_kernel<false>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      MR_LAUNCH(cg_matvec_largek_kernel<false>, dim3(n_part), dim3(256), lds, s, st, update_p, E,
                k, G, Gs, Gn, v, vb, r, rb, y, yb, partials, fst, phase, mirror, beta_seq);
    }
    MR_HIP(hipGetLastError());
    return 0;
  }
#define MR_MV_CASE(NB)                                                                   \
  case NB:                                                                               \
    if (user_side)                                                                       \
      MR_LAUNCH((cg_matvec_kernel<NB, true>), dim3(n_part), dim3(256), 0, s, st, update_p, \
                E, k, ldk_of(k), G, Gs, Gn, v, vb, r, rb, y, yb, partials, fst, phase,    \
                mirror, beta_seq);                                                       \
    else                                                                                 \
      MR_LAUNCH((cg_matvec_kernel<NB, false>), dim3(n_part), dim3(256), 0, s, st,         \
                update_p, E, k, ldk_of(k), G, Gs, Gn, v, vb, r, rb, y, yb, partials, fst, \
                phase, mirror, beta_seq);                                                \
    break;
  switch (nb16_of(k)) {
    MR_MV_CASE(1) MR_MV_CASE(2) MR_MV_CASE(3) MR_MV_CASE(4)
    MR_MV_CASE(5) MR_MV_CASE(6) MR_MV_CASE(7) MR_MV_CASE(8)
    default: set_error("k > 128 not supported by the CG matvec"); return -1;
  }
#undef MR_MV_CASE
  MR_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// CG vector update (matrix.cpp:468-476 init, :501-507 step) + r.r partials.
// x is the fp32 factor table, r / p / q are fp64; four elements per thread
// and step.  Fixed grid, grid-stride: reproducible partial sums.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cg_update_kernel(
    const CgState* __restrict__ st, int mode, int64_t n4, int64_t nb,
    float* __restrict__ x, double* __restrict__ r, double* __restrict__ p,
    const double* __restrict__ q, const float* __restrict__ c,
    float* __restrict__ xb, double* __restrict__ rb, double* __restrict__ pb,
    const double* __restrict__ qb, const float* __restrict__ cb,
    double* __restrict__ partials, CgState* fst, CgMirror* mirror, int seq) {
  // UPD_FINISH (one-pass CG): the stopped solve's deferred last update, if any
  if (mode == UPD_FINISH ? !ald(&st->pending) : ald(&st->done) != 0) return;
  __shared__ double sh[4];
  // sharded runs: alpha = rr / (all-reduced p.Ap), the ALPHA rule inline
  const double alpha = ald(&st->sharded) && mode != UPD_INIT ? ald(&st->rr) / ald(&st->comm[0])
                                                             : ald(&st->alpha);
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double2* r2 = reinterpret_cast<double2*>(r);
  double2* p2 = reinterpret_cast<double2*>(p);
  const double2* q2 = reinterpret_cast<const double2*>(q);
  if (mode == UPD_INIT) {
    const float4* c4 = reinterpret_cast<const float4*>(c);
    for (int64_t i = tid; i < n4; i += stride) {
      const double2 qa = q2[2 * i], qb2 = q2[2 * i + 1];
      const float4 cv = c4[i];
      const double2 ra = make_double2(qa.x - (double)cv.x, qa.y - (double)cv.y);
      const double2 rb2 = make_double2(qb2.x - (double)cv.z, qb2.y - (double)cv.w);
      r2[2 * i] = ra;
      r2[2 * i + 1] = rb2;
      p2[2 * i] = make_double2(-ra.x, -ra.y);
      p2[2 * i + 1] = make_double2(-rb2.x, -rb2.y);
      acc = fma(ra.x, ra.x, acc);
      acc = fma(ra.y, ra.y, acc);
      acc = fma(rb2.x, rb2.x, acc);
      acc = fma(rb2.y, rb2.y, acc);
    }
    for (int64_t i = tid; i < nb; i += stride) {
      const double rv = qb[i] - (double)cb[i];
      rb[i] = rv;
      pb[i] = -rv;
      acc = fma(rv, rv, acc);
    }
  } else if (mode == UPD_FINISH) {
    // the stopped one-pass solve's last x update only: its residual update
    // would be dead (the next solve of this side starts from r0 = G x - c)
    float4* x4 = reinterpret_cast<float4*>(x);
    for (int64_t i = tid; i < n4; i += stride) {
      float4 xv = x4[i];
      const double2 pa = p2[2 * i], pb2 = p2[2 * i + 1];
      xv.x = (float)fma(alpha, pa.x, (double)xv.x);
      xv.y = (float)fma(alpha, pa.y, (double)xv.y);
      xv.z = (float)fma(alpha, pb2.x, (double)xv.z);
      xv.w = (float)fma(alpha, pb2.y, (double)xv.w);
      x4[i] = xv;
    }
    for (int64_t i = tid; i < nb; i += stride) xb[i] = (float)fma(alpha, pb[i], (double)xb[i]);
    return;
  } else {
    float4* x4 = reinterpret_cast<float4*>(x);
    for (int64_t i = tid; i < n4; i += stride) {
      float4 xv = x4[i];
      const double2 pa = p2[2 * i], pb2 = p2[2 * i + 1];
      const double2 qa = q2[2 * i], qb2 = q2[2 * i + 1];
      double2 ra = r2[2 * i], rb2 = r2[2 * i + 1];
      xv.x = (float)fma(alpha, pa.x, (double)xv.x);
      xv.y = (float)fma(alpha, pa.y, (double)xv.y);
      xv.z = (float)fma(alpha, pb2.x, (double)xv.z);
      xv.w = (float)fma(alpha, pb2.y, (double)xv.w);
      ra.x = fma(alpha, qa.x, ra.x);
      ra.y = fma(alpha, qa.y, ra.y);
      rb2.x = fma(alpha, qb2.x, rb2.x);
      rb2.y = fma(alpha, qb2.y, rb2.y);
      x4[i] = xv;
      r2[2 * i] = ra;
      r2[2 * i + 1] = rb2;
      acc = fma(ra.x, ra.x, acc);
      acc = fma(ra.y, ra.y, acc);
      acc = fma(rb2.x, rb2.x, acc);
      acc = fma(rb2.y, rb2.y, acc);
    }
    for (int64_t i = tid; i < nb; i += stride) {
      xb[i] = (float)fma(alpha, pb[i], (double)xb[i]);
      const double rv = fma(alpha, qb[i], rb[i]);
      rb[i] = rv;
      acc = fma(rv, rv, acc);
    }
  }
  if (mode == UPD_FINISH) return;
  const double tot = block_sum_f64<256>(acc, sh);
  if (fst) store_partial(partials, tot);
  else if (threadIdx.x == 0) partials[blockIdx.x] = tot;
  if (fst)
    last_block_finalize(fst, mode == UPD_INIT ? CG_INIT : CG_BETA, partials, mirror, seq, sh);
}

int launch_cg_update(hipStream_t s, const CgState* st, int mode, int64_t n,
                     int64_t nb, float* x, double* r, double* p, const double* q,
                     const float* c, float* xb, double* rb, double* pb,
                     const double* qb, const float* cb, double* partials,
                     int n_part, CgState* fst, CgMirror* mirror, int seq) {
  MR_LAUNCH(cg_update_kernel, dim3(n_part), dim3(256), 0, s,
      st, mode, n / 4, nb, x, r, p, q, c, xb, rb, pb, qb, cb, partials, fst, mirror, seq);
  MR_HIP(hipGetLastError());
  return 0;
}

// Unfused CG start: v = x (fp32 factor rows, + bias) as fp64, so the matvec
// can form G x.
__global__ void x_to_vec_kernel(int64_t n, int64_t nb, const float* __restrict__ x,
                                const float* __restrict__ xb, double* __restrict__ v,
                                double* __restrict__ vb) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    v[t] = x[t];
    if (t < nb) vb[t] = xb[t];
  }
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

__device__ bool start_reduce_xbins(CgState* st, int64_t* start_xbins, bool exchange,
                                   CgMirror* mirror, int seq);
__device__ void start_rule(CgState* st, CgMirror* mirror, int seq, double min_dec, int max_it,
                           int sharded);

constexpr int CTL_THREADS = 1024;
__global__ __launch_bounds__(CTL_THREADS) void cg_control_kernel(
    CgState* __restrict__ st, int phase, int ctl,
    const double* __restrict__ partials, int n_part, CgMirror* mirror, int seq,
    double min_dec, int max_it, int sharded, int64_t* __restrict__ start_xbins) {
  if (phase != CG_INIT && phase != CG_START && ald(&st->done)) return;
  __shared__ double sh[CTL_THREADS / 64];
  if (ctl & CTL_REDUCE) {
    if (phase == CG_START && start_xbins) {
      // one-pass CG: the start's sums from the order-independent bins (wave
      // 0), exchanged as integers with the peers, then to fp64
      if (threadIdx.x >= 64) return;
      if (!start_reduce_xbins(st, start_xbins, (ctl & CTL_FINALIZE) != 0, mirror, seq)) return;
    } else if (phase == CG_START) {
      // (r.r, p.Gp, q.q) triples (one per Gram block: ~E/4 of them, written
      // by every XCD): thread t sums triples t, t + T, t + 2T, ... in order,
      // 8 loads in flight, then the fixed-order block tree.
      double a = 0.0, b = 0.0, c = 0.0;
      for (int base = 0; base < n_part; base += 8 * CTL_THREADS) {
        double v[8][3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = base + j * CTL_THREADS + threadIdx.x;
#pragma unroll
          for (int m = 0; m < 3; ++m) v[j][m] = (i < n_part) ? partials[3 * (int64_t)i + m] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a += v[j][0];
          b += v[j][1];
          c += v[j][2];
        }
      }
      const double ta = block_sum_f64<CTL_THREADS>(a, sh);
      __syncthreads();
      const double tb = block_sum_f64<CTL_THREADS>(b, sh);
      __syncthreads();
      const double tc = block_sum_f64<CTL_THREADS>(c, sh);
      if (threadIdx.x == 0) {
        double t3[3] = {ta, tb, tc};
        PeerComm* pc = ald(&st->peer);
        if (pc && (ctl & CTL_FINALIZE) && !peer_sum(pc, t3, 3)) {
          ast(&st->comm[0], 0.0);
          ast(&st->comm[1], 0.0);
          peer_fail(st, mirror, seq);
          return;
        }
        ast(&st->comm[0], t3[0]);
        ast(&st->comm[1], t3[1]);
        ast(&st->comm[2], t3[2]);
      }
    } else {
      double acc = 0.0;
      for (int i = threadIdx.x; i < n_part; i += blockDim.x) acc += partials[i];
      const double tot = block_sum_f64<CTL_THREADS>(acc, sh);
      if (threadIdx.x == 0) ast(&st->comm[0], tot);
    }
  }
  if (threadIdx.x != 0 || !(ctl & CTL_FINALIZE)) return;
  if (phase == CG_START) {
    start_rule(st, mirror, seq, min_dec, max_it, sharded);
    return;
  }
  cg_finalize(st, phase, ald(&st->comm[0]), mirror, seq);
}

// The start's three sums from the order-independent bins, by one wave: peers
// exchange the integer containers (when `exchange` and sharded), lane 0
// stores the fp64 values into comm[0..2].  False on a peer timeout (the state
// is then failed and published).
__device__ bool start_reduce_xbins(CgState* st, int64_t* start_xbins, bool exchange,
                                   CgMirror* mirror, int seq) {
  const int lane = threadIdx.x & 63;
  __shared__ int64_t xs[3 * kXW];
  int64_t t = xsum_collect<3>(start_xbins, lane);
  PeerComm* pc = ald(&st->peer);
  if (pc && exchange && !peer_sum_lanes(pc, t, 3 * kXW)) {
    if (lane == 0) {
      ast(&st->comm[0], 0.0);
      ast(&st->comm[1], 0.0);
      peer_fail(st, mirror, seq);
    }
    return false;
  }
  if (lane < 3 * kXW) xs[lane] = t;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    ast(&st->comm[0], xsum_value(&xs[0]));
    ast(&st->comm[1], xsum_value(&xs[kXW]));
    ast(&st->comm[2], xsum_value(&xs[2 * kXW]));
  }
  return true;
}

__device__ void start_fold_finalize(const StartFold& f, int64_t* start_xbins) {
  // the counter is reset first, so a failed peer exchange leaves it clean too
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store(&f.st->arrive_start, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!start_reduce_xbins(f.st, start_xbins, true, f.mirror, f.seq)) return;
  if ((threadIdx.x & 63) == 0) start_rule(f.st, f.mirror, f.seq, f.min_dec, f.max_it, f.sharded);
}

// CG_START rule, by one thread: fresh state (cg_least_squares entry), then
// the INIT rule on r0.r0 and, unless that ended the solve, alpha of
// iteration 0 from p0.G p0 (comm[0..2] hold r0.r0, p0.q0, q0.q0)
__device__ void start_rule(CgState* st, CgMirror* mirror, int seq, double min_dec, int max_it,
                           int sharded) {
  {
    CgScalars v;
    const double rr = ald(&st->comm[0]), pq = ald(&st->comm[1]);
    const int onepass = (sharded >> 1) & 1;   // bit 1 of the argument
    v.min_dec = min_dec;
    v.max_it = max_it;
    v.sharded = sharded & 1;
    ast(&st->onepass, onepass);
    v.n_matvec = 0;
    v.alpha = 0.0;
    v.beta = 0.0;
    v.rr = rr;
    v.final_rr = rr;
    v.it = 0;
    v.fails = 0;
    v.ret = 0;
    v.comm0 = rr;
    v.comm1 = pq;
    v.done = (max_it <= 0 || (rr < 1e-6 && !MR_SP_PROBE)) ? 1 : 0;
    if (!v.done) {
      v.alpha = rr / pq;
      v.comm0 = pq;      // sharded updates derive alpha as rr / comm[0]
      v.n_matvec = 1;    // the fused iteration-0 matvec
    }
    ast(&st->arrive, 0u);
    ast(&st->pending, 0);
    if (onepass && !v.done) {
      // one-pass CG: iteration 0's BETA step now, from r1.r1 = r0.r0 +
      // 2 alpha r0.q0 + alpha^2 q0.q0 with r0.q0 = -p0.q0 (p0 = -r0 exactly);
      // its x / r update is applied by iteration 1's kernel (or the finish)
      const double qq = ald(&st->comm[2]);
      const double a = v.alpha;
      apply_beta(v, fma(a * a, qq, fma(-2.0 * a, pq, rr)));
      ast(&st->pending, 1);
    }
    store_state(st, v);
    publish(v, mirror, seq);
  }
}

int launch_cg_control(hipStream_t s, CgState* st, int phase, int ctl,
                      const double* partials, int n_part, CgMirror* mirror, int seq,
                      double min_dec, int max_it, int sharded, int64_t* start_xbins) {
  MR_LAUNCH(cg_control_kernel, dim3(1), dim3(CTL_THREADS), 0, s, st, phase, ctl, partials, n_part,
                                                  mirror, seq, min_dec, max_it, sharded, start_xbins);
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
  const int nb = nb16_of(k);
  const float* Ge = G + e * gsize_of(k);
  for (int t = threadIdx.x; t < K * K; t += blockDim.x) {
    const int i = t / K, j = t - (t / K) * K;
    double v;
    if (i < k && j < k) v = Ge[packed_offset(i, j, nb)];
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
  MR_CHECK(k <= kMaxK, "the exact (Cholesky) solver holds K x K in LDS: k <= 128");
  const int K = user_side ? k + 1 : k;
  const size_t lds = (size_t)(K * K + K) * sizeof(double);
  if (user_side) {
    MR_HIP(hipFuncSetAttribute((const void*)solve_kernel<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    MR_LAUNCH(solve_kernel<true>, dim3((unsigned)E), dim3(256), lds, s,
        E, k, ldk_of(k), ridge, G, Gs, Gn, C, Cb, x, xb, nonpd);
  } else {
    MR_HIP(hipFuncSetAttribute((const void*)solve_kernel<false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    MR_LAUNCH(solve_kernel<false>, dim3((unsigned)E), dim3(256), lds, s,
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

__global__ void pack_rows_kernel(int64_t n4, int ldk4, const float4* __restrict__ fac,
                                 const float* __restrict__ bias, float4* __restrict__ send,
                                 float* __restrict__ send_b) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4;
       t += (int64_t)gridDim.x * blockDim.x) {
    send[t] = fac[t];
    if (bias && t % ldk4 == 0) send_b[t / ldk4] = bias[t / ldk4];
  }
}

int launch_pack_rows(hipStream_t s, int64_t r0, int64_t n, int ldk, const float* fac,
                     const float* bias, float* send, float* send_b) {
  if (n <= 0) return 0;
  const int ldk4 = ldk / 4;
  pack_rows_kernel<<<grid_for(n * ldk4), 256, 0, s>>>(
      n * ldk4, ldk4, reinterpret_cast<const float4*>(fac + r0 * ldk), bias ? bias + r0 : nullptr,
      reinterpret_cast<float4*>(send), send_b);
  MR_HIP(hipGetLastError());
  return 0;
}

// The gathered buffer holds one block per rank: maxrows x ldk factor floats,
// then (users) maxrows bias floats padded to a multiple of 4 (ag_block_floats),
// so factors and biases travel in ONE all-gather.
__global__ void unstage_rows_kernel(int world, int skip, const int64_t* __restrict__ rb,
                                    int64_t maxrows, int ldk4, int64_t stride4,
                                    const float4* __restrict__ recv, float4* __restrict__ fac,
                                    float* __restrict__ bias) {
  const int64_t per = maxrows * ldk4;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < (int64_t)world * per;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(t / per);
    const int64_t rem = t - (int64_t)r * per;
    const int64_t j = rem / ldk4;
    if (r == skip || j >= rb[r + 1] - rb[r]) continue;
    const int c = (int)(rem - j * ldk4);
    fac[(rb[r] + j) * ldk4 + c] = recv[r * stride4 + rem];
    if (bias && c == 0)
      bias[rb[r] + j] = reinterpret_cast<const float*>(recv + r * stride4 + per)[j];
  }
}

int64_t ag_block_floats(int64_t maxrows, int ldk, bool with_bias) {
  return maxrows * ldk + (with_bias ? (maxrows + 3) / 4 * 4 : 0);
}

int launch_unstage_rows(hipStream_t s, int world, int skip, const int64_t* rb,
                        int64_t maxrows, int ldk, const float* recv, float* fac, float* bias) {
  const int ldk4 = ldk / 4;
  const int64_t stride4 = ag_block_floats(maxrows, ldk, bias != nullptr) / 4;
  unstage_rows_kernel<<<grid_for((int64_t)world * maxrows * ldk4), 256, 0, s>>>(
      world, skip, rb, maxrows, ldk4, stride4, reinterpret_cast<const float4*>(recv),
      reinterpret_cast<float4*>(fac), bias);
  MR_HIP(hipGetLastError());
  return 0;
}

// Seeded uniform(-1, 1) factors generated on the device (splitmix64 of the
// (table, row, column) index): identical on every rank, no host table
// (multi-GB at C5).  Padding columns stay 0.
__device__ __forceinline__ double unit_hash(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (double)(x >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

__global__ void init_factors_kernel(int64_t rows, int k, int ldk, uint64_t seed, int table,
                                    float* __restrict__ fac, float* __restrict__ bias) {
  const int64_t n = rows * ldk;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / ldk;
    const int c = (int)(t - r * ldk);
    const uint64_t base = (seed * 0x100000001B3ull) ^ ((uint64_t)table << 60);
    fac[t] = c < k ? (float)unit_hash(base + (uint64_t)r * (k + 1) + c) : 0.f;
    if (bias && c == 0) bias[r] = (float)unit_hash(base + (uint64_t)r * (k + 1) + k);
  }
}

int launch_init_factors(hipStream_t s, int64_t rows, int k, int ldk, uint64_t seed, int table,
                        float* fac, float* bias) {
  if (rows <= 0) return 0;
  init_factors_kernel<<<grid_for(rows * ldk), 256, 0, s>>>(rows, k, ldk, seed, table, fac, bias);
  MR_HIP(hipGetLastError());
  return 0;
}

int launch_x_to_vec(hipStream_t s, int64_t n, int64_t nb, const float* x, const float* xb,
                    double* v, double* vb) {
  if (n <= 0) return 0;
  x_to_vec_kernel<<<grid_for(n), 256, 0, s>>>(n, nb, x, xb, v, vb);
  MR_HIP(hipGetLastError());
  return 0;
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
// General CSR least squares in fp64 (cg_least_squares_from_python,
// matrix.cpp:456-529): three kernels per CG iteration on A (CSR) and its
// explicit transpose At (CSR of A^T, built once per context):
//   K1  t = A p           rows of A; p = -r + beta p formed at each gather
//                         (matrix.cpp:521 of the previous iteration)
//   K2  q = At t          rows of At = columns of A; each writes its new p_j
//                         and adds p_j q_j to the p.Ap partial; the last
//                         workgroup computes alpha (:497)
//   K3  x += alpha p, r += alpha q, r.r partial; the last workgroup applies
//       the BETA rule and publishes the state (:501-518)
// K1 / K2 are CSR-stream SpMVs: a workgroup takes a "row block" (consecutive
// rows holding <= SP_TILE non-zeros, <= 256 rows; a longer row is a block of
// its own), streams the block's values / column ids with consecutive lanes
// on consecutive non-zeros (fully coalesced), stages the products in LDS,
// then sums each row from LDS with a group of G threads (G = the largest
// power of two <= 256 / rows; G = 1: one thread per row in index order, the
// reference's own row order).  Row blocks are dealt to a fixed grid
// (grid-stride), so every partial sum has a fixed order: results are
// reproducible.  Arithmetic follows the reference's expressions with
// contraction off (x86 -O2 builds do not fuse): -1*r + beta*p, x + alpha*p,
// r + alpha*q, sum += v*x.
// ---------------------------------------------------------------------------
constexpr int SP_THREADS = 256;
#ifndef MR_SP_ORDER   // 1: a block's gathers issued before the next block's stream loads
#define MR_SP_ORDER 1
#endif
#ifndef MR_SP_PRELOAD   // 1: the CG output pass preloads its rows' (r, p) pairs
#define MR_SP_PRELOAD 1
#endif
#ifndef MR_SP_OUT   // policy of the output stores: 0 default, 1 non-temporal, 2 write-through (sc1)
#define MR_SP_OUT 0
#endif
#ifndef MR_SP_AUX   // cache policy of the once-read id / value streams (0: default; nt measured 4 % slower)
#define MR_SP_AUX 0
#endif
constexpr int SP_TILE = kSpTile;     // staged products per row block (16 KiB fp64)

template <int GATHER, int OUT, bool BUF>
__global__ __launch_bounds__(SP_THREADS) void csr_spmv_kernel(
    const CgState* __restrict__ st, int64_t n_blk, const int64_t* __restrict__ blk,
    const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
    const double* __restrict__ v, const double* __restrict__ xa, const double* __restrict__ xb,
    uint32_t xbytes,
    double* __restrict__ out, double* __restrict__ pv, const double* __restrict__ rv,
    int update_p, double* __restrict__ partials, CgState* fst) {
#pragma clang fp contract(off)
  if (st && ald(&st->done)) return;
  const double beta = (st && (GATHER == SPG_P || update_p)) ? ald(&st->beta) : 0.0;
  static_assert(OUT != SPO_CG || GATHER == SPG_X, "the CG output pass gathers t");
  __shared__ double prod[SP_TILE];
  __shared__ double sh[SP_THREADS / 64];
  const int t = threadIdx.x;
  double d = 0.0;   // OUT == SPO_CG: this thread's share of p.q
  // BUF (gathered vectors < 4 GiB): buffer resources, so a load is a 32-bit
  // offset from SGPR bases instead of 64-bit per-lane address arithmetic
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(xa), (short)0, (int)xbytes, 0x00020000);
  auto gather = [&](int32_t c) -> double {
    if constexpr (GATHER == SPG_P) {   // p_c = -r_c + beta p_c from one 16-byte (r, p) pair
      double2 w;
      if constexpr (BUF)
        w = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(ra, (int)((uint32_t)c * 16u), 0, 0));
      else
        w = reinterpret_cast<const double2*>(xa)[c];
      return -1.0 * w.x + beta * w.y;
    } else {
      const uint32_t i = GATHER == SPG_P0 ? 2u * (uint32_t)c + 1u : (uint32_t)c;
      if constexpr (BUF)
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(ra, (int)(i * 8u), 0, 0));
      else
        return xa[GATHER == SPG_P0 ? 2 * (int64_t)c + 1 : (int64_t)c];
    }
  };
  double probe_sink = 0.0;
  auto emit = [&](int64_t row, double s) {
    if (MR_SP_PROBE & 4) probe_sink += s;
    else if (MR_SP_OUT == 1) __builtin_nontemporal_store(s, out + row);
    else if (MR_SP_OUT == 2) asm volatile("global_store_dwordx2 %0, %1, off sc1" : : "v"(out + row), "v"(s) : "memory");
    else out[row] = s;
    if constexpr (OUT == SPO_CG) {   // pv = the interleaved (r, p) pairs
      double pn = pv[2 * row + 1];
      if (update_p) {
        pn = -1.0 * pv[2 * row] + beta * pn;   // vect_add(-1, r, beta, p, p)
        pv[2 * row + 1] = pn;
      }
      d += pn * s;
    }
  };
  // the CG output pass with the row's (r, p) pair loaded beside the block's
  // gathers (and staged in LDS for the summing thread) instead of after the
  // row sum: the same arithmetic without a dependent global load per block
  auto emit_cg = [&](int64_t row, double s, double2 rp) {
    if (MR_SP_PROBE & 4) probe_sink += s;
    else out[row] = s;
    double pn = rp.y;
    if (update_p) {
      pn = -1.0 * rp.x + beta * pn;   // vect_add(-1, r, beta, p, p)
      pv[2 * row + 1] = pn;
    }
    d += pn * s;
  };
  // Software pipeline over the workgroup's row blocks b, b + grid, ...: the
  // next short block's column ids, values and row offsets are loaded into a
  // second register set at the top of the current block (in flight during
  // its gathers, products and sums), and block bounds (blk: (first row, first
  // non-zero) pairs) are fetched two blocks ahead, so no load chain is
  // exposed per block.  Products and
  // row sums are unchanged: results are bitwise those of the plain loop.
  constexpr int PER = SP_TILE / SP_THREADS;
  __shared__ int32_t srp[kSpMaxRows + 1];   // the block's row offsets - n0
  __shared__ double2 spv[OUT == SPO_CG && MR_SP_PRELOAD && MR_SP_ORDER ? kSpMaxRows : 1];   // their (r, p) pairs
  struct Stage {
    int32_t cc[PER];
    double vv[PER];
    int64_t ro;   // rp[first row + t] (raw: converted where it is used)
  };
  auto load_short = [&](Stage& S, int64_t r0, int64_t r1, int64_t n0, int64_t n1) {
    if constexpr (BUF) {
      // thread t takes the entry pairs m = 256 u + t, u = 0..3 (entries 2m,
      // 2m + 1: one 16-byte value load and one 8-byte id load each, so every
      // instruction reads one contiguous run -- 1 KiB of values, 512 B of
      // ids; lanes 64 B apart measured 2.6 % slower).  The arrays are padded
      // by kSpPad entries, so no load leaves the allocation; entries past the
      // block are read but never used (their products are not staged), and a
      // gather of such an id is bounded by the vector's resource (resources
      // end at the block's entry count rounded up to 8: every load is wholly
      // inside -- within the padding -- or wholly out of range, and
      // out-of-range loads read 0 without touching memory)
      const int n8 = ((int)(n1 - n0) + 7) & ~7;
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(ci + n0), (short)0, n8 * 4, 0x00020000);
      const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<double*>(v + n0), (short)0, n8 * 8, 0x00020000);
      static_assert(PER == 8, "8 entries per thread");
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = 256 * u + t;
        const u32x2_t c2 = __builtin_bit_cast(
            u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(rc, m * 8, 0, MR_SP_AUX));
        S.cc[2 * u] = (int32_t)c2[0];
        S.cc[2 * u + 1] = (int32_t)c2[1];
        const u32x4_t w4 = __builtin_bit_cast(
            u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rw, m * 16, 0, MR_SP_AUX));
        S.vv[2 * u] = __builtin_bit_cast(double, ((uint64_t)w4[1] << 32) | w4[0]);
        S.vv[2 * u + 1] = __builtin_bit_cast(double, ((uint64_t)w4[3] << 32) | w4[2]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int64_t j = n0 + t + (int64_t)u * SP_THREADS;
        const int64_t js = j < n1 ? j : 0;     // a valid address (arrays hold >= 1 entry)
        const int32_t c = ci[js];
        S.vv[u] = v[js];
        S.cc[u] = j < n1 ? c : 0;
      }
    }
    // every thread loads (a clamped row: rp holds rows + 1 entries) and the
    // offset is formed where it is used: a load under `t < rows` (or a select
    // right behind it) made the compiler wait for it at once -- draining the
    // next block's stream loads issued just before
    const int64_t nr = r1 - r0;
    if (MR_SP_PROBE & 8)
      S.ro = n0 + min((int64_t)t * ((n1 - n0) / (nr > 0 ? nr : 1)), n1 - n0);
    else
      S.ro = rp[r0 + (t < nr ? t : nr)];

  };
  Stage cur, nxt;
  int64_t b = blockIdx.x;
  const int64_t gs = gridDim.x;
  int64_t r0 = 0, r1 = 0, n0 = 0, n1 = 0;      // block b
  int64_t qr0 = 0, qr1 = 0, qn0 = 0, qn1 = 0;  // block b + gs
  if (b < n_blk) {
    r0 = blk[2 * b];
    n0 = blk[2 * b + 1];
    r1 = blk[2 * b + 2];
    n1 = blk[2 * b + 3];
    if (b + gs < n_blk) {
      qr0 = blk[2 * (b + gs)];
      qn0 = blk[2 * (b + gs) + 1];
      qr1 = blk[2 * (b + gs) + 2];
      qn1 = blk[2 * (b + gs) + 3];
    }
    if (n1 - n0 <= SP_TILE) load_short(cur, r0, r1, n0, n1);
  }
  for (; b < n_blk; b += gs) {
    const bool has_next = b + gs < n_blk, has_next2 = b + 2 * gs < n_blk;
    const bool next_short = has_next && qn1 - qn0 <= SP_TILE;
    const bool cur_short = n1 - n0 <= SP_TILE;
    double gx[PER];
    double2 rpair;   // OUT == SPO_CG: row r0 + t's (r, p) pair, loaded with the gathers
    if (MR_SP_ORDER && cur_short) {
      // this block's gathers first, then the next block's stream: waiting for
      // the gathers (in-order vmcnt) then leaves the stream in flight
#pragma unroll
      for (int u = 0; u < PER; ++u) gx[u] = (MR_SP_PROBE & 1) ? 1.0 + (double)cur.cc[u] : gather(cur.cc[u]);
      if constexpr (OUT == SPO_CG && MR_SP_PRELOAD) {
        const int64_t nr = r1 - r0;
        rpair = reinterpret_cast<const double2*>(pv)[r0 + (t < nr ? t : nr - 1)];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (next_short) load_short(nxt, qr0, qr1, qn0, qn1);
    int64_t sr0 = 0, sr1 = 0, sn0 = 0, sn1 = 0;   // bounds of block b + 2 gs
    if (has_next2) {
      sr0 = blk[2 * (b + 2 * gs)];
      sn0 = blk[2 * (b + 2 * gs) + 1];
      sr1 = blk[2 * (b + 2 * gs) + 2];
      sn1 = blk[2 * (b + 2 * gs) + 3];
    }
    if (cur_short) {
      if (!MR_SP_ORDER) {
#pragma unroll
        for (int u = 0; u < PER; ++u) gx[u] = (MR_SP_PROBE & 1) ? 1.0 + (double)cur.cc[u] : gather(cur.cc[u]);
      }
      const int nl = (int)(n1 - n0);
      if constexpr ((MR_SP_PROBE & 2) != 0) {
        double sum = 0.0;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int jl = BUF ? 2 * (256 * (u >> 1) + t) + (u & 1) : t + u * SP_THREADS;
          if (jl < nl) sum += cur.vv[u] * gx[u];
        }
        const int R = (int)(r1 - r0);
        if (t < R) emit(r0 + t, sum + (double)cur.ro);
      } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int jl = BUF ? 2 * (256 * (u >> 1) + t) + (u & 1)
                           : t + u * SP_THREADS;   // load_short's entry map
        // unconditional (jl < SP_TILE always; products past the block are
        // never read): a store under `jl < nl` put the wait for its gather
        // inside a branch, where the wait-count pass falls back to vmcnt(0)
        // -- draining the next block's stream loads
        if (MR_SP_ORDER || jl < nl) prod[jl] = cur.vv[u] * gx[u];
      }
      const int R = (int)(r1 - r0);
      if (t < R) srp[t] = (int32_t)(cur.ro - n0);
      if (t == 0) srp[R] = (int32_t)(n1 - n0);
      if constexpr (OUT == SPO_CG && MR_SP_PRELOAD && MR_SP_ORDER) {
        if (t < R) spv[t] = rpair;
      }
      __syncthreads();
      int G = 1;
      while (G < 64 && 2 * G * R <= SP_THREADS) G *= 2;
      const int lr = t / G, g = t & (G - 1);
      double sum = 0.0;
      if (lr < R) {
        const int e = srp[lr + 1];
        const int j0 = srp[lr] + g;
        if (j0 + 15 * G >= e) {
          // <= 16 terms: all LDS reads issued first, then the adds in order
          double pv16[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) pv16[i] = (j0 + i * G < e) ? prod[j0 + i * G] : 0.0;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (j0 + i * G < e) sum += pv16[i];
        } else {
          for (int j = j0; j < e; j += G) sum += prod[j];
        }
      }
      for (int o = G / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
      if (lr < R && g == 0) {
        if constexpr (OUT == SPO_CG && MR_SP_PRELOAD && MR_SP_ORDER) emit_cg(r0 + lr, sum, spv[lr]);
        else emit(r0 + lr, sum);
      }
      __syncthreads();   // prod / srp are reused by the next block
      }
    } else {             // one long row: per-thread strided sums, fixed-order tree
      double sum = 0.0;
      for (int64_t j = n0 + t; j < n1; j += SP_THREADS) sum += v[j] * gather(ci[j]);
      sum = block_sum_f64<SP_THREADS>(sum, sh);
      if (t == 0) emit(r0, sum);
      __syncthreads();
    }
    r0 = qr0; r1 = qr1; n0 = qn0; n1 = qn1;
    qr0 = sr0; qr1 = sr1; qn0 = sn0; qn1 = sn1;
    cur = nxt;
  }
  if constexpr ((MR_SP_PROBE & 4) != 0) {
    if (probe_sink == 1.2345e300) out[blockIdx.x] = probe_sink;   // keeps the work alive
  }
  if constexpr (OUT == SPO_CG) {
    const double tot = block_sum_f64<SP_THREADS>(d, sh);
    if (fst) {
      store_partial(partials, tot);
      last_block_finalize(fst, CG_ALPHA, partials, nullptr, 0, sh);
    } else if (t == 0) {
      partials[blockIdx.x] = tot;
    }
  }
}

int launch_csr_spmv(hipStream_t s, int gather, int out_mode, const CgState* st, int64_t n_blk,
                    const int64_t* blk, const int64_t* rp, const int32_t* ci, const double* v,
                    const double* xa, const double* xb, int64_t nx, double* out, double* pv,
                    const double* rv, int update_p, double* partials, int n_part,
                    CgState* fst) {
  if (n_blk <= 0) return 0;
  // at most the workgroups the chip holds at once: a fixed grid larger than
  // that runs a second, partial round of grid-stride loops (general CG at
  // 27e6 x 2.8e6: 2,048 blocks at 5 per CU measured slower than 1,280)
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      return 0;
    return n;
  }();
  const bool buf = nx >= 0 && nx * 8 < (int64_t)0xFFFFFFF0;
  const void* fn = nullptr;
#define MR_SP_FN(GA, OU)                                                                   \
  fn = buf ? (const void*)csr_spmv_kernel<GA, OU, true> : (const void*)csr_spmv_kernel<GA, OU, false>
  if (out_mode == SPO_CG) {
    if (gather != SPG_X) {
      set_error("the CG output pass gathers a plain vector");
      return -1;
    }
    MR_SP_FN(SPG_X, SPO_CG);
  } else {
    if (gather == SPG_P) MR_SP_FN(SPG_P, SPO_STORE);
    else if (gather == SPG_P0) MR_SP_FN(SPG_P0, SPO_STORE);
    else MR_SP_FN(SPG_X, SPO_STORE);
  }
#undef MR_SP_FN
  int bpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, fn, SP_THREADS, 0) != hipSuccess) bpc = 0;
  int64_t parts = n_part;
  if (bpc > 0 && cus > 0) parts = std::min<int64_t>(parts, (int64_t)bpc * cus);
  const dim3 grid((unsigned)std::min<int64_t>(n_blk, parts));
  const uint32_t xbytes = buf ? (uint32_t)(nx * 8) : 0u;
#define MR_SP(GA, OU)                                                                      \
  if (buf)                                                                                  \
    MR_LAUNCH((csr_spmv_kernel<GA, OU, true>), grid, dim3(SP_THREADS), 0, s, st, n_blk, blk, \
              rp, ci, v, xa, xb, xbytes, out, pv, rv, update_p, partials, fst);            \
  else                                                                                      \
    MR_LAUNCH((csr_spmv_kernel<GA, OU, false>), grid, dim3(SP_THREADS), 0, s, st, n_blk,    \
              blk, rp, ci, v, xa, xb, xbytes, out, pv, rv, update_p, partials, fst)
  if (out_mode == SPO_CG) {
    MR_SP(SPG_X, SPO_CG);
  } else {
    if (gather == SPG_P) MR_SP(SPG_P, SPO_STORE);
    else if (gather == SPG_P0) MR_SP(SPG_P0, SPO_STORE);
    else MR_SP(SPG_X, SPO_STORE);
  }
#undef MR_SP
  MR_HIP(hipGetLastError());
  return 0;
}

// K3 (and the INIT update): x += alpha p, r += alpha q (vect_add(1, x, alpha,
// p, x), matrix.cpp:501-503) / r0 = q - b2, p0 = -r0 (:468-476); r.r partials
// (:507 / :485) in a fixed grid; the last workgroup applies the INIT / BETA
// rule and publishes the state.
__global__ __launch_bounds__(256) void cgls_update_kernel(
    const CgState* __restrict__ st, int mode, int64_t n, double* __restrict__ x,
    double2* __restrict__ rp, const double* __restrict__ q,
    const double* __restrict__ b2, double* __restrict__ partials, CgState* fst,
    CgMirror* mirror, int seq) {
#pragma clang fp contract(off)
  if (ald(&st->done)) return;
  __shared__ double sh[4];
  const double alpha = ald(&st->alpha);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double rv, pv;
    if (mode == UPD_INIT) {
      rv = 1.0 * q[i] + -1.0 * b2[i];
      pv = -1.0 * rv;
    } else {
      const double2 w = rp[i];   // (r, p)
      pv = w.y;
      x[i] = 1.0 * x[i] + alpha * pv;
      rv = 1.0 * w.x + alpha * q[i];
    }
    rp[i] = make_double2(rv, pv);
    acc += rv * rv;
  }
  const double tot = block_sum_f64<256>(acc, sh);
  store_partial(partials, tot);
  last_block_finalize(fst, mode == UPD_INIT ? CG_INIT : CG_BETA, partials, mirror, seq, sh);
}

int launch_cgls_update(hipStream_t s, const CgState* st, int mode, int64_t n, double* x,
                       double* rp, const double* q, const double* b2,
                       double* partials, int n_part, CgState* fst, CgMirror* mirror, int seq) {
  MR_LAUNCH(cgls_update_kernel, dim3(n_part), dim3(256), 0, s, st, mode, n, x,
            reinterpret_cast<double2*>(rp), q, b2, partials, fst, mirror, seq);
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

__global__ void gather_i32_kernel(int64_t n, const int64_t* __restrict__ pos,
                                  const int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    dst[t] = src[pos[t]];
}
int launch_gather_i32(hipStream_t s, int64_t n, const int64_t* pos, const int32_t* src,
                      int32_t* dst) {
  if (n <= 0) return 0;
  gather_i32_kernel<<<grid_for(n), 256, 0, s>>>(n, pos, src, dst);
  MR_HIP(hipGetLastError());
  return 0;
}

__global__ void gather_f64_kernel(int64_t n, const int32_t* __restrict__ pos,
                                  const double* __restrict__ src, double* __restrict__ dst) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    dst[t] = src[pos[t]];
}
int launch_gather_f64(hipStream_t s, int64_t n, const int32_t* pos, const double* src,
                      double* dst) {
  if (n <= 0) return 0;
  gather_f64_kernel<<<grid_for(n), 256, 0, s>>>(n, pos, src, dst);
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
