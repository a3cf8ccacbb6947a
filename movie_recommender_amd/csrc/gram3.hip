// Normal equations with bf16 matrix cores at fp32 accuracy ("bf16x3").
//
// Same result as gram_kernel (kernels.hip): per entity G = sum a a^T over its
// ratings, the rhs c = sum a w and (user side) the row sums, written in tri16
// order.  gram_kernel spends ~60 % of its time in v_mfma_f32_16x16x4_f32 (32
// cycles per 4 ratings per 16x16 block, the f32 vector rate).  Here every
// factor is split once per half-step into three bf16 parts a = h + m + l
// (24 significant bits, so the split is exact to fp32 precision), and each
// block accumulates the six products whose weight is >= 2^-16 of h h^T:
//   hh + hm + mh + hl + lh + mm
// with v_mfma_f32_16x16x32_bf16 (16 cycles per 32 ratings), fp32 accumulate.
// The dropped terms (ml, lm, ll) are below 2^-24 relative: fp32-level
// agreement with gram_kernel, which the parity tests check.
//
// Per wave and 32-rating chunk: the gathered rows (pre-split table, virtual
// column order) are transposed through LDS into [part][column][rating] so that
// each lane reads its MFMA operand (8 ratings of one column) as one 16-byte
// LDS read; the rhs / row sums come from an extra 16-column B operand holding
// the weight's parts in column 0 and ones in column 1.  The next chunk's
// gathers are in flight during the current chunk's 84 MFMAs (k = 64).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mr_internal.h"

namespace mr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint16_t bf16_bits(float x) {
  const __bf16 h = (__bf16)x;   // v_cvt_pk_bf16_f32: round to nearest even
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float bf16_float(uint16_t b) {
  return __uint_as_float((uint32_t)b << 16);
}
// a = h + m + l, each part bf16 (exact residuals in fp32)
__device__ __forceinline__ void split3(float a, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = bf16_bits(a);
  const float r1 = a - bf16_float(h);
  m = bf16_bits(r1);
  const float r2 = r1 - bf16_float(m);
  l = bf16_bits(r2);
}

// Fs[row][p][v] = part p of F[row][nat_of(v)] (virtual column order, C = ldk)
__global__ void split_table_kernel(int64_t rows, int nb, int ldk, const float* __restrict__ F,
                                   uint16_t* __restrict__ Fs) {
  const int64_t n = rows * ldk;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / ldk;
    const int v = (int)(e - row * ldk);
    uint16_t h, m, l;
    split3(F[row * ldk + nat_of(v, nb)], h, m, l);
    uint16_t* o = Fs + row * 3 * ldk + v;
    o[0] = h;
    o[ldk] = m;
    o[2 * ldk] = l;
  }
}

int launch_split_table(hipStream_t s, int64_t rows, int k, const float* F, uint16_t* Fs) {
  const int ldk = ldk_of(k);
  const int64_t n = rows * ldk;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
  MR_LAUNCH(split_table_kernel, grid, dim3(256), 0, s, rows, nb16_of(k), ldk, F, Fs);
  MR_HIP(hipGetLastError());
  return 0;
}

bool gram3_supported(int k) {
  const int nb = nb16_of(k);
  return nb == 2 || nb == 4;
}

// LDS image of a chunk: [part][row][32 ratings] bf16, 64-byte rows.  Column c
// lives in row g3_row(c); its four 16-byte slots (8 ratings each) are XORed
// with g3_swz(c).  Both were found by exhaustive search over the gfx950 LDS
// banking of MI355X_MICROARCH.md (ds_write_b64: 4 x 16 contiguous lanes, 32
// banks; ds_write_b32: 2 x 32; ds_read_b128: its 4 interleaved 16-lane groups,
// 64 banks) so that the transposing writes (lane: 4 ratings of one column, 2
// for k <= 32) and the operand reads (lane: 8 ratings of one column) are free
// of bank conflicts.  The plain layout spent ~80 % of its LDS cycles in
// conflicts (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
__device__ __forceinline__ int g3_row(int c) { return c ^ ((c >> 3) & 3) ^ ((c >> 5) & 1); }
__device__ __forceinline__ int g3_swz(int c) {
  const int x = (c >> 3) & 3;
  return x ^ ((x & 1) << 1);
}

template <int NB, bool USER>
__global__ __launch_bounds__(256) void gram3_kernel(
    const WorkItem* __restrict__ work, int64_t n_work, const int32_t* __restrict__ idx,
    const float* __restrict__ val, const uint16_t* __restrict__ Fs,
    const float* __restrict__ bias, int k, int ldk, int zrow, GramDst direct, GramDst slab) {
  constexpr int C = 16 * NB;            // columns (virtual order), == ldk
  constexpr int LPR = 2 * NB;           // lanes per gathered row (8 columns each)
  constexpr int T = NB * (NB + 1) / 2;  // 16x16 blocks of the upper triangle
  constexpr int WPB = 4;
  __shared__ __attribute__((aligned(16))) uint16_t lp[WPB][3][C][32];
  __shared__ __attribute__((aligned(16))) uint16_t lw[WPB][3][16][32];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wi = (int64_t)blockIdx.x * WPB + wid;
  if (wi >= n_work) return;   // waves are independent (own LDS region)
  const int64_t wbeg = work[wi].begin;
  const int wlen = work[wi].len;
  const int went = work[wi].entity;
  const int wslab = work[wi].slab;
  const int64_t end = wbeg + wlen;
  const int nchunks = (wlen + 31) >> 5;
  const int g = lane / LPR, o = lane % LPR;   // this lane gathers rows NB*g .. NB*g+NB-1
  const int q = lane >> 4, col = lane & 15;
  const uint32_t row_elems = 3u * C;
  // LDS element offsets within a part image: transposing writes (column 8o+j,
  // this lane's ratings) and operand reads (column 16b+col, ratings 8q..8q+7)
  int wofs[8], rofs[NB];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = 8 * o + j;
    const int r0 = NB * g;   // first rating of this lane's rows
    wofs[j] = g3_row(c) * 32 + 8 * ((r0 >> 3) ^ g3_swz(c)) + (r0 & 7);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int c = 16 * b + col;
    rofs[b] = g3_row(c) * 32 + 8 * (q ^ g3_swz(c));
  }

  // chunk registers: lanes 0..31 own rating (32c + lane) of chunk c
  auto load_ids = [&](int c, int& id, float& r) {
    const int64_t jj = wbeg + 32 * (int64_t)c + (lane & 31);
    const bool ok = jj < end;
    const int64_t js = ok ? jj : wbeg;
    const int i0 = idx[js];
    const float v0 = val[js];
    id = ok ? i0 : zrow;
    r = ok ? v0 : 0.f;
  };
  // gathered parts: [part][row] 8 bf16 = 16 B
  auto gather = [&](uint4 (&gv)[3][NB], int id_reg) {
#pragma unroll
    for (int rr = 0; rr < NB; ++rr) {
#if defined(MR_GRAM_PROBE) && MR_GRAM_PROBE == 1
      const int ri = __shfl(id_reg, NB * g + rr, 64) & 1023;   // probe: cache-resident rows
#else
      const int ri = __shfl(id_reg, NB * g + rr, 64);
#endif
      const uint16_t* p = Fs + (uint64_t)(uint32_t)ri * row_elems + 8 * o;
#pragma unroll
      for (int pp = 0; pp < 3; ++pp) gv[pp][rr] = *reinterpret_cast<const uint4*>(p + pp * C);
    }
  };

  f32x4 acc[T], accx[NB];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < NB; ++b) accx[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float wsum = 0.f;

  // constant parts of the extra B operand: column 1 = ones (part 0), 2..15 zero
  {
    const uint16_t one = bf16_bits(1.0f);
    for (int e = lane; e < 3 * 16 * 32; e += 64) {
      const int pp = e / 512, cc = (e / 32) & 15;
      lw[wid][pp][cc][e & 31] = (cc == 1 && pp == 0) ? one : (uint16_t)0;
    }
  }
  // lane's extra-operand row: 0 (weights), 1 (ones) or 2 (zeros; broadcast)
  const int xrow0 = (col == 0) ? 0 : (col == 1 ? 1 : 2);
  const int xrow = (col == 0) ? 0 : 2;   // parts 1, 2 have no ones column

  // chunk ring (4 slots): ids / ratings loaded 4 chunks ahead, bias (item
  // side) when the chunk's rows are gathered; rows gathered 2 chunks ahead
  int id0, id1, id2, id3;
  float r0, r1, r2, r3, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  load_ids(0, id0, r0);
  load_ids(1, id1, r1);
  load_ids(2, id2, r2);
  load_ids(3, id3, r3);
  if (!USER) {
    b0 = bias[id0];
    b1 = bias[id1];
  }
  uint4 gA[3][NB], gB[3][NB];
  gather(gA, id0);
  gather(gB, id1);

  auto body = [&](uint4 (&gv)[3][NB], int c, float rc, float bc, int& id_ahead,
                  float& b_ahead, int& id_reload, float& r_reload) {
    // ---- stage chunk c in LDS: rows transposed to [part][column][rating]
#pragma unroll
    for (int pp = 0; pp < 3; ++pp) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(&gv[pp][0]);
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) {
        // column 8o+cc of rows NB*g .. +NB-1: bf16 (cc&1) of dword (cc>>1)
        const uint32_t sel = (cc & 1) ? 0x07060302u : 0x05040100u;
        uint32_t out[NB / 2];
#pragma unroll
        for (int h = 0; h < NB / 2; ++h)
          out[h] = __builtin_amdgcn_perm(w[(2 * h + 1) * 4 + (cc >> 1)],
                                         w[(2 * h) * 4 + (cc >> 1)], sel);
        uint16_t* dst = &lp[wid][pp][0][0] + wofs[cc];
        if constexpr (NB == 4) {
          *reinterpret_cast<uint2*>(dst) = make_uint2(out[0], out[1]);
        } else {
          *reinterpret_cast<uint32_t*>(dst) = out[0];
        }
      }
    }
    const float wgt = rc - bc;   // user side: bc == 0
    if (lane < 32) {
      uint16_t h, m, l;
      split3(wgt, h, m, l);
      lw[wid][0][0][lane] = h;
      lw[wid][1][0][lane] = m;
      lw[wid][2][0][lane] = l;
      if (USER) wsum += wgt;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- operand fragments: 8 ratings of one column per lane
    bf16x8 fr[3][NB], fx[3];
#pragma unroll
    for (int pp = 0; pp < 3; ++pp) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        fr[pp][b] = *reinterpret_cast<const bf16x8*>(&lp[wid][pp][0][0] + rofs[b]);
      fx[pp] = *reinterpret_cast<const bf16x8*>(&lw[wid][pp][pp == 0 ? xrow0 : xrow][8 * q]);
    }
    __builtin_amdgcn_wave_barrier();
    // ---- rows of chunk c+2 into this buffer (in flight under the MFMAs);
    // ids of chunk c+4 into the slot chunk c used
    if (c + 2 < nchunks) {
      if (!USER) b_ahead = bias[id_ahead];
      gather(gv, id_ahead);
    }
    load_ids(c + 4, id_reload, r_reload);
    // ---- 6 products per block pair: hh, hm, mh, hl, lh, mm
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int pa = (s == 0) ? 0 : (s == 1) ? 0 : (s == 2) ? 1 : (s == 3) ? 0 : (s == 4) ? 2 : 1;
      const int pb = (s == 0) ? 0 : (s == 1) ? 1 : (s == 2) ? 0 : (s == 3) ? 2 : (s == 4) ? 0 : 1;
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) {
#pragma unroll
        for (int bj = bi; bj < NB; ++bj) {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[pa][bi], fr[pb][bj], acc[t], 0, 0, 0);
          ++t;
        }
        accx[bi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[pa][bi], fx[pb], accx[bi], 0, 0, 0);
      }
    }
  };
  for (int c = 0; c < nchunks; c += 4) {
    body(gA, c, r0, b0, id2, b2, id0, r0);
    if (c + 1 < nchunks) body(gB, c + 1, r1, b1, id3, b3, id1, r1);
    if (c + 2 < nchunks) body(gA, c + 2, r2, b2, id0, b0, id2, r2);
    if (c + 3 < nchunks) body(gB, c + 3, r3, b3, id1, b1, id3, r3);
  }

  // ---- epilogue (tri16 layout, as gram_kernel)
  const bool to_slab = wslab >= 0;
  const int64_t di = to_slab ? (int64_t)wslab : (int64_t)went;
  const GramDst& D = to_slab ? slab : direct;
  float* __restrict__ Gd = D.G + di * D.sG;
  float* __restrict__ Cd = D.C + di * D.sV;
  if (col == 0 || (USER && col == 1)) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nat_of(16 * b + 4 * q + r, NB);   // natural column, < ldk
        const float v = (n < k) ? accx[b][r] : 0.f;
        if (col == 0) Cd[n] = v;
        else D.Gs[di * D.sV + n] = v;
      }
  }
  if (USER) {
    float wt = wsum;   // lanes >= 32 hold 0
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) wt += __shfl_xor(wt, m, 64);
    if (lane == 0) {
      D.Cb[di * D.sS] = wt;
      D.Gn[di * D.sS] = (float)wlen;
    }
  }
  constexpr int NO = NB * (NB - 1) / 2, NF = NB / 2, NTILE = NO + NF + (NB & 1);
  int t = 0;
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
#pragma unroll
    for (int bj = bi; bj < NB; ++bj) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        const float v = acc[t][r];
        if (bi != bj) {
          Gd[off_index(bi, bj, NB) * 256 + row * 16 + col] = v;
        } else if ((NB & 1) && bi == NB - 1) {
          Gd[(NO + NF) * 256 + row * 16 + col] = v;
        } else if ((bi & 1) == 0) {
          if (col >= row) Gd[(NO + (bi >> 1)) * 256 + row * 16 + col] = v;
        } else {
          if (col < row) Gd[(NO + (bi >> 1)) * 256 + row * 16 + col] = v;
          else if (col == row) Gd[NTILE * 256 + (bi >> 1) * 16 + row] = v;
        }
      }
      ++t;
    }
  }
}

int launch_gram3(hipStream_t s, bool user_side, int k, const WorkItem* work, int64_t n_work,
                 const int32_t* idx, const float* val, const uint16_t* Fs, const float* bias,
                 int zrow, GramDst direct, GramDst slab) {
  if (n_work <= 0) return 0;
  const int64_t grid = (n_work + 3) / 4;
  const int ldk = ldk_of(k);
#define MR_G3(NB, U)                                                                 \
  MR_LAUNCH((gram3_kernel<NB, U>), dim3((unsigned)grid), dim3(256), 0, s, work, n_work, idx, val, Fs, \
                                                                   bias, k, ldk, zrow, direct, slab)
  switch (nb16_of(k)) {
    case 2:
      if (user_side) MR_G3(2, true); else MR_G3(2, false);
      break;
    case 4:
      if (user_side) MR_G3(4, true); else MR_G3(4, false);
      break;
    default:
      set_error("gram3: unsupported k");
      return -1;
  }
#undef MR_G3
  MR_HIP(hipGetLastError());
  return 0;
}

}  // namespace mr
