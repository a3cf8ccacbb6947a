// Internal declarations shared by the HIP kernels and the host engine.
// Target: MI355X (gfx950, CDNA4) only.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <cstdlib>
#include <string>

namespace mr {

// Per-thread launch-timing slot, set by the engine around a timed launcher
// (Engine::tic/toc).  Kernels launched through MR_LAUNCH record the slot's
// events from their own dispatch packets (hipExtLaunchKernel): the first
// launch takes the start event, every launch the stop event.  No marker
// packets go between kernels, so timing does not add gaps to the stream.
struct LaunchTiming {
  hipEvent_t start = nullptr;
  hipEvent_t stop = nullptr;
};
extern thread_local LaunchTiming t_launch;

// Untimed launches (no slot events) take the plain launch path.
#define MR_LAUNCH(kernel, grid, block, shm, s, ...)                                  \
  do {                                                                               \
    hipEvent_t mr_ev0_ = ::mr::t_launch.start;                                       \
    ::mr::t_launch.start = nullptr;                                                  \
    if (mr_ev0_ || ::mr::t_launch.stop)                                              \
      hipExtLaunchKernelGGL(kernel, grid, block, shm, s, mr_ev0_, ::mr::t_launch.stop, \
                            0, __VA_ARGS__);                                         \
    else                                                                             \
      hipLaunchKernelGGL(kernel, grid, block, shm, s, __VA_ARGS__);                  \
  } while (0)

// Error handling --------------------------------------------------------------
void set_error(const std::string& msg);
const char* last_error();

#define MR_HIP(call)                                                          \
  do {                                                                        \
    hipError_t _e = (call);                                                   \
    if (_e != hipSuccess) {                                                   \
      ::mr::set_error(std::string(#call) + ": " + hipGetErrorString(_e) +    \
                      " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")"); \
      return -1;                                                              \
    }                                                                         \
  } while (0)

#define MR_CHECK(cond, msg)                                                   \
  do {                                                                        \
    if (!(cond)) {                                                            \
      ::mr::set_error(msg);                                                   \
      return -1;                                                              \
    }                                                                         \
  } while (0)

// Host <-> device copies through two pinned chunks (xfer.hip), stream-ordered
// on s; both return with their copies complete.  Caller buffers are never
// handed to the DMA engine as pageable memory.
struct Stager {
  static constexpr size_t kChunk = size_t(16) << 20;
  void* buf[2] = {nullptr, nullptr};
  ~Stager();
  int init();
  int h2d(hipStream_t s, void* dst, const void* src, size_t bytes);
  int d2h(hipStream_t s, void* dst, const void* src, size_t bytes);
};
extern thread_local Stager t_stager;

#define MR_H2D(dst, src, bytes, s)                                         \
  do {                                                                     \
    if (::mr::t_stager.h2d((s), (dst), (src), (size_t)(bytes))) return -1; \
  } while (0)
#define MR_D2H(dst, src, bytes, s)                                         \
  do {                                                                     \
    if (::mr::t_stager.d2h((s), (dst), (src), (size_t)(bytes))) return -1; \
  } while (0)

constexpr int kMaxK = 128;        // largest k of the register-tiled (MFMA) Gram and GEMV kernels
constexpr int kMaxKLarge = 512;   // k > 128: streamed large-k kernels (gram_largek_kernel, ...)
constexpr int kMfmaMinK = 32;     // k < 32: VALU Gram (gram_valu_kernel), no fused CG start
// Row stride of factor tables / CG vectors: k rounded up to a multiple of 16
// (one 16-wide block of the tri16 storage), so every Gram lane's NB-float segment of a row
// lies inside the row; padding columns are kept at zero.
__host__ __device__ inline int ldk_of(int k) { return (k + 15) & ~15; }

// Normal-equation storage ("tri16").  G_e, over the permuted ("virtual")
// factor index below, is cut into NB x NB blocks of 16 x 16 (NB = ceil(k/16)):
//   * the NB(NB-1)/2 strictly-upper blocks (bi < bj) as full tiles, row-major
//     inside, row-major upper order;
//   * the diagonal blocks folded in pairs (2m, 2m+1) into ONE tile F_m:
//     F_m[r][c] = D_2m[r][c] for c >= r, D_2m+1[r][c] for c < r, and the
//     diagonal of D_2m+1 in a 16-float side array; an odd last diagonal
//     block is stored full but only its upper triangle is G.  The bf16x3 MFMA
//     sums are NOT bitwise symmetric (B[i][j] and B[j][i] add the hm / mh
//     products in opposite orders), so every reader -- GEMV, fused CG start,
//     Cholesky, read-back -- takes each diagonal entry pair from the one
//     stored triangle: G is exactly symmetric.
// k = 64: 8 tiles + 32 floats = 2,080 floats = k(k+1)/2 (full: 4,096).
// Rows/cols >= k are zero.
__host__ __device__ inline int nb16_of(int k) { return (k + 15) / 16; }
__host__ __device__ inline int n_off_of(int nb) { return nb * (nb - 1) / 2; }
__host__ __device__ inline int n_fold_of(int nb) { return nb / 2; }
__host__ __device__ inline int n_tiles_of(int nb) { return n_off_of(nb) + nb / 2 + (nb & 1); }
__host__ __device__ inline int64_t gsize_of(int k) {
  const int nb = nb16_of(k);
  return (int64_t)n_tiles_of(nb) * 256 + n_fold_of(nb) * 16;
}
// strictly-upper tile (bi < bj)
__host__ __device__ inline int off_index(int bi, int bj, int nb) {
  return bi * nb - bi * (bi + 1) / 2 + (bj - bi - 1);
}
// Blocks are formed over a permuted ("virtual") factor index so that every
// lane of the Gram kernel gathers NB contiguous floats of a row (one dwordx4
// for k = 64): virtual v = 16*b + i  <->  natural n = NB*i + b.
__host__ __device__ inline int virt_of(int n, int nb) { return 16 * (n % nb) + n / nb; }
__host__ __device__ inline int nat_of(int v, int nb) { return nb * (v & 15) + (v >> 4); }
// Offset of natural element (i, j) of a tri16 G_e.
__host__ __device__ inline int64_t packed_offset(int i, int j, int nb) {
  int vi = virt_of(i, nb), vj = virt_of(j, nb);
  if ((vi >> 4) > (vj >> 4) || ((vi >> 4) == (vj >> 4) && (vi & 15) > (vj & 15))) {
    const int t = vi; vi = vj; vj = t;      // symmetric: use (min, max)
  }
  const int bi = vi >> 4, bj = vj >> 4, ri = vi & 15, rj = vj & 15;   // ri <= rj if bi == bj
  if (bi != bj) return (int64_t)off_index(bi, bj, nb) * 256 + ri * 16 + rj;
  const int base = n_off_of(nb);
  if ((nb & 1) && bi == nb - 1) return (int64_t)(base + n_fold_of(nb)) * 256 + ri * 16 + rj;
  const int m = bi >> 1;
  if ((bi & 1) == 0) return (int64_t)(base + m) * 256 + ri * 16 + rj;       // upper incl. diag
  if (ri == rj) return (int64_t)n_tiles_of(nb) * 256 + m * 16 + ri;         // side array
  return (int64_t)(base + m) * 256 + rj * 16 + ri;                          // strict lower
}

// One wave's unit of Gram work: ratings [begin, begin+len) of one entity's
// CSR row; slab >= 0 writes a partial record to be combined by slab_reduce.
struct WorkItem {
  int64_t begin;
  int32_t len;
  int32_t entity;   // local entity index
  int32_t slab;     // -1: write the entity's normal equations directly
  int32_t pad;
};

// Split entity: partial records [slab0, slab0+nslab) sum into `entity`.
struct SplitItem {
  int32_t entity;
  int32_t slab0;
  int32_t nslab;
  int32_t pad;
};

// Destination of normal equations: entity / slab i writes
//   G  + i*sG  (tri16 tiles)     Gs + i*sV (sum of rows, user side)
//   C  + i*sV  (rhs)            Cb + i*sS (sum of ratings, user side)
//   Gn + i*sS  (rating count, user side)
struct GramDst {
  float* G;
  float* Gs;
  float* C;
  float* Cb;
  float* Gn;
  int64_t sG, sV, sS;
};

// Fused CG start (Gram epilogue): the iterate and the CG vectors of one side,
// and the (r.r, p.Gp) pair slots, one pair per Gram block then one per
// split-start block.
struct CgStart {
  const float* x;    // this side's iterate (local rows), ldk stride
  const float* xb;   // user side: bias column of the iterate
  double *r, *rb, *p, *pb, *q, *qb;   // fp64 CG vectors
  double* parts;
  // one-pass CG: the start's (r.r, p.Gp, q.q) as order-independent sums in
  // these kXBins x 3 x 11 int64 bins instead of per-block parts (nullptr:
  // the parts); read and reset by the CG_START control
  int64_t* xbins;
};

// Peer all-reduce of the CG scalars over IPC-mapped device memory (sharded
// runs; Engine::set_peer).  Every rank owns an exchange buffer of
// kPeerSlots x world records {v0 .. v62, tag} in uncached device memory and
// maps every peer's.  Reduction s writes this rank's values into record
// (s % kPeerSlots, rank) of EVERY rank's buffer, then the tag s (release,
// system scope); each rank then waits for the tag of every record of its own
// buffer and sums the values in rank order -- so all ranks get the same bits.
constexpr int kPeerSlots = 16;
constexpr int kPeerRec = 64;   // 8-byte words per record: up to 63 values, then the tag
constexpr int kMaxPeers = 64;
struct PeerComm {
  int32_t world, rank;
  uint32_t seq;            // reductions done (advanced by the reducing thread)
  int32_t error;           // 1: a peer did not arrive within the timeout
  uint64_t timeout_ticks;  // give up on a peer after this many s_memrealtime
                           // ticks (100 MHz; MR_OPT_PEER_TIMEOUT_S)
  double* buf[kMaxPeers];  // rank q's exchange buffer, mapped into this process
  // accounting (mr_stats peer_wait_ms / peer_reductions): s_memrealtime
  // ticks the reducing thread spent inside reductions, and their number
  uint64_t wait_ticks, n_reduce;
};

// One peer reduction of {rank + 1, 1} into out[0..2] = {sum, count, ok}.
int launch_peer_selftest(hipStream_t s, PeerComm* pc, double* out);
// Test hook: the order-independent sum (kernels.hip xterm / xsum_value) of
// n terms over `blocks` blocks; bins: 16 x 1 x 11 int64 zeros (left zero).
int launch_xsum_test(hipStream_t s, const double* t, int64_t n, int blocks, int64_t* bins,
                     double* out);
// `iters` reductions of one value back to back; out = {ok, iters done}.
int launch_peer_bench(hipStream_t s, PeerComm* pc, int iters, double* out);

// CG scalar state, device resident (matrix.cpp:456-529 scalars).
struct CgState {
  double rr;        // r.r of the current iterate
  double alpha;
  double beta;
  double final_rr;
  double min_dec;   // min_r_decrease
  double comm[3];   // local sums exchanged by all-reduce in sharded runs
  int32_t it;       // iteration counter
  int32_t fails;    // consecutive beta > 1 - min_dec
  int32_t done;     // solve finished: every later kernel is a no-op
  int32_t ret;      // iteration count returned by cg_least_squares
  int32_t max_it;
  int32_t n_matvec; // matvec launches that did work (for kernel timing)
  uint32_t arrive;  // blocks finished (fused control: the last one finalizes)
  int32_t sharded;  // 1: the last block only sums into comm[0] for the all-reduce
  PeerComm* peer;   // non-null: the finalizing thread all-reduces its sum with
                    // the peers itself (no collective launches; rules as unsharded)
  int32_t onepass;  // one kernel per CG iteration (cg_matvec_kernel, DESIGN.md
                    // "One-pass CG iteration"); set by the host per solve
  int32_t pending;  // one-pass: the last iteration's x / r update is not applied yet
  uint32_t arrive_start;  // cg_start_split blocks finished (folded CG_START control)
  // resident CG solve (cg_resident_kernel): the last block's per-iteration
  // broadcast to every block, written and read with sc1 (write-through)
  // accesses; res_done 1: stopped, 2: failed
  double res_alpha, res_beta;
  int32_t res_done;
};
// Generation words of the resident CG's per-iteration broadcast: 16 copies
// on lines of their own (block b polls copy b mod 16), each bumped by the
// last block to (seq << 32) | (t + 1) after iteration t.
constexpr int kResGenCopies = 16;
constexpr int kResGenStride = 16;   // uint64 words: 128 B per copy
constexpr int kResGenWords = kResGenCopies * kResGenStride;
// The CG_START control folded into cg_start_split's last block (one-pass
// solves with split entities): st == nullptr keeps the separate control launch.
struct CgMirror;
struct StartFold {
  CgState* st;
  CgMirror* mirror;
  int seq;
  double min_dec;
  int max_it;
  int sharded;   // cg_control's `sharded` argument (bit 1: one-pass)
};

// Host-visible copies of the CG state: a ring of kMirrorSlots records in
// pinned, host-mapped coherent memory.  Every INIT / BETA step publishes its
// state under a sequence number into slot seq % kMirrorSlots (seqlock: odd
// while being written), so the host reads the state of an EXACT iteration --
// what makes launch decisions identical on every rank of a sharded run.
constexpr int kMirrorSlots = 32;
struct CgMirror {
  int32_t seq;
  int32_t done;
  int32_t fails;
  int32_t it;
  int32_t ret;
  int32_t n_matvec;
  double rr;
  double final_rr;
};

// CG_START: INIT then ALPHA on a fused start's (r.r, p.Gp) pair sums; the
// control kernel also (re)initialises the state from its arguments.
enum CgPhase { CG_INIT = 0, CG_ALPHA = 1, CG_BETA = 2, CG_START = 3 };
enum CgCtl { CTL_REDUCE = 1, CTL_FINALIZE = 2, CTL_BOTH = 3 };
enum CgUpd { UPD_INIT = 0, UPD_STEP = 1, UPD_FINISH = 2 };

// Kernel launchers (kernels.hip) ---------------------------------------------
// F has zrow+1 rows; row zrow (and bias[zrow]) is all zero.
// start != nullptr: every wave also starts the CG solve on its (unsplit)
// entity -- r0 = Gx - c, p0 = -r0, q0 = G p0 -- and each block stores its
// (r.r, p.Gp, q.q) triple to start->parts[3 * block]; split entities follow
// with launch_cg_start_split after slab_reduce (triples after the Gram
// blocks').  rhs_mfma (user side, MFMA Gram): every weight is exact in bf16,
// so the rhs is taken by the matrix cores with the row sums (gram_wave).
int launch_gram(hipStream_t s, bool user_side, int k, const WorkItem* work,
                int64_t n_work, const int32_t* idx, const float* val,
                const float* F, const float* bias, int zrow, GramDst direct,
                GramDst slab, const CgStart* start = nullptr, bool rhs_mfma = false);
// Gram blocks of a launch over n_work work items: four one-wave items per
// block, or (k = 113 ... 128, MR_GRAM_PAIR) one item per pair-of-waves block
#ifndef MR_GRAM_PAIR
#define MR_GRAM_PAIR 1
#endif
inline bool gram_pair_of(int k) { return MR_GRAM_PAIR && k > 112 && k <= 128; }
// waves (one work item each) per block of the one-wave Gram kernels
#ifndef MR_GRAM_WAVES
#define MR_GRAM_WAVES 4
#endif
constexpr int GRAM_WAVES = MR_GRAM_WAVES;
inline int64_t gram_blocks(int64_t n_work, int k) {
  return gram_pair_of(k) ? n_work : (n_work + GRAM_WAVES - 1) / GRAM_WAVES;
}
int launch_cg_start_split(hipStream_t s, bool user_side, int k, const SplitItem* split,
                          int64_t n_split, GramDst direct, const CgStart& cs, double* parts,
                          const StartFold& fold = StartFold{});
int launch_slab_reduce(hipStream_t s, bool user_side, int k,
                       const SplitItem* split, int64_t n_split,
                       const float* slab, int64_t rec, GramDst direct);
// Fused control (single-GPU runs): fst != nullptr makes the last block of
// the matvec compute alpha (phase CG_ALPHA) and the last block of the update
// apply the INIT / BETA rules and publish to `mirror` -- no control kernels.
// Sharded runs: beta_seq > 0 makes the matvec first apply the previous
// iteration's BETA rule (all-reduced r.r in comm[0]) and its last block
// publish that state under beta_seq (no finalize launch).
int launch_cg_matvec(hipStream_t s, bool user_side, const CgState* st,
                     int update_p, int64_t E, int k, const float* G,
                     const float* Gs, const float* Gn, double* v, double* vb,
                     const double* r, const double* rb, double* y, double* yb,
                     double* partials, int n_part, CgState* fst = nullptr,
                     int phase = CG_INIT, CgMirror* mirror = nullptr, int beta_seq = 0);
// One-pass CG iteration (kernels.hip cg_onepass_kernel): the previous
// iteration's deferred x / r update (update != 0), p = -r + beta p, q = G p,
// p.q / r.q / q.q partials (3 x n_part doubles in partials) and, in the last
// block, alpha, r'.r', the BETA rule and the publish under `seq`.  k <= 128.
// Blocks of cg_onepass_kernel one CU holds at once for this side and k (0:
// unknown); the one-pass grid is that times the CU count.
int onepass_blocks_per_cu(bool user_side, int k, bool nt);
// diagnostic timeline of the last one-pass launch (MR_OP_PROF builds; 0 otherwise)
int op_prof_read(int64_t* out, int n);
int launch_cg_onepass(hipStream_t s, bool user_side, CgState* st, int update, int rev, int64_t E, int k,
                      const float* G, const float* Gs, const float* Gn, double* p, double* pb,
                      double* r, double* rb, double* q, double* qb, float* x, float* xb,
                      int64_t* xbins, int n_part, CgMirror* mirror, int seq, bool nt);
// Resident CG solve (kernels.hip cg_resident_kernel): every iteration of
// one solve in one launch, from iteration t0 (0: unfused start, 1: after a
// fused start) until the stop; publishes the final state under `seq` and
// applies the pending x update.  Needs every block of the grid resident at
// once: n_part = resident_blocks_per_cu(...) x CUs at most.  ctl->gen:
// kResGenWords uint64 (any content except a value (seq << 32) | t of this
// launch).  ctl->timeout_ticks: a block whose broadcast does not come gives
// up (the host's wait then reports the unpublished state).
struct ResCtl {   // device memory, written by the engine (Engine::write_res_ctl)
  CgState* st;
  int64_t* xbins;         // kXBinWords bins of the iteration sums
  uint64_t* gen;          // kResGenWords generation words
  CgMirror* mirror;       // host-mapped ring the final state is published into
  uint64_t timeout_ticks; // s_memrealtime ticks (100 MHz) a block waits for a broadcast
};
int resident_blocks_per_cu(bool user_side, int k, bool nt);
int launch_cg_resident(hipStream_t s, bool user_side, const ResCtl* ctl, int t0, int sweep,
                       int64_t E, int k, const float* G, const float* Gs, const float* Gn, double* p,
                       double* pb, double* r, double* rb, double* q, double* qb, float* x,
                       float* xb, int n_part, int seq, bool nt);
// x is the fp32 factor table (and bias), r / p / q the fp64 CG vectors;
// nt: non-temporal G tile loads (Engine::tile_nt_for);
// xbins: kXBins x 4 x 11 int64 bins of the order-independent sums (zero
// between launches: the last block reads and resets them).
constexpr int kXBinWords = 16 * 4 * 11;       // kXBins x sums x (kXD + 1), kernels.hip
constexpr int kXBinStartWords = 16 * 3 * 11;  // the fused start's three sums
// mode UPD_FINISH: apply a one-pass solve's pending last update (no sums).
int launch_cg_update(hipStream_t s, const CgState* st, int mode, int64_t n,
                     int64_t nb, float* x, double* r, double* p, const double* q,
                     const float* c, float* xb, double* rb, double* pb,
                     const double* qb, const float* cb, double* partials,
                     int n_part, CgState* fst = nullptr, CgMirror* mirror = nullptr,
                     int seq = 0);
// v[0..n) = x, vb[0..nb) = xb as fp64 (unfused CG start).
int launch_x_to_vec(hipStream_t s, int64_t n, int64_t nb, const float* x, const float* xb,
                    double* v, double* vb);
// phase CG_START: partials are n_part (r.r, p.Gp) pairs; min_dec / max_it /
// sharded initialise the state.
int launch_cg_control(hipStream_t s, CgState* st, int phase, int ctl,
                      const double* partials, int n_part, CgMirror* mirror = nullptr,
                      int seq = 0, double min_dec = 0.0, int max_it = 0, int sharded = 0,
                      int64_t* start_xbins = nullptr);
int launch_solve(hipStream_t s, bool user_side, int64_t E, int k, double ridge,
                 const float* G, const float* Gs, const float* Gn,
                 const float* C, const float* Cb, float* x, float* xb,
                 int* nonpd);
int launch_unpack_factors(hipStream_t s, int64_t rows, int width, int k,
                          int ldk, const double* src, float* fac, float* bias);
int launch_pack_factors(hipStream_t s, int64_t rows, int width, int k, int ldk,
                        const float* fac, const float* bias, double* dst);
// Sharded all-gather staging: pack rows [r0, r0+n) of fac (and bias) into
// send (bias at send_b); unstage the world gathered blocks -- each
// ag_block_floats(maxrows, ldk, bias != null) floats: maxrows x ldk factors,
// then the bias column padded to 4 -- into their table rows (rb[s] ..
// rb[s+1]) for every rank s != skip.
int64_t ag_block_floats(int64_t maxrows, int ldk, bool with_bias);
int launch_pack_rows(hipStream_t s, int64_t r0, int64_t n, int ldk, const float* fac,
                     const float* bias, float* send, float* send_b);
int launch_unstage_rows(hipStream_t s, int world, int skip, const int64_t* rb,
                        int64_t maxrows, int ldk, const float* recv, float* fac, float* bias);
// Seeded uniform(-1, 1) factor table on the device (table 0: U with bias,
// 1: V); the same values on every rank.
int launch_init_factors(hipStream_t s, int64_t rows, int k, int ldk, uint64_t seed, int table,
                        float* fac, float* bias);
int launch_predict(hipStream_t s, int64_t n, int k, int ldk, const int* uid,
                   const int* iid, const float* Ufac, const float* Ubias,
                   const float* Vfac, double* out);
// General CSR (fp64) CG least squares (cg_least_squares_from_python):
// CSR-stream SpMV over row blocks b = 0..n_blk-1 (consecutive rows with
// <= 2048 non-zeros, <= 256 rows, or one longer row; blk[2b] = first row,
// blk[2b+1] = its first non-zero, n_blk + 1 pairs), fixed grid of
// min(n_blk, n_part) workgroups.  The CG's r and p live interleaved, rp[2j]
// = r_j, rp[2j+1] = p_j (one 16-byte gather per non-zero).  gather SPG_X:
// x_c = xa[c]; SPG_P: p_c = -r_c + beta p_c from xa = rp; SPG_P0: p_c from
// xa = rp.  out SPO_STORE: out[row] = sum; SPO_CG: out[row] = q_row, p_row
// updated in pv = rp (update_p) and p.q summed, the last workgroup computes
// alpha (fst, partials[n_part]).  nx: doubles in the gathered array.
enum SpGather { SPG_X = 0, SPG_P = 1, SPG_P0 = 2 };
enum SpOut { SPO_STORE = 0, SPO_CG = 1 };
constexpr int kSpTile = 2048;
constexpr int kSpPad = 16;   // entries past nnz every SpMV id / value array holds
constexpr int kSpMaxRows = 256;
int launch_csr_spmv(hipStream_t s, int gather, int out_mode, const CgState* st, int64_t n_blk,
                    const int64_t* blk, const int64_t* rp, const int32_t* ci, const double* v,
                    const double* xa, const double* xb, int64_t nx, double* out, double* pv,
                    const double* rv, int update_p, double* partials, int n_part,
                    CgState* fst);   // nx: length of the gathered vector(s) xa / xb
int launch_cgls_update(hipStream_t s, const CgState* st, int mode, int64_t n, double* x,
                       double* rp, const double* q, const double* b2,
                       double* partials, int n_part, CgState* fst, CgMirror* mirror, int seq);
int launch_rows_of(hipStream_t s, int64_t rows, const int64_t* rp,
                   int32_t* row_of);
int launch_i32_to_i64(hipStream_t s, int64_t n, const int32_t* in, int64_t* out);
// dst[t] = src[pos[t]] (t < n)
int launch_gather_i32(hipStream_t s, int64_t n, const int64_t* pos, const int32_t* src,
                      int32_t* dst);
// dst[t] = src[pos[t]] (t < n), fp64
int launch_gather_f64(hipStream_t s, int64_t n, const int32_t* pos, const double* src,
                      double* dst);
int launch_validate_ids(hipStream_t s, int64_t n, const int32_t* ids, int32_t lo,
                        int32_t hi, int* bad);

// CSR construction (csr_build.hip) ------------------------------------------
// Stable sort of n (key, other, value) triples by key - key_base, which must
// lie in [0, E).  Produces off[E+1] (int64), idx[n] = other, val[n] (as TV).
template <typename TV, typename TIn>
int build_csr(hipStream_t s, int64_t n, int64_t E, const int32_t* d_key,
              int32_t key_base, const int32_t* d_other, const TIn* d_val, int64_t* off,
              int32_t* idx, TV* val);

// Rows of a CSR matrix stably sorted by first column (empty rows last):
// perm[i] = original row of new row i; (rp2, ci2, v2) = the matrix in that
// row order (rp2 has rows + 1 entries).
int sort_rows_by_first_col(hipStream_t s, int64_t rows, int64_t cols, const int64_t* rp,
                           const int32_t* ci, const double* v, int32_t* perm, int64_t* rp2,
                           int32_t* ci2, double* v2);

}  // namespace mr
