// Host engine state for one device-resident ALS context (see engine.hip).
#pragma once
#include <vector>

#include "../../include/mr_als.h"
#include "mr_internal.h"

namespace mr {

constexpr int kMaxParts = 2048;   // partial-sum slots (fixed grids)
constexpr int kUpdParts = 1024;   // grid of the CG update kernels

// One side of the bipartite problem: its entities' CSR rows, work list,
// normal equations and CG vectors.  Users: K = k+1 (bias in Gs/Gn/Cb and the
// *b vectors); items: K = k.
struct Side {
  bool user = false;
  int64_t E = 0, e0 = 0, nnz = 0;
  int64_t* off = nullptr;
  int32_t* idx = nullptr;
  float* val = nullptr;
  WorkItem* work = nullptr;
  int64_t n_work = 0;
  SplitItem* split = nullptr;
  int64_t n_split = 0;
  float* slab = nullptr;
  int64_t n_slab = 0, rec = 0;
  float *G = nullptr, *Gs = nullptr, *Gn = nullptr, *C = nullptr, *Cb = nullptr;
  double *r = nullptr, *p = nullptr, *q = nullptr;     // fp64 CG vectors [E][ldk]
  double *rb = nullptr, *pb = nullptr, *qb = nullptr;  // user side: bias entries [E]
  int n_part_mv = 1;
  int n_part_op[2] = {1, 1};   // one-pass CG kernel grid (resident blocks) per tile
                               // cache policy: [0] plain loads, [1] non-temporal
  int n_part_rs[2] = {0, 0};   // resident CG solve grid (0: not available)
  double* start_parts = nullptr;   // fused CG start: (r.r, p.Gp) per block
  int64_t n_start_pairs = 0;
};

// All-gather staging of one factor table (sharded runs, RCCL).
struct AgStage {
  int64_t maxrows = 0;                  // rows of the largest shard
  int64_t per = 0;                      // floats per rank block (ag_block_floats)
  float *send = nullptr, *recv = nullptr;       // one block, world blocks
  int64_t* rb = nullptr;                // device copy of the world+1 row boundaries
};

struct Pending {
  int cls, tag;
  hipEvent_t a, b;
  int n_real;   // CG launches with tag >= n_real ran after the solve ended
  long long units = 1;   // work units (resident solve: its CG iterations)
};

// A resident CG solve launched but not yet read back (Engine::iterate keeps
// up to kMaxInflight of them on the stream: the host never leaves the GPU
// idle while it waits for a solve's published state).
struct Inflight {
  int seq;          // mirror sequence number of its final state
  bool user;
  bool started;     // fused start: iteration 0's matvec ran in the Gram
  long long pend;   // its timing entry in `pending` (-1: not timed)
};
constexpr size_t kMaxInflight = 2;

// One timed phase (Gram or solve of a half-step): pending entries
// [first, last) plus, in sharded runs, a marker after the RCCL exchange.
struct PhaseSpan {
  int phase;
  size_t first, last;
  hipEvent_t end;
};

struct Engine {
  int device = 0;
  hipStream_t stream = nullptr;
  int k = 0, ldk = 0;
  int64_t U = 0, I = 0, N = 0;
  float *Ufac = nullptr, *Ubias = nullptr, *Vfac = nullptr;
  Side su, si;
  CgState* d_state = nullptr;
  CgState* h_state = nullptr;
  CgState* h_init = nullptr;
  double* h_stage = nullptr;
  double* h_fac = nullptr;   // pinned factor staging (set/get_factors)
  int64_t h_fac_n = 0;
  CgMirror* h_mirror = nullptr;   // pinned, host-mapped, coherent
  CgMirror* d_mirror = nullptr;   // its device address
  int mirror_seq = 0;
  double* partials = nullptr;
  // bins of the one-pass CG's order-independent sums: kXBinWords for the
  // iteration kernel, then 16 x 3 x 11 for the fused start (kernels.hip)
  int64_t* xbins = nullptr;
  int* d_flag = nullptr;
  int cur_parts = 1;
  int solver = MR_SOLVER_CG;
  double ridge = 0.0;
  int chunk = 2048;
  bool fuse_start = true;   // CG start in the Gram epilogue (MR_OPT_FUSE_START)
  bool onepass = true;      // one kernel per CG iteration (MR_OPT_CG_ONEPASS)
  bool resident = true;     // one-pass solves as one resident launch (MR_OPT_CG_RESIDENT)
  uint64_t* d_resgen = nullptr;   // the resident solve's generation words
  ResCtl* d_resctl = nullptr;     // its control block (write_res_ctl)
  int write_res_ctl();
  bool rhs_mfma = true;     // user-side rhs on the matrix cores (MR_OPT_GRAM_RHS_MFMA)
  int sweep = 1;            // one-pass sweep direction per iteration (MR_OPT_CG_SWEEP)
  int tile_nt = -1;         // one-pass G tile loads: -1 by size, 0 default policy, 1
                            // non-temporal (MR_OPT_CG_TILE_NT)
  bool w_bf16 = false;      // every user-view rating is exact in bf16 (set by init)
  int speculate = 1;        // 0: never enqueue ahead; 1: enqueue t+2 while t+1 runs when
                            // state t proves t+1 cannot stop; 2: always one ahead
                            // when t provably cannot stop (MR_OPT_CG_SPECULATE;
                            // decided on exact published states, so every rank
                            // of a sharded run issues the same launches)
  double wait_timeout_s = 300.0;   // host wait for a published CG state
  double peer_timeout_s = 30.0;    // device wait for a peer's record (peer all-reduce)
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<Pending> pending;
  std::vector<PhaseSpan> spans;
  std::vector<Inflight> inflight;   // deferred resident solves, oldest first
  bool defer = false;               // half_step may leave its solve in flight
  mr_stats stats{};
  // sharded runs: native RCCL communicator (ncclComm_t) or host callbacks
  void* rccl = nullptr;
  int rccl_world = 1, rccl_rank = 0;
  bool has_comm = false;
  mr_comm comm{};
  std::vector<long long> row_begin_u, row_begin_i;
  AgStage ag_u, ag_i;
  std::vector<float> h_ag;   // host staging of the padded exchange (callback transport)
  // peer all-reduce of the CG scalars (include/mr_als.h mr_als_set_peer)
  double* peer_buf = nullptr;            // this rank's exchange buffer (uncached)
  PeerComm* d_peer = nullptr;
  std::vector<void*> peer_opened;        // peers' buffers mapped by IPC
  bool peer_on = false;
  bool peer_used = false;                // set_peer ran (it runs once per context)
  uint64_t peer_ticks0 = 0, peer_n0 = 0;  // PeerComm accounting at the last stats reset
  int peer_account(double* wait_ms, long long* n, bool reset);

  ~Engine();
  int init(int dev, int k, int64_t U, int64_t I, int64_t n_u, const int* uv_uid,
           const int* uv_iid, const double* uv_r, int64_t n_i, const int* iv_uid,
           const int* iv_iid, const double* iv_r, int64_t u0, int64_t u1, int64_t i0,
           int64_t i1);
  int build_work_xcd(Side& S, const std::vector<int64_t>& off, int64_t chunk,
                     std::vector<WorkItem>& work, std::vector<SplitItem>& split,
                     int32_t& nslab, bool& applied);
  int build_side(Side& S, bool user, int64_t n, const int32_t* d_key,
                 const int32_t* d_other, const double* d_r);
  int set_factors(const double* hU, const double* hV);
  int get_factors(double* hU, double* hV);
  int fac_stage(int64_t n);
  // RCCL attached (any world size, so the collective path is exercised even
  // single-rank) or host callbacks with more than one rank.
  bool sharded() const { return rccl != nullptr || (has_comm && comm.world > 1); }
  int set_rccl(const unsigned char* id, int rank, int world);
  int peer_handle(unsigned char* out64);
  int set_peer(const unsigned char* handles, int rank, int world);
  int set_peer_timeout(double seconds);
  bool tile_nt_for(const Side& S) const;
  int weights_bf16(int force);
  int peer_selftest();
  int peer_latency(int iters, double* us);
  // padded all-gather staging (both transports): every shard padded to the
  // largest one; needs row_begin_u / row_begin_i
  int alloc_ag(int world);
  int ag_world() const { return rccl ? rccl_world : comm.world; }
  int ag_rank() const { return rccl ? rccl_rank : comm.rank; }
  int allreduce_state_slot(int count = 1);
  int allgather_side(bool user);
  int allgather_rows_side(bool user);
  int finalize_sharded(int phase, int seq);
  int wait_mirror(int target, CgMirror* out);
  GramDst direct_dst(Side& S);
  GramDst slab_dst(Side& S);
  int gram(Side& S, bool start = false);
  int x_ptrs(Side& S, float** xf, float** xb);
  int cg(Side& S, double min_dec, int max_it, double* final_rr, bool started = false,
         Inflight* deferred = nullptr);
  // the one-pass CG iteration runs this side's solve (Engine::cg)
  bool onepass_for(const Side& S) const;
  // the resident launch runs this side's one-pass solve
  bool resident_for(const Side& S) const;
  int cg_onepass(Side& S, double min_dec, int max_it, double* final_rr, bool started,
                 Inflight* deferred = nullptr);
  CgStart cg_start_of(Side& S);
  int solve(Side& S);
  int half_step(bool user, double min_dec, int max_it, double* final_rr);
  // read back the deferred solves until at most `keep` remain in flight:
  // their CG counts into the stats, errors reported here
  int drain(size_t keep = 0);
  void count_solve(bool user, int its, double rr);
  int run(double min_dec, int max_it);
  int iterate(int n);
  int predict(int64_t n, const int* uid, const int* iid, double* out);
  int get_normal_equations(bool user, int n, const int* ents, double* G, double* c);
  int get_cg_vectors(bool user, double* r, double* p, double* q);
  int get_layout(bool user, long long* off, int* idx, float* val, long long* wbegin,
                 int* wlen, int* went, int* wslab);
  // timing
  int ev_get(hipEvent_t* e);
  int tic(int cls, int tag, hipEvent_t* a);
  int toc(int cls, int tag, hipEvent_t a);
  int resolve_timing();
};

// Spin on slot target % kMirrorSlots of a host-mapped seqlock ring until the
// state published under sequence number `target` is there (Engine::cg,
// CgLs::solve); checks `stream` for errors / idleness, gives up after
// timeout_s.
int wait_published(CgMirror* ring, int target, hipStream_t stream, double timeout_s,
                   CgMirror* out);

}  // namespace mr
