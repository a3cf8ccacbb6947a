// Host-side ALS engine: device-resident context, work lists, CG driver, ALS
// loop, sharded exchange hooks, kernel timing.
//
// Control flow follows the reference exactly:
//   cg()         cg_least_squares        cpp/ls_lib/matrix.cpp:456-529
//   run()        als() outer loop        cpp/ls_lib/matrix.cpp:814-892
// but every numeric step runs on the GPU; the host only enqueues kernels and
// reads the 72-byte CG state once per chunk of CG iterations.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

#include "engine.h"

namespace mr {

// ----------------------------------------------------------------------------
// errors
// ----------------------------------------------------------------------------
static thread_local std::string g_err;
void set_error(const std::string& msg) {
  g_err = msg;
  if (!getenv("MR_QUIET")) fprintf(stderr, "[movie_recommender_amd] %s\n", msg.c_str());
}
const char* last_error() { return g_err.c_str(); }

// Device buffers come from hipMalloc, never from the stream-ordered pool
// (hipMallocAsync): on this ROCm (7.2, gfx950) a hipMemcpyAsync into a pool
// buffer can overtake a kernel still reading that buffer on the same stream,
// and a D2H copy out of one can return data older than the kernel that wrote
// it -- pinned or pageable host side alike; the same copies on hipMalloc
// buffers stay ordered (tools/probes/xfer_order.hip, profiles/r02/xfer_order.txt).
// That was the root cause of round 1's stale set -> get round trips.
template <typename T>
static int dalloc(T** p, int64_t n, hipStream_t s) {
  (void)s;
  *p = nullptr;
  if (n <= 0) n = 1;
  MR_HIP(hipMalloc((void**)p, (size_t)n * sizeof(T)));
  return 0;
}
template <typename T>
static void dfree(T*& p, hipStream_t s) {
  if (p) {
    (void)hipStreamSynchronize(s);
    (void)hipFree(p);
  }
  p = nullptr;
}

static void free_side(Side& S, hipStream_t s) {
  dfree(S.off, s); dfree(S.idx, s); dfree(S.val, s);
  dfree(S.work, s); dfree(S.split, s); dfree(S.slab, s);
  dfree(S.G, s); dfree(S.Gs, s); dfree(S.Gn, s); dfree(S.C, s); dfree(S.Cb, s);
  dfree(S.r, s); dfree(S.p, s); dfree(S.q, s);
  dfree(S.rb, s); dfree(S.pb, s); dfree(S.qb, s);
  dfree(S.start_parts, s);
}

Engine::~Engine() {
  if (stream) {
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    free_side(su, stream);
    free_side(si, stream);
    dfree(Ufac, stream); dfree(Ubias, stream); dfree(Vfac, stream);
    for (AgStage* A : {&ag_u, &ag_i}) {
      dfree(A->send, stream); dfree(A->recv, stream); dfree(A->rb, stream);
    }
    dfree(d_state, stream); dfree(partials, stream); dfree(d_flag, stream); dfree(xbins, stream);
    dfree(d_resgen, stream); dfree(d_resctl, stream);
    dfree(d_peer, stream);
    for (void* q : peer_opened) (void)hipIpcCloseMemHandle(q);
    if (peer_buf) (void)hipFree(peer_buf);
    (void)hipStreamSynchronize(stream);
    if (h_state) (void)hipHostFree(h_state);
    if (h_init) (void)hipHostFree(h_init);
    if (h_stage) (void)hipHostFree(h_stage);
    if (h_fac) (void)hipHostFree(h_fac);
    if (h_mirror) (void)hipHostFree(h_mirror);
    for (auto& e : ev_pool) (void)hipEventDestroy(e);
    for (auto& p : pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto& sp : spans) if (sp.end) (void)hipEventDestroy(sp.end);
    if (rccl) (void)ncclCommDestroy((ncclComm_t)rccl);
    (void)hipStreamDestroy(stream);
  }
}

// ----------------------------------------------------------------------------
// timing
// ----------------------------------------------------------------------------
int Engine::ev_get(hipEvent_t* e) {
  if (!ev_pool.empty()) {
    *e = ev_pool.back();
    ev_pool.pop_back();
    return 0;
  }
  MR_HIP(hipEventCreate(e));
  return 0;
}

// Timed launchers: tic hands a (start, stop) event pair to the launch-timing
// slot (mr_internal.h), which the launcher's kernels record from their own
// dispatch packets; toc files the pair for resolve_timing.
thread_local LaunchTiming t_launch;

int Engine::tic(int cls, int tag, hipEvent_t* a) {
  (void)cls; (void)tag;
  if (!timing) return 0;
  hipEvent_t b;
  if (ev_get(a) || ev_get(&b)) return -1;
  t_launch.start = *a;
  t_launch.stop = b;
  return 0;
}

int Engine::toc(int cls, int tag, hipEvent_t a) {
  if (!timing) return 0;
  if (t_launch.start) {  // the launcher had nothing to launch: empty interval
    MR_HIP(hipEventRecord(a, stream));
    MR_HIP(hipEventRecord(t_launch.stop, stream));
  }
  pending.push_back({cls, tag, a, t_launch.stop, 1 << 30});
  t_launch = LaunchTiming{};
  return 0;
}

// Attribute pending kernel and phase times (one stream sync; called when the
// stats are read, not per half-step, so timing does not stall the stream).
// Launches tagged with a CG iteration index >= their solve's n_real ran after
// the solve had finished (early-exit no-ops) and are not counted.
int Engine::resolve_timing() {
  if (drain()) return -1;   // every timed resident solve knows its CG count
  if (pending.empty() && spans.empty()) return 0;
  MR_HIP(hipStreamSynchronize(stream));
  for (auto& p : pending) {
    if (p.tag < 0 || p.tag < p.n_real) {
      float ms = 0.f;
      MR_HIP(hipEventElapsedTime(&ms, p.a, p.b));
      stats.kernel_ms[p.cls] += ms;
      stats.kernel_launches[p.cls] += 1;
      stats.kernel_units[p.cls] += p.units;
    }
  }
  for (auto& sp : spans) {
    if (sp.first >= sp.last && !sp.end) continue;
    hipEvent_t e0 = sp.first < sp.last ? pending[sp.first].a : sp.end;
    hipEvent_t e1 = sp.end ? sp.end : pending[sp.last - 1].b;
    float ms = 0.f;
    MR_HIP(hipEventElapsedTime(&ms, e0, e1));
    stats.phase_ms[sp.phase] += ms;
    if (sp.end) ev_pool.push_back(sp.end);
  }
  for (auto& p : pending) {
    ev_pool.push_back(p.a);
    ev_pool.push_back(p.b);
  }
  pending.clear();
  spans.clear();
  return 0;
}

// ----------------------------------------------------------------------------
// construction
// ----------------------------------------------------------------------------
// Gram work list with XCD-aligned opposite-id ranges (round 3).  Gram block b
// holds work items 4b .. 4b+3 and blocks are dealt round-robin over the 8
// XCDs (MI355X_MICROARCH.md), so list position p runs on XCD (p / 4) mod 8.
// Every heavy entity (more than `chunk` ratings) is cut at the opposite-id
// boundaries x * n_other / 8 (its ratings are ordered by opposite id: the
// CSR build sorts stably and ML-style input arrives grouped by user; an
// entity whose list is not sorted keeps fixed-size chunks, labelled by their
// middle id), each range into chunks of <= `chunk` ratings, and range x's
// chunks are dealt to positions on XCD x: each XCD's L2 then holds 1/8 of
// the opposite table (3.3 MB of U at k = 64) for the heavy entities'
// gathers, instead of every XCD streaming all of it.  The chunks come first
// (longest first within each XCD's queue; a queue that runs dry takes from
// the fullest), then the unsplit entities heavy first.  A split entity's
// partial records are summed by slab_reduce in range order, so its Gram sum
// order differs from a plain 2048-rating cut (results change at rounding
// level; tests/test_gpu_parity.py expected_layout restates this exactly).
// Applied to the matrix-core Gram (32 <= k <= 128) when the opposite table
// exceeds 16 MiB (ML-full k = 64: the items side, U = 26 MB); returns
// applied = false otherwise.
int Engine::build_work_xcd(Side& S, const std::vector<int64_t>& off, int64_t chunk,
                           std::vector<WorkItem>& work, std::vector<SplitItem>& split,
                           int32_t& nslab, bool& applied) {
  constexpr int64_t kWaves = 4, kXcds = 8;
  applied = false;
  const int64_t n_other = S.user ? I : U;
  const int64_t table = n_other * (int64_t)ldk * 4;
  if (k < 32 || k > 128 || table <= ((int64_t)16 << 20)) return 0;
  bool any_heavy = false;
  for (int64_t e = 0; e < S.E && !any_heavy; ++e) any_heavy = off[e + 1] - off[e] > chunk;
  if (!any_heavy) return 0;
  std::vector<int32_t> idx(S.nnz);
  if (S.nnz) MR_D2H(idx.data(), S.idx, S.nnz * sizeof(int32_t), stream);
  std::vector<std::vector<WorkItem>> q(kXcds);
  std::vector<WorkItem> light;
  for (int64_t e = 0; e < S.E; ++e) {
    const int64_t b0 = off[e], b1 = off[e + 1], len = b1 - b0;
    if (len <= chunk) {
      light.push_back({b0, (int32_t)len, (int32_t)e, -1, 0});
      continue;
    }
    const bool sorted = std::is_sorted(idx.begin() + b0, idx.begin() + b1);
    const int32_t s0 = nslab;
    auto cut = [&](int64_t a, int64_t z, int x) {   // [a, z) into chunks on XCD x
      for (int64_t c = a; c < z; c += chunk) {
        const int64_t l = std::min<int64_t>(chunk, z - c);
        q[x].push_back({c, (int32_t)l, (int32_t)e, nslab++, 0});
      }
    };
    if (sorted) {
      int64_t a = b0;
      for (int x = 0; x < kXcds; ++x) {
        const int32_t hi = (int32_t)((x + 1) * n_other / kXcds);
        const int64_t z = x == kXcds - 1 ? b1
                                         : std::lower_bound(idx.begin() + a, idx.begin() + b1, hi) -
                                               idx.begin();
        cut(a, z, x);
        a = z;
      }
    } else {
      for (int64_t c = b0; c < b1; c += chunk) {
        const int64_t l = std::min<int64_t>(chunk, b1 - c);
        const int x = (int)std::min<int64_t>(kXcds - 1, idx[c + l / 2] * kXcds / n_other);
        q[x].push_back({c, (int32_t)l, (int32_t)e, nslab++, 0});
      }
    }
    split.push_back({(int32_t)e, s0, nslab - s0, 0});
  }
  int64_t n_chunks = 0;
  for (auto& v : q) {
    std::stable_sort(v.begin(), v.end(),
                     [](const WorkItem& a, const WorkItem& b) { return a.len > b.len; });
    n_chunks += (int64_t)v.size();
  }
  std::vector<size_t> head(kXcds, 0);
  for (int64_t p = 0; p < n_chunks; ++p) {
    int x = (int)((p / kWaves) % kXcds);
    if (head[x] == q[x].size()) {   // this XCD's queue ran dry: the fullest one
      size_t best = 0;
      for (int y = 0; y < kXcds; ++y)
        if (q[y].size() - head[y] > best) {
          best = q[y].size() - head[y];
          x = y;
        }
    }
    work.push_back(q[x][head[x]++]);
  }
  std::stable_sort(light.begin(), light.end(),
                   [](const WorkItem& a, const WorkItem& b) { return a.len > b.len; });
  work.insert(work.end(), light.begin(), light.end());
  applied = true;
  return 0;
}

int Engine::build_side(Side& S, bool user, int64_t n, const int32_t* d_key,
                       const int32_t* d_other, const double* d_r) {
  S.user = user;
  MR_CHECK(S.E >= 0, "negative entity range");
  if (dalloc(&S.off, S.E + 1, stream) || dalloc(&S.idx, n, stream) ||
      dalloc(&S.val, n, stream))
    return -1;
  S.nnz = n;
  if (build_csr<float, double>(stream, n, S.E, d_key, (int32_t)S.e0, d_other, d_r,
                               S.off, S.idx, S.val))
    return -1;
  // host copy of the offsets -> work list (chunks, heavy first)
  std::vector<int64_t> off(S.E + 1);
  MR_D2H(off.data(), S.off, (S.E + 1) * sizeof(int64_t), stream);
  MR_HIP(hipStreamSynchronize(stream));
  std::vector<WorkItem> work;
  std::vector<SplitItem> split;
  work.reserve(S.E + n / chunk + 1);
  int32_t nslab = 0;
  bool xcd = false;
  if (build_work_xcd(S, off, chunk, work, split, nslab, xcd)) return -1;
  for (int64_t e = 0; e < (xcd ? 0 : S.E); ++e) {
    const int64_t len = off[e + 1] - off[e];
    if (len <= chunk) {
      work.push_back({off[e], (int32_t)len, (int32_t)e, -1, 0});
    } else {
      const int32_t nc = (int32_t)((len + chunk - 1) / chunk);
      split.push_back({(int32_t)e, nslab, nc, 0});
      for (int32_t c = 0; c < nc; ++c) {
        const int64_t b = off[e] + (int64_t)c * chunk;
        const int64_t l = std::min<int64_t>(chunk, off[e + 1] - b);
        work.push_back({b, (int32_t)l, (int32_t)e, nslab + c, 0});
      }
      nslab += nc;
    }
  }
  if (!xcd)
    std::stable_sort(work.begin(), work.end(),
                     [](const WorkItem& a, const WorkItem& b) { return a.len > b.len; });
  S.n_work = (int64_t)work.size();
  S.n_split = (int64_t)split.size();
  S.n_slab = nslab;
  S.rec = gsize_of(k) + 2 * ldk + 4;
  if (dalloc(&S.work, S.n_work, stream) || dalloc(&S.split, S.n_split, stream) ||
      dalloc(&S.slab, S.n_slab * S.rec, stream))
    return -1;
  if (S.n_work)
    MR_H2D(S.work, work.data(), S.n_work * sizeof(WorkItem), stream);
  if (S.n_split)
    MR_H2D(S.split, split.data(), S.n_split * sizeof(SplitItem), stream);
  // normal equations + CG vectors
  const int64_t ef = S.E * ldk;
  if (dalloc(&S.G, S.E * gsize_of(k), stream) || dalloc(&S.C, ef, stream) ||
      dalloc(&S.r, ef, stream) || dalloc(&S.p, ef, stream) || dalloc(&S.q, ef, stream))
    return -1;
  // padding columns (n >= k) of the CG vectors stay exactly zero
  if (user) {
    if (dalloc(&S.Gs, ef, stream) || dalloc(&S.Gn, S.E, stream) ||
        dalloc(&S.Cb, S.E, stream) || dalloc(&S.rb, S.E, stream) ||
        dalloc(&S.pb, S.E, stream) || dalloc(&S.qb, S.E, stream))
      return -1;
  }
  MR_HIP(hipMemsetAsync(S.r, 0, ef * sizeof(double), stream));
  MR_HIP(hipMemsetAsync(S.p, 0, ef * sizeof(double), stream));
  MR_HIP(hipMemsetAsync(S.q, 0, ef * sizeof(double), stream));
  if (user) {
    MR_HIP(hipMemsetAsync(S.rb, 0, S.E * sizeof(double), stream));
    MR_HIP(hipMemsetAsync(S.pb, 0, S.E * sizeof(double), stream));
    MR_HIP(hipMemsetAsync(S.qb, 0, S.E * sizeof(double), stream));
  }
  // fused CG start: one (r.r, p.Gp, q.q) triple per Gram block, then per split block
  S.n_start_pairs = gram_blocks(S.n_work, k) + (S.n_split + 3) / 4;
  if (dalloc(&S.start_parts, 3 * std::max<int64_t>(1, S.n_start_pairs), stream)) return -1;
  // matvec grid: one wave per entity, fixed grid for reproducible partials
  const int64_t g = (S.E + 3) / 4;
  S.n_part_mv = (int)std::max<int64_t>(1, std::min<int64_t>(g, kMaxParts));
  // one-pass CG kernel: exactly the blocks the chip holds at once (a second,
  // partial round of blocks measured up to 30 % slower: users k = 64, 3
  // blocks per CU, 768 blocks 216 us, 1024 blocks 286 us, 2048 blocks 238
  // us); MR_MV_PARTS overrides it for tuning experiments
  static const int64_t parts_env = [] {
    const char* e = getenv("MR_MV_PARTS");
    return e ? (int64_t)atoll(e) : (int64_t)0;
  }();
  // (per instantiation: the plain-load and the non-temporal variant are
  // separate code objects whose occupancy may differ; tile_nt_for picks one
  // at launch time)
  for (int nt = 0; nt < 2; ++nt) {
    int64_t op = g;
    if (k <= kMaxK) {
      int cus = 0;
      MR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
      const int bpc = onepass_blocks_per_cu(S.user, k, nt != 0);
      if (bpc > 0 && cus > 0) op = std::min<int64_t>(op, (int64_t)bpc * cus);
    }
    if (parts_env > 0) op = std::min(g, parts_env);
    S.n_part_op[nt] = (int)std::max<int64_t>(1, std::min<int64_t>(op, kMaxParts));
    // the resident solve: never more blocks than the chip holds at once
    // (its per-iteration broadcast waits for every block)
    S.n_part_rs[nt] = 0;
    if (k <= kMaxK) {
      int cus = 0;
      MR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
      const int bpc = resident_blocks_per_cu(S.user, k, nt != 0);
      if (bpc > 0 && cus > 0)
        S.n_part_rs[nt] = (int)std::min<int64_t>({g, (int64_t)bpc * cus, (int64_t)kMaxParts});
    }
  }
  MR_HIP(hipStreamSynchronize(stream));
  return 0;
}

int Engine::init(int dev, int k_, int64_t U_, int64_t I_, int64_t n_u,
                 const int* uv_uid, const int* uv_iid, const double* uv_r,
                 int64_t n_i, const int* iv_uid, const int* iv_iid,
                 const double* iv_r, int64_t u0, int64_t u1, int64_t i0,
                 int64_t i1) {
  device = dev;
  k = k_;
  ldk = ldk_of(k);
  U = U_;
  I = I_;
  MR_CHECK(k >= 1 && k <= kMaxKLarge, "k must be in [1, 512]");
  MR_CHECK(U >= 0 && I >= 0, "negative table size");
  MR_CHECK(0 <= u0 && u0 <= u1 && u1 <= U && 0 <= i0 && i0 <= i1 && i1 <= I,
           "bad shard range");
  MR_HIP(hipSetDevice(device));
  MR_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  MR_HIP(hipHostMalloc((void**)&h_state, sizeof(CgState), hipHostMallocDefault));
  MR_HIP(hipHostMalloc((void**)&h_init, sizeof(CgState), hipHostMallocDefault));
  MR_HIP(hipHostMalloc((void**)&h_stage, 64, hipHostMallocDefault));
  MR_HIP(hipHostMalloc((void**)&h_mirror, kMirrorSlots * sizeof(CgMirror),
                       hipHostMallocMapped | hipHostMallocCoherent));
  memset(h_mirror, 0, kMirrorSlots * sizeof(CgMirror));
  MR_HIP(hipHostGetDevicePointer((void**)&d_mirror, h_mirror, 0));
  if (dalloc(&d_state, 1, stream) || dalloc(&partials, 4 * kMaxParts, stream) ||
      dalloc(&d_flag, 4, stream) || dalloc(&xbins, kXBinWords + kXBinStartWords, stream) ||
      dalloc(&d_resgen, kResGenWords, stream) || dalloc(&d_resctl, 1, stream))
    return -1;
  MR_HIP(hipMemsetAsync(xbins, 0, (kXBinWords + kXBinStartWords) * sizeof(int64_t), stream));
  MR_HIP(hipMemsetAsync(d_resgen, 0, kResGenWords * sizeof(uint64_t), stream));
  if (write_res_ctl()) return -1;
  // every field defined before any kernel reads it: the fused CG start
  // re-initialises the scalars but not `peer` (set only by set_peer)
  MR_HIP(hipMemsetAsync(d_state, 0, sizeof(CgState), stream));
  su.e0 = u0; su.E = u1 - u0;
  si.e0 = i0; si.E = i1 - i0;
  // factor tables (replicated), zero padding columns
  // one extra all-zero row per table: the Gram kernel's padding target
  if (dalloc(&Ufac, (U + 1) * ldk, stream) || dalloc(&Ubias, U + 1, stream) ||
      dalloc(&Vfac, (I + 1) * ldk, stream))
    return -1;
  MR_HIP(hipMemsetAsync(Ufac, 0, (U + 1) * ldk * 4, stream));
  MR_HIP(hipMemsetAsync(Ubias, 0, (U + 1) * 4, stream));
  MR_HIP(hipMemsetAsync(Vfac, 0, (I + 1) * ldk * 4, stream));
  // user-side weights (the ratings as fp32) exact in bf16? -> the Gram may
  // take the rhs on the matrix cores (MR_OPT_GRAM_RHS_MFMA)
  w_bf16 = true;
  for (int64_t t = 0; t < n_u && w_bf16; ++t) {
    const float f = (float)uv_r[t];
    uint32_t bits;
    memcpy(&bits, &f, 4);
    w_bf16 = (bits & 0xFFFFu) == 0;
  }
  // upload + build both views
  const bool same = (uv_uid == iv_uid && uv_iid == iv_iid && uv_r == iv_r && n_u == n_i);
  for (int view = 0; view < (same ? 1 : 2); ++view) {
    const int64_t n = view == 0 ? n_u : n_i;
    const int* hu = view == 0 ? uv_uid : iv_uid;
    const int* hi = view == 0 ? uv_iid : iv_iid;
    const double* hr = view == 0 ? uv_r : iv_r;
    int32_t *du = nullptr, *di = nullptr;
    double* dr = nullptr;
    if (dalloc(&du, n, stream) || dalloc(&di, n, stream) || dalloc(&dr, n, stream)) return -1;
    if (n > 0) {
      MR_H2D(du, hu, n * 4, stream);
      MR_H2D(di, hi, n * 4, stream);
      MR_H2D(dr, hr, n * 8, stream);
    }
    // id range validation (the reference has none: out-of-range ids are UB)
    MR_HIP(hipMemsetAsync(d_flag, 0, 16, stream));
    if (launch_validate_ids(stream, n, du, view == 0 || same ? (int32_t)u0 : 0,
                            view == 0 || same ? (int32_t)u1 : (int32_t)U, d_flag))
      return -1;
    if (launch_validate_ids(stream, n, di, view == 1 || same ? (int32_t)i0 : 0,
                            view == 1 || same ? (int32_t)i1 : (int32_t)I, d_flag + 1))
      return -1;
    int flags[2] = {0, 0};
    MR_D2H(flags, d_flag, 8, stream);
    MR_HIP(hipStreamSynchronize(stream));
    if (view == 0 && !same) {
      MR_CHECK(!flags[0], "user view: user id outside this shard's user range");
      MR_CHECK(!flags[1], "user view: item id outside [0, num_items)");
    } else if (view == 1) {
      MR_CHECK(!flags[0], "item view: user id outside [0, num_users)");
      MR_CHECK(!flags[1], "item view: item id outside this shard's item range");
    } else {
      MR_CHECK(!flags[0], "user id outside [0, num_users)");
      MR_CHECK(!flags[1], "item id outside [0, num_items)");
    }
    int rc = 0;
    if (view == 0) rc = build_side(su, true, n, du, di, dr);
    if (rc == 0 && (view == 1 || same)) rc = build_side(si, false, n, di, du, dr);
    dfree(du, stream); dfree(di, stream); dfree(dr, stream);
    if (rc) return -1;
  }
  N = su.nnz;
  MR_HIP(hipStreamSynchronize(stream));
  return 0;
}

// ----------------------------------------------------------------------------
// factors
// ----------------------------------------------------------------------------
// Factor transfers stage through pinned host memory that the pack / unpack
// kernels read and write directly (zero-copy; fine-grained, system-coherent).
// The earlier form -- a pageable hipMemcpyAsync into a pool buffer, then a
// kernel -- let replays from one snapshot diverge run to run (a kernel saw
// stale staging data).
int Engine::fac_stage(int64_t n) {
  if (n <= h_fac_n) return 0;
  if (h_fac) MR_HIP(hipHostFree(h_fac));
  h_fac = nullptr;
  h_fac_n = 0;
  MR_HIP(hipHostMalloc((void**)&h_fac, (size_t)n * sizeof(double), hipHostMallocDefault));
  h_fac_n = n;
  return 0;
}

int Engine::set_factors(const double* hU, const double* hV) {
  if (drain()) return -1;
  MR_HIP(hipSetDevice(device));
  const int64_t nU = U * (k + 1), nV = I * (int64_t)k;
  int rc = 0;
  MR_HIP(hipStreamSynchronize(stream));   // no kernel may still read h_fac
  if (fac_stage(nU + nV)) return -1;
  if (hU && U) {
    memcpy(h_fac, hU, nU * 8);
    rc |= launch_unpack_factors(stream, U, k + 1, k, ldk, h_fac, Ufac, Ubias);
  }
  if (hV && I) {
    memcpy(h_fac + nU, hV, nV * 8);
    rc |= launch_unpack_factors(stream, I, k, k, ldk, h_fac + nU, Vfac, nullptr);
  }
  MR_HIP(hipStreamSynchronize(stream));
  return rc ? -1 : 0;
}

int Engine::get_factors(double* hU, double* hV) {
  if (drain()) return -1;
  MR_HIP(hipSetDevice(device));
  const int64_t nU = U * (k + 1), nV = I * (int64_t)k;
  int rc = 0;
  MR_HIP(hipStreamSynchronize(stream));
  if (fac_stage(nU + nV)) return -1;
  if (hU && U) rc |= launch_pack_factors(stream, U, k + 1, k, ldk, Ufac, Ubias, h_fac);
  if (hV && I) rc |= launch_pack_factors(stream, I, k, k, ldk, Vfac, nullptr, h_fac + nU);
  MR_HIP(hipStreamSynchronize(stream));
  if (hU && U) memcpy(hU, h_fac, nU * 8);
  if (hV && I) memcpy(hV, h_fac + nU, nV * 8);
  return rc ? -1 : 0;
}

// ----------------------------------------------------------------------------
// collectives (sharded runs); host-staged callbacks
// ----------------------------------------------------------------------------
#define MR_NCCL(call)                                                        \
  do {                                                                       \
    ncclResult_t _r = (call);                                                \
    MR_CHECK(_r == ncclSuccess, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

int Engine::set_rccl(const unsigned char* id, int rank, int world) {
  MR_CHECK(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
  MR_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  static_assert(sizeof(uid.internal) == 128, "ncclUniqueId size");
  memcpy(uid.internal, id, 128);
  ncclComm_t c;
  MR_NCCL(ncclCommInitRank(&c, world, uid, rank));
  rccl = (void*)c;
  rccl_world = world;
  rccl_rank = rank;
  return alloc_ag(world);
}

// Peer all-reduce of the CG scalars: this rank's exchange buffer (kPeerSlots x
// kMaxPeers records of kPeerRec doubles, uncached device memory so that peers'
// stores over xGMI are seen by this GPU's loads) and its IPC handle.
int Engine::peer_handle(unsigned char* out64) {
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t size");
  MR_HIP(hipSetDevice(device));
  if (!peer_buf) {
    const size_t bytes = (size_t)kPeerSlots * kMaxPeers * kPeerRec * sizeof(double);
    MR_HIP(hipExtMallocWithFlags((void**)&peer_buf, bytes, hipDeviceMallocUncached));
    MR_HIP(hipMemsetAsync(peer_buf, 0, bytes, stream));
    MR_HIP(hipStreamSynchronize(stream));
  }
  hipIpcMemHandle_t h;
  MR_HIP(hipIpcGetMemHandle(&h, peer_buf));
  memcpy(out64, &h, 64);
  return 0;
}

// Map every peer's exchange buffer and switch the CG scalars to the peer
// all-reduce: the finalizing thread of each reduction exchanges its sum with
// the peers itself, so a sharded CG iteration issues the unsharded launch
// sequence (matvec, update) with no collective launch in between.  All
// ranks must call this (after exchanging the handles of peer_handle) before
// their next solve; the factor all-gather keeps its transport.
//
// Once only: the exchange buffers' sequence numbers start at 0 with the first
// mapping, so a second set_peer (stale tags of the earlier setup still in the
// peers' buffers could satisfy a new reduction) is refused; world == 0
// switches back to the collective scalars for good (the mappings stay open
// until the context is destroyed).
int Engine::set_peer(const unsigned char* handles, int rank, int world) {
  if (world == 0) {   // back to the collective scalars (e.g. a failed self-test)
    MR_HIP(hipSetDevice(device));
    PeerComm* none = nullptr;
    MR_H2D((char*)d_state + offsetof(CgState, peer), &none, sizeof(none), stream);
    MR_HIP(hipStreamSynchronize(stream));
    peer_on = false;
    peer_used = true;
    return 0;
  }
  MR_CHECK(handles, "null handles");
  MR_CHECK(world >= 1 && world <= kMaxPeers && rank >= 0 && rank < world, "bad rank/world");
  MR_CHECK(peer_buf, "mr_als_peer_handle must be called first");
  MR_CHECK(!peer_used, "the peer all-reduce is set up once per context");
  MR_HIP(hipSetDevice(device));
  peer_used = true;
  PeerComm pc{};
  pc.world = world;
  pc.rank = rank;
  pc.timeout_ticks = (uint64_t)(peer_timeout_s * 1e8);
  for (int q = 0; q < world; ++q) {
    if (q == rank) {
      pc.buf[q] = peer_buf;
      continue;
    }
    hipIpcMemHandle_t h;
    memcpy(&h, handles + (size_t)q * 64, 64);
    void* ptr = nullptr;
    MR_HIP(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
    peer_opened.push_back(ptr);
    pc.buf[q] = (double*)ptr;
  }
  if (!d_peer && dalloc(&d_peer, 1, stream)) return -1;
  MR_H2D(d_peer, &pc, sizeof(PeerComm), stream);
  PeerComm* dp = d_peer;
  MR_H2D((char*)d_state + offsetof(CgState, peer), &dp, sizeof(dp), stream);
  MR_HIP(hipStreamSynchronize(stream));
  peer_on = true;
  return 0;
}

// Cache policy of the one-pass kernel's G tile loads for side S: a side
// whose per-iteration stream (tri16 blocks + the fp64 CG vectors) exceeds
// kTileNtBytes is streamed non-temporally -- little of it survives in the
// 256 MiB Infinity Cache to the next sweep, and plain loads measured 25 %
// slower at the full ML-full users side (1.26 GB; DESIGN.md "Sweep
// direction"); a smaller side keeps the default policy, so the alternating
// sweeps find the previous sweep's tail on-die: measured 5-6 % faster at the
// 4- and 8-rank shard sizes of ML-full (users 260 / 157 MB per iteration,
// profiles/r04 session r04b).
constexpr int64_t kTileNtBytes = 320ll << 20;
bool Engine::tile_nt_for(const Side& S) const {
  if (tile_nt >= 0) return tile_nt != 0;
  const int64_t vec = (int64_t)S.E * (ldk + (S.user ? 1 : 0)) * (3 * 8 + 4);
  return (int64_t)S.E * gsize_of(k) * 4 + vec > kTileNtBytes;
}

// Device wait for a peer's record, seconds (MR_OPT_PEER_TIMEOUT_S); takes
// effect at once when the peer all-reduce is already mapped.
int Engine::set_peer_timeout(double seconds) {
  MR_CHECK(seconds > 0.0 && seconds <= 1e5, "peer timeout must be in (0, 1e5] s");
  peer_timeout_s = seconds;
  if (d_peer) {
    MR_HIP(hipSetDevice(device));
    const uint64_t ticks = (uint64_t)(seconds * 1e8);
    MR_H2D((char*)d_peer + offsetof(PeerComm, timeout_ticks), &ticks, sizeof(ticks), stream);
    MR_HIP(hipStreamSynchronize(stream));
  }
  if (d_resctl) {   // the resident broadcast outwaits the peers
    MR_HIP(hipSetDevice(device));
    if (drain() || write_res_ctl()) return -1;
  }
  return 0;
}

// The user-side Gram's rhs path (W block on the matrix cores) needs every
// weight exact in bf16; a sharded run must take the same path on every rank
// (the paths round differently), so the ranks agree on the flag:
// force < 0 reads it, force == 0 clears it (force == 1 is rejected unless
// this rank's ratings allow it).
int Engine::weights_bf16(int force) {
  if (force < 0) return w_bf16 ? 1 : 0;
  MR_CHECK(force == 0 || w_bf16, "this rank's ratings are not exact in bf16");
  w_bf16 = force != 0;
  return w_bf16 ? 1 : 0;
}

// One reduction of {rank + 1, 1} through the mapped buffers (collective: all
// ranks call it): 0 if every rank's record arrived and the sums are right.
int Engine::peer_selftest() {
  MR_CHECK(peer_on && d_peer, "peer all-reduce not set up");
  MR_HIP(hipSetDevice(device));
  double* d_out = nullptr;
  if (dalloc(&d_out, 3, stream)) return -1;
  double out[3] = {0, 0, 0};
  int rc = launch_peer_selftest(stream, d_peer, d_out);
  if (!rc) rc = t_stager.d2h(stream, out, d_out, sizeof(out));
  dfree(d_out, stream);
  if (rc) return -1;
  PeerComm pc{};
  MR_D2H(&pc, d_peer, sizeof(PeerComm), stream);
  const double w = pc.world;
  MR_CHECK(out[2] == 1.0, "peer all-reduce self-test: a rank did not arrive");
  MR_CHECK(out[0] == w * (w + 1) / 2 && out[1] == w, "peer all-reduce self-test: wrong sum");
  return 0;
}

// The peer all-reduce's accounting since the last reset (stats): device
// time of the reducing threads (s_memrealtime, 100 MHz) and reductions.
int Engine::peer_account(double* wait_ms, long long* n, bool reset) {
  *wait_ms = 0.0;
  *n = 0;
  if (!d_peer) return 0;
  MR_HIP(hipSetDevice(device));
  PeerComm pc{};
  MR_D2H(&pc, d_peer, sizeof(PeerComm), stream);
  if (reset) {
    peer_ticks0 = pc.wait_ticks;
    peer_n0 = pc.n_reduce;
  }
  *wait_ms = (double)(pc.wait_ticks - peer_ticks0) / 1e5;
  *n = (long long)(pc.n_reduce - peer_n0);
  return 0;
}

// Device-side latency of the peer all-reduce (collective: every rank calls it
// with the same iters): mean microseconds per reduction over `iters`
// back-to-back reductions by one thread, from HIP events around the kernel.
int Engine::peer_latency(int iters, double* us) {
  MR_CHECK(peer_on && d_peer, "peer all-reduce not set up");
  MR_CHECK(iters >= 1 && iters <= 1000000, "iters must be in [1, 1e6]");
  MR_HIP(hipSetDevice(device));
  double* d_out = nullptr;
  if (dalloc(&d_out, 2, stream)) return -1;
  hipEvent_t a, b;
  MR_HIP(hipEventCreate(&a));
  MR_HIP(hipEventCreate(&b));
  MR_HIP(hipEventRecord(a, stream));
  int rc = launch_peer_bench(stream, d_peer, iters, d_out);
  MR_HIP(hipEventRecord(b, stream));
  double out[2] = {0, 0};
  if (!rc) rc = t_stager.d2h(stream, out, d_out, sizeof(out));
  float ms = 0.f;
  MR_HIP(hipEventSynchronize(b));
  MR_HIP(hipEventElapsedTime(&ms, a, b));
  MR_HIP(hipEventDestroy(a));
  MR_HIP(hipEventDestroy(b));
  dfree(d_out, stream);
  if (rc) return -1;
  MR_CHECK(out[0] == 1.0 && out[1] == iters, "peer all-reduce latency probe: wrong sum or timeout");
  *us = 1e3 * ms / iters;
  return 0;
}

// All-gather staging, the same for both transports: every rank's shard padded
// to the largest one (maxrows rows of ldk floats, + the user bias column).
// Row boundaries are checked here, on the host, against everything the pack /
// unstage kernels assume (monotone, covering the table, own shard <= maxrows).
int Engine::alloc_ag(int world) {
  MR_HIP(hipSetDevice(device));
  for (int side = 0; side < 2; ++side) {
    const std::vector<long long>& rb = side == 0 ? row_begin_u : row_begin_i;
    MR_CHECK((int)rb.size() == world + 1 && rb[0] == 0 && rb[world] == (side == 0 ? U : I),
             "row boundaries must cover the table");
    long long mx = 1;
    for (int r = 0; r < world; ++r) {
      MR_CHECK(rb[r + 1] >= rb[r], "row boundaries not monotone");
      mx = std::max(mx, rb[r + 1] - rb[r]);
    }
    AgStage& A = side == 0 ? ag_u : ag_i;
    dfree(A.send, stream); dfree(A.recv, stream); dfree(A.rb, stream);
    A.maxrows = mx;
    A.per = ag_block_floats(mx, ldk, side == 0);
    if (dalloc(&A.send, A.per, stream) || dalloc(&A.recv, (int64_t)world * A.per, stream) ||
        dalloc(&A.rb, world + 1, stream))
      return -1;
    std::vector<int64_t> rb64(rb.begin(), rb.end());
    MR_H2D(A.rb, rb64.data(), rb64.size() * 8, stream);
  }
  // this rank's shard must be the one the context was built for
  const int rk = ag_rank();
  MR_CHECK(row_begin_u[rk] == su.e0 && row_begin_u[rk + 1] == su.e0 + su.E &&
               row_begin_i[rk] == si.e0 && row_begin_i[rk + 1] == si.e0 + si.E,
           "row boundaries disagree with this context's shard ranges");
  return 0;
}

// Sum the CG scalar slot over ranks.  RCCL: in place on the device, ordered on
// the engine stream (no host synchronisation).  Callbacks: staged via host.
int Engine::allreduce_state_slot(int count) {
  if (!sharded()) return 0;
  if (rccl) {
    MR_NCCL(ncclAllReduce(&d_state->comm[0], &d_state->comm[0], (size_t)count, ncclDouble,
                          ncclSum, (ncclComm_t)rccl, stream));
    return 0;
  }
  MR_HIP(hipMemcpyAsync(h_stage, &d_state->comm[0], count * sizeof(double), hipMemcpyDeviceToHost, stream));
  MR_HIP(hipStreamSynchronize(stream));
  MR_CHECK(comm.allreduce_f64(comm.user, (double*)h_stage, count) == 0,
           "allreduce callback failed");
  MR_HIP(hipMemcpyAsync(&d_state->comm[0], h_stage, count * sizeof(double), hipMemcpyHostToDevice, stream));
  return 0;
}

// Replicate the freshly solved shard rows of a factor table on every rank:
// the own rows are packed into a send buffer, exchanged as ONE all-gather of
// equal, padded shards (world x maxrows rows; users: the bias column rides in
// the same block), and every other rank's rows unstaged into place by one
// kernel.  The
// device side (pack_rows -> padded buffers -> unstage_rows) is the same for
// both transports: RCCL gathers the device buffers directly; the callback
// transport carries the same padded buffers through host memory and
// comm.allgather_rows (padded row boundaries r * maxrows), so the gloo tests
// run the exact staging code of the RCCL path at any world size.
int Engine::allgather_side(bool user) {
  if (!sharded()) return 0;
  // timed as one span (MR_K_EXCHANGE): pack, the collective, unstage
  hipEvent_t ea = nullptr, eb = nullptr;
  if (timing) {
    if (ev_get(&ea) || ev_get(&eb)) return -1;
    MR_HIP(hipEventRecord(ea, stream));
  }
  const int rc = allgather_rows_side(user);
  if (timing) {
    MR_HIP(hipEventRecord(eb, stream));
    pending.push_back({MR_K_EXCHANGE, -1, ea, eb, 1 << 30});
  }
  return rc;
}

int Engine::allgather_rows_side(bool user) {
  const std::vector<long long>& rb = user ? row_begin_u : row_begin_i;
  const int world = ag_world(), rank = ag_rank();
  AgStage& A = user ? ag_u : ag_i;
  MR_CHECK(A.recv != nullptr, "all-gather staging not allocated");
  float* fac = user ? Ufac : Vfac;
  float* bias = user ? Ubias : nullptr;
  if (launch_pack_rows(stream, rb[rank], rb[rank + 1] - rb[rank], ldk, fac, bias, A.send,
                       bias ? A.send + A.maxrows * ldk : nullptr))
    return -1;
  if (rccl) {
    MR_NCCL(ncclAllGather(A.send, A.recv, (size_t)A.per, ncclFloat, (ncclComm_t)rccl, stream));
  } else {
    // the callback carries each rank's block as one padded "row" of A.per floats
    h_ag.resize((size_t)world * A.per);
    float* tab = h_ag.data();
    MR_D2H(tab + (size_t)rank * A.per, A.send, A.per * 4, stream);
    std::vector<long long> prb(world + 1);
    for (int r = 0; r <= world; ++r) prb[r] = r;
    MR_CHECK(comm.allgather_rows(comm.user, tab, (long long)A.per, prb.data(), world) == 0,
             "allgather callback failed");
    MR_H2D(A.recv, tab, (size_t)world * A.per * 4, stream);
  }
  return launch_unstage_rows(stream, world, rank, A.rb, A.maxrows, ldk, A.recv, fac, bias);
}

// Sharded CG: all-reduce the slot the last block filled, then apply the rule.
int Engine::finalize_sharded(int phase, int seq) {
  if (allreduce_state_slot()) return -1;
  hipEvent_t a = nullptr;
  if (tic(MR_K_CG_CONTROL, -1, &a)) return -1;
  if (launch_cg_control(stream, d_state, phase, CTL_FINALIZE, partials, cur_parts,
                        seq > 0 ? d_mirror : nullptr, seq))
    return -1;
  return toc(MR_K_CG_CONTROL, -1, a);
}

// Spin on the host-mapped mirror ring until the state published under
// sequence number `target` is in its slot.  Seqlock protocol (publish(),
// kernels.hip): the device stores 2 seq - 1 (odd: write in progress), the
// fields, then 2 seq (release); a copy is accepted only if it was bracketed by
// 2 target.  Checks the stream for errors and for "stream idle but nothing
// published" (a bug), and gives up after wait_timeout_s (a stalled peer rank
// in a sharded run).
int wait_published(CgMirror* ring, int target, hipStream_t stream, double timeout_s,
                   CgMirror* out) {
  const int want = 2 * target;
  CgMirror* slot = ring + (target & (kMirrorSlots - 1));
  long spins = 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    const int s1 = __atomic_load_n(&slot->seq, __ATOMIC_ACQUIRE);
    if (s1 == want) {
      CgMirror m;
      memcpy(&m, (const void*)slot, sizeof(CgMirror));
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      if (__atomic_load_n(&slot->seq, __ATOMIC_ACQUIRE) == s1) {
        *out = m;
        out->seq = target;
        return 0;
      }
      continue;  // overwritten while copying (cannot happen within the ring depth)
    }
    MR_CHECK(s1 < want, "CG state slot overwritten before it was read");
    if ((++spins & 1023) == 0) {
      const hipError_t q = hipStreamQuery(stream);
      if (q == hipSuccess) {
        if (__atomic_load_n(&slot->seq, __ATOMIC_ACQUIRE) == want) continue;
        MR_CHECK(false, "CG state was not published (stream idle)");
      }
      MR_CHECK(q == hipErrorNotReady,
               std::string("stream error while polling CG state: ") + hipGetErrorString(q));
      const double el =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      MR_CHECK(el < timeout_s, "timed out waiting for the CG state (" + std::to_string(el) +
                                   " s; stalled peer rank?)");
    }
    __builtin_ia32_pause();
  }
}

int Engine::wait_mirror(int target, CgMirror* out) {
  return wait_published(h_mirror, target, stream, wait_timeout_s, out);
}

// ----------------------------------------------------------------------------
// half-step pieces
// ----------------------------------------------------------------------------
GramDst Engine::direct_dst(Side& S) {
  GramDst d;
  d.G = S.G; d.Gs = S.Gs; d.C = S.C; d.Cb = S.Cb; d.Gn = S.Gn;
  d.sG = gsize_of(k); d.sV = ldk; d.sS = 1;
  return d;
}

GramDst Engine::slab_dst(Side& S) {
  GramDst d;
  const int64_t nG = gsize_of(k);
  d.G = S.slab; d.Gs = S.slab + nG; d.C = S.slab + nG + ldk;
  d.Cb = S.slab + nG + 2 * ldk; d.Gn = S.slab + nG + 2 * ldk + 1;
  d.sG = d.sV = d.sS = S.rec;
  return d;
}

CgStart Engine::cg_start_of(Side& S) {
  CgStart cs{};
  float *xf, *xb;
  x_ptrs(S, &xf, &xb);
  cs.x = xf;
  cs.xb = xb;
  cs.r = S.r; cs.rb = S.rb; cs.p = S.p; cs.pb = S.pb; cs.q = S.q; cs.qb = S.qb;
  cs.parts = S.start_parts;
  cs.xbins = onepass_for(S) ? xbins + kXBinWords : nullptr;
  return cs;
}

// The resident solve's control block: pointers fixed for the context's
// life, and the broadcast timeout (the peer timeout plus 30 s, rewritten
// when that changes).
int Engine::write_res_ctl() {
  ResCtl c{d_state, xbins, d_resgen, d_mirror, (uint64_t)((peer_timeout_s + 30.0) * 1e8)};
  MR_H2D(d_resctl, &c, sizeof(ResCtl), stream);
  return 0;
}

bool Engine::resident_for(const Side& S) const {
  return resident && onepass_for(S) && S.n_part_rs[tile_nt_for(S) ? 1 : 0] > 0;
}

bool Engine::onepass_for(const Side& S) const {
  // one pass per CG iteration on both sides for k <= 128.  At k > 64 the
  // tiles stream through a register ring (tile_matvec_stream, no spills):
  // k = 128, ML-full shape, fixed 20 iterations, users 0.2411 ms per CG
  // iteration against 0.2617 for matvec + update (0.2724 in round 3's
  // two-kernel form), items 0.1093 against 0.1356 (profiles/r04 session r04d)
  return onepass && k <= kMaxK && (!sharded() || peer_on);
}

// The user-side rhs / row sums on the matrix cores (the W block) from NB =
// MR_RHSM_MIN_NB up (A/B knob; below it they stay on the VALU)
#ifndef MR_RHSM_MIN_NB
#define MR_RHSM_MIN_NB 5
#endif

// start: the Gram waves also start the CG solve (r0, p0, q0 = G p0 and the
// block pairs of r.r / p.Gp); Engine::cg(started = true) finishes the start.
int Engine::gram(Side& S, bool start) {
  const bool user = S.user;
  const float* F = user ? Vfac : Ufac;
  const float* bias = user ? nullptr : Ubias;
  hipEvent_t a = nullptr;
  const int cls = user ? MR_K_GRAM_USERS : MR_K_GRAM_ITEMS;
  if (tic(cls, -1, &a)) return -1;
  const int zrow = (int)(user ? I : U);
  const CgStart cs = cg_start_of(S);
  if (launch_gram(stream, user, k, S.work, S.n_work, S.idx, S.val, F, bias, zrow,
                  direct_dst(S), slab_dst(S), start ? &cs : nullptr,
                  user && rhs_mfma && w_bf16 && nb16_of(k) >= MR_RHSM_MIN_NB))
    return -1;
  if (toc(cls, -1, a)) return -1;
  if (S.n_split) {
    if (tic(MR_K_SLAB_REDUCE, -1, &a)) return -1;
    if (launch_slab_reduce(stream, user, k, S.split, S.n_split, S.slab, S.rec, direct_dst(S)))
      return -1;
    if (toc(MR_K_SLAB_REDUCE, -1, a)) return -1;
  }
  return 0;
}

int Engine::x_ptrs(Side& S, float** xf, float** xb) {
  if (S.user) {
    *xf = Ufac + S.e0 * ldk;
    *xb = Ubias + S.e0;
  } else {
    *xf = Vfac + S.e0 * ldk;
    *xb = nullptr;
  }
  return 0;
}

// One global CG solve (cg_least_squares, matrix.cpp:456-529) on the side's
// block-diagonal normal equations.  Host protocol: every BETA step publishes
// the CG state to host-mapped memory; iteration t+1 is enqueued before
// iteration t's state is known only when the known state (after t-1) proves
// that t cannot terminate (fails == 0, rr far above 1e-6, t+1 < max_it) --
// so the stream stays busy without launching iterations that would be idle.
int Engine::cg(Side& S, double min_dec, int max_it, double* final_rr, bool started,
               Inflight* deferred) {
  if (onepass_for(S))
    return cg_onepass(S, min_dec, max_it, final_rr, started, deferred);
  float *xf, *xb;
  x_ptrs(S, &xf, &xb);
  const bool user = S.user;
  const int mv_cls = user ? MR_K_MATVEC_USERS : MR_K_MATVEC_ITEMS;
  const int64_t n = S.E * ldk;
  const int64_t nb = user ? S.E : 0;
  const size_t pend0 = pending.size();
  // peer all-reduce: the scalars are exchanged inside the finalizing thread,
  // so the CG runs the unsharded launch protocol (no collective launches)
  const bool shard = sharded() && !peer_on;
  memset(h_init, 0, sizeof(CgState));
  h_init->min_dec = min_dec;
  h_init->max_it = max_it;
  h_init->sharded = shard ? 1 : 0;
  h_init->peer = peer_on ? d_peer : nullptr;
  // The control steps run in the last-arriving block of the matvec (alpha)
  // and of the update (INIT / BETA rules + publish): two kernels per
  // iteration.  Sharded runs: those blocks only sum the local partials into
  // the state slot, RCCL all-reduces it, the update derives alpha from the
  // reduced slot itself, and a one-block finalize applies the INIT / BETA
  // rules -- three kernels and two all-reduces per iteration.
  CgState* fst = d_state;
  hipEvent_t a = nullptr;
  const int seq_init = ++mirror_seq;
  if (started) {
    // The Gram waves already formed r0, p0 = -r0 and q0 = G p0 with block
    // pairs of (r0.r0, p0.q0); split entities follow here, then one control
    // block applies the INIT rule and alpha of iteration 0 (CG_START).
    if (S.n_split) {
      const CgStart cs = cg_start_of(S);
      if (tic(MR_K_CG_START, -1, &a)) return -1;
      if (launch_cg_start_split(stream, user, k, S.split, S.n_split, direct_dst(S), cs,
                                S.start_parts + 3 * gram_blocks(S.n_work, k)))
        return -1;
      if (toc(MR_K_CG_START, -1, a)) return -1;
    }
    const int np = (int)S.n_start_pairs;
    if (tic(MR_K_CG_CONTROL, -1, &a)) return -1;
    if (shard) {
      if (launch_cg_control(stream, d_state, CG_START, CTL_REDUCE, S.start_parts, np) ||
          allreduce_state_slot(2) ||
          launch_cg_control(stream, d_state, CG_START, CTL_FINALIZE, S.start_parts, np,
                            d_mirror, seq_init, min_dec, max_it, 1))
        return -1;
    } else if (launch_cg_control(stream, d_state, CG_START, CTL_BOTH, S.start_parts, np,
                                 d_mirror, seq_init, min_dec, max_it, 0)) {
      return -1;
    }
    if (toc(MR_K_CG_CONTROL, -1, a)) return -1;
  } else {
    MR_HIP(hipMemcpyAsync(d_state, h_init, sizeof(CgState), hipMemcpyHostToDevice, stream));
    // r0 = G x - c ; p0 = -r0 ; rr  (matrix.cpp:464-485): p holds x in fp64
    // for the matvec, which forms q = G x; the INIT update overwrites p
    if (launch_x_to_vec(stream, n, nb, xf, xb, S.p, S.pb)) return -1;
    if (tic(mv_cls, -1, &a)) return -1;
    if (launch_cg_matvec(stream, user, d_state, 0, S.E, k, S.G, S.Gs, S.Gn, S.p, S.pb,
                         S.r, S.rb, S.q, S.qb, partials, S.n_part_mv))
      return -1;
    if (toc(mv_cls, -1, a)) return -1;
    if (tic(MR_K_CG_UPDATE, -1, &a)) return -1;
    if (launch_cg_update(stream, d_state, UPD_INIT, n, nb, xf, S.r, S.p, S.q, S.C, xb,
                         S.rb, S.pb, S.qb, S.Cb, partials, kUpdParts, fst, d_mirror, seq_init))
      return -1;
    if (toc(MR_K_CG_UPDATE, -1, a)) return -1;
    cur_parts = kUpdParts;
    if (shard && finalize_sharded(CG_INIT, seq_init)) return -1;
  }

  std::vector<int> seq_of;   // publish seq of iteration t's BETA step
  // One CG iteration t = head(t) + tail(t):
  //   head(t): matvec (skipped for t = 0 after a fused start), sharded: its
  //            p.Ap all-reduce; with sharding the matvec of t >= 1 also
  //            applies and publishes the BETA step of t-1 (no finalize)
  //   tail(t): update (+ BETA / publish in its last block when unsharded),
  //            sharded: its r.r all-reduce
  // Heads and tails are always enqueued alternately.
  int heads = 0, tails = 0;
  auto launch_head = [&]() -> int {
    const int t = heads++;
    if (started && t == 0) return 0;   // a fused start has done iteration 0's matvec
    hipEvent_t ev = nullptr;
    if (tic(mv_cls, t, &ev)) return -1;
    const int bseq = (shard && t > 0) ? seq_of[t - 1] : 0;
    if (launch_cg_matvec(stream, user, d_state, t > 0, S.E, k, S.G, S.Gs, S.Gn, S.p, S.pb,
                         S.r, S.rb, S.q, S.qb, partials, S.n_part_mv, fst, CG_ALPHA,
                         d_mirror, bseq))
      return -1;
    if (toc(mv_cls, t, ev)) return -1;
    cur_parts = S.n_part_mv;
    return shard ? allreduce_state_slot() : 0;
  };
  auto launch_tail = [&]() -> int {
    const int t = tails++;
    hipEvent_t ev = nullptr;
    seq_of.push_back(++mirror_seq);
    if (tic(MR_K_CG_UPDATE, t, &ev)) return -1;
    if (launch_cg_update(stream, d_state, UPD_STEP, n, nb, xf, S.r, S.p, S.q, S.C, xb, S.rb,
                         S.pb, S.qb, S.Cb, partials, kUpdParts, fst, d_mirror, seq_of.back()))
      return -1;
    if (toc(MR_K_CG_UPDATE, t, ev)) return -1;
    cur_parts = kUpdParts;
    return shard ? allreduce_state_slot() : 0;
  };
  // Enqueue the alternating sequence until `nh` heads are out (tails follow
  // their heads; no tail past max_it - 1, no head past max_it).
  auto enqueue_to = [&](int nh) -> int {
    while (heads < nh && heads <= max_it) {
      if (tails < heads) {
        if (tails >= max_it) break;
        if (launch_tail()) return -1;
      }
      if (heads <= tails && launch_head()) return -1;
    }
    return 0;
  };
  // State t is published by tail(t) unsharded, by head(t+1) sharded.
  const int lag = shard ? 1 : 0;
  auto enqueue_iterations = [&](int n_it) -> int {   // iterations 0 .. n_it-1 complete
    if (enqueue_to(n_it)) return -1;
    while (tails < n_it && tails < max_it)
      if (launch_tail()) return -1;
    return 0;
  };

  // Host protocol.  Iteration t publishes the state after it (its BETA step)
  // under seq_of[t]; the host always reads the state of an EXACT iteration
  // (ring slot), so every decision below is a function of states that are
  // bitwise identical on all ranks of a sharded run (they derive from the
  // all-reduced scalars): every rank issues the same launches, and with them
  // the same collectives.  Iteration 0 cannot stop by stagnation (fails
  // starts at 0), so iterations 0 and 1 are enqueued behind the start without
  // waiting (no-ops if the start already finished the solve).  Afterwards,
  // with the exact state S after iteration t known and not done:
  //   * iteration t+1 is in flight (launched if it was not), and so is what
  //     publishes its state (sharded: the head of t+2);
  //   * iteration t+2 is enqueued too when S proves t+1 cannot stop
  //     (fails == 0, rr far above 1e-6, t+2 < max_it) -- the stream stays
  //     busy while the host waits for the state after t+1.
  const int spec = speculate;
  if (enqueue_iterations(std::min(spec ? 2 : 1, max_it))) return -1;
  CgMirror ms{};
  if (wait_mirror(seq_init, &ms)) return -1;
  int known = -1;            // ms = exact state after iteration `known` (-1: the start)
  while (!ms.done) {
    if (enqueue_iterations(known + 2)) return -1;
    if (spec && known + 2 < max_it &&
        (spec >= 2 || (ms.fails == 0 && ms.rr > 1e-4))) {
      if (enqueue_iterations(known + 3)) return -1;
    }
    if (lag && enqueue_to(known + 3)) return -1;   // the publisher of state known+1
    if (wait_mirror(seq_of[known + 1], &ms)) return -1;
    ++known;
    MR_CHECK(known <= max_it, "CG did not terminate");
  }
  for (size_t i = pend0; i < pending.size(); ++i) pending[i].n_real = ms.n_matvec;
  MR_CHECK(ms.ret >= 0, "peer all-reduce of the CG scalars timed out (a rank did not arrive)");
  if (final_rr) *final_rr = ms.final_rr;
  return ms.ret;
}

// One-pass CG (DESIGN.md "One-pass CG iteration"): the same solve as cg()
// with ONE kernel per CG iteration (cg_onepass_kernel: the previous
// iteration's deferred x / r update, p, q = G p and the four sums whose last
// block takes alpha, r'.r' and the BETA rule, and publishes) and a finish
// launch that applies the last iteration's update after the stop.  The
// state after iteration t is published by kernel t (by the CG_START control
// for t = 0 after a fused start); launch decisions follow exact published
// states as in cg().  Unsharded, or sharded with the peer all-reduce (every
// reduction happens in a last block, so ranks issue identical launches).
int Engine::cg_onepass(Side& S, double min_dec, int max_it, double* final_rr, bool started,
                       Inflight* deferred) {
  float *xf, *xb;
  x_ptrs(S, &xf, &xb);
  const bool user = S.user;
  const int mv_cls = user ? MR_K_MATVEC_USERS : MR_K_MATVEC_ITEMS;
  const int64_t n = S.E * ldk;
  const int64_t nb = user ? S.E : 0;
  const size_t pend0 = pending.size();
  memset(h_init, 0, sizeof(CgState));
  h_init->min_dec = min_dec;
  h_init->max_it = max_it;
  h_init->peer = peer_on ? d_peer : nullptr;
  h_init->onepass = 1;
  hipEvent_t a = nullptr;
  std::vector<int> seq_of;   // publish seq of the state after iteration t
  int launched = 0;          // iteration kernels enqueued (t = 0 .. launched-1)
  CgMirror ms{};
  if (started) {
    // INIT rule, alpha_0 and iteration 0's BETA step (its update deferred):
    // by the last block of the split entities' start when there are any
    // (the CG_START control folded in, one launch less), else by the control
    seq_of.push_back(++mirror_seq);
    const CgStart cs = cg_start_of(S);
    if (S.n_split && cs.xbins) {
      StartFold fold{d_state, d_mirror, seq_of[0], min_dec, max_it, 2};
      if (tic(MR_K_CG_START, -1, &a)) return -1;
      if (launch_cg_start_split(stream, user, k, S.split, S.n_split, direct_dst(S), cs,
                                S.start_parts + 3 * gram_blocks(S.n_work, k), fold))
        return -1;
      if (toc(MR_K_CG_START, -1, a)) return -1;
    } else {
      if (tic(MR_K_CG_CONTROL, -1, &a)) return -1;
      if (launch_cg_control(stream, d_state, CG_START, CTL_BOTH, S.start_parts,
                            (int)S.n_start_pairs, d_mirror, seq_of[0], min_dec, max_it, 2,
                            xbins + kXBinWords))
        return -1;
      if (toc(MR_K_CG_CONTROL, -1, a)) return -1;
    }
    launched = 1;
  } else {
    MR_HIP(hipMemcpyAsync(d_state, h_init, sizeof(CgState), hipMemcpyHostToDevice, stream));
    // r0 = G x - c ; p0 = -r0 ; rr (matrix.cpp:464-485), as in cg()
    if (launch_x_to_vec(stream, n, nb, xf, xb, S.p, S.pb)) return -1;
    if (tic(mv_cls, -1, &a)) return -1;
    if (launch_cg_matvec(stream, user, d_state, 0, S.E, k, S.G, S.Gs, S.Gn, S.p, S.pb, S.r,
                         S.rb, S.q, S.qb, partials, S.n_part_mv))
      return -1;
    if (toc(mv_cls, -1, a)) return -1;
    const int seq_init = ++mirror_seq;
    if (tic(MR_K_CG_UPDATE, -1, &a)) return -1;
    if (launch_cg_update(stream, d_state, UPD_INIT, n, nb, xf, S.r, S.p, S.q, S.C, xb, S.rb,
                         S.pb, S.qb, S.Cb, partials, kUpdParts, d_state, d_mirror, seq_init))
      return -1;
    if (toc(MR_K_CG_UPDATE, -1, a)) return -1;
    if (!resident_for(S)) {
      if (wait_mirror(seq_init, &ms)) return -1;
      MR_CHECK(ms.ret >= 0, "peer all-reduce of the CG scalars timed out (a rank did not arrive)");
    }
  }
  if (resident_for(S)) {
    // every iteration and the finish in one launch (DESIGN.md "Resident CG
    // solve"); it publishes the final state under its own sequence number
    const bool nt = tile_nt_for(S);
    const int seq = ++mirror_seq;
    const int cls = user ? MR_K_CG_RES_USERS : MR_K_CG_RES_ITEMS;
    if (tic(cls, -1, &a)) return -1;
    if (launch_cg_resident(stream, user, d_resctl, started ? 1 : 0, sweep, S.E, k, S.G, S.Gs,
                           S.Gn, S.p, S.pb, S.r, S.rb, S.q, S.qb, xf, xb, S.n_part_rs[nt ? 1 : 0],
                           seq, nt))
      return -1;
    if (toc(cls, -1, a)) return -1;
    const long long pend = timing ? (long long)pending.size() - 1 : -1;
    if (deferred) {   // read back later (Engine::drain)
      *deferred = Inflight{seq, user, started, pend};
      return 0;
    }
    if (wait_mirror(seq, &ms)) return -1;
    MR_CHECK(ms.ret >= 0, "peer all-reduce of the CG scalars timed out (a rank did not arrive)");
    // its CG iterations (a fused start did iteration 0's matvec itself)
    if (pend >= 0) pending[pend].units = ms.n_matvec - (started && ms.n_matvec > 0 ? 1 : 0);
    if (final_rr) *final_rr = ms.final_rr;
    return ms.ret;
  }
  auto launch_iter = [&](int t) -> int {
    seq_of.push_back(++mirror_seq);
    hipEvent_t ev = nullptr;
    if (tic(mv_cls, t, &ev)) return -1;
    // sweep 1: iteration 1 (the first kernel behind a fused start) runs
    // backwards over the entities the Gram just wrote, then alternate
    const int rev = sweep == 0 ? 0 : ((t & 1) ^ (sweep == 2 ? 1 : 0));
    if (launch_cg_onepass(stream, user, d_state, t > 0 ? 1 : 0, rev, S.E, k, S.G, S.Gs, S.Gn, S.p,
                          S.pb, S.r, S.rb, S.q, S.qb, xf, xb, xbins, S.n_part_op[tile_nt_for(S) ? 1 : 0],
                          d_mirror, seq_of.back(), tile_nt_for(S)))
      return -1;
    return toc(mv_cls, t, ev);
  };
  auto enqueue_to = [&](int nt) -> int {   // iterations 0 .. nt-1 enqueued
    while (launched < std::min(nt, max_it))
      if (launch_iter(launched++)) return -1;
    return 0;
  };
  const int spec = speculate;
  int known = -1;   // ms = the exact state after iteration `known`
  if (started || !ms.done) {
    while (true) {
      // iteration known+1 is what publishes the next state; with the state
      // after `known` proving known+1 cannot stop, known+2 goes out too
      int ahead = known + 2;
      if (spec && known >= 0 && known + 2 < max_it &&
          (spec >= 2 || (ms.fails == 0 && ms.rr > 1e-4)))
        ahead = known + 3;
      if (enqueue_to(ahead)) return -1;
      MR_CHECK(known + 1 < (int)seq_of.size(), "CG did not terminate");
      if (wait_mirror(seq_of[known + 1], &ms)) return -1;
      ++known;
      MR_CHECK(ms.ret >= 0, "peer all-reduce of the CG scalars timed out (a rank did not arrive)");
      if (ms.done) break;
    }
  }
  // the stopped iteration's x / r update (pending flag checked on the device)
  if (tic(MR_K_CG_UPDATE, -1, &a)) return -1;
  if (launch_cg_update(stream, d_state, UPD_FINISH, n, nb, xf, S.r, S.p, S.q, S.C, xb, S.rb,
                       S.pb, S.qb, S.Cb, partials, kUpdParts))
    return -1;
  if (toc(MR_K_CG_UPDATE, -1, a)) return -1;
  for (size_t i = pend0; i < pending.size(); ++i) pending[i].n_real = ms.n_matvec;
  if (final_rr) *final_rr = ms.final_rr;
  return ms.ret;
}

int Engine::solve(Side& S) {
  float *xf, *xb;
  x_ptrs(S, &xf, &xb);
  MR_HIP(hipMemsetAsync(d_flag, 0, 4, stream));
  hipEvent_t a = nullptr;
  if (tic(MR_K_SOLVE, -1, &a)) return -1;
  if (launch_solve(stream, S.user, S.E, k, ridge, S.G, S.Gs, S.Gn, S.C, S.Cb, xf, xb,
                   d_flag))
    return -1;
  if (toc(MR_K_SOLVE, -1, a)) return -1;
  int bad = 0;
  MR_D2H(&bad, d_flag, 4, stream);
  MR_HIP(hipStreamSynchronize(stream));
  if (S.user) stats.nonpd_users += bad;
  else stats.nonpd_items += bad;
  return 0;
}

int Engine::half_step(bool user, double min_dec, int max_it, double* final_rr) {
  MR_HIP(hipSetDevice(device));
  Side& S = user ? su : si;
  // a deferred solve (iterate) may only ride ahead of half-steps that
  // report nothing: the caller of this one wants its count
  Inflight dfr{-1, user, false, -1};
  const bool may_defer = defer && !final_rr && solver == MR_SOLVER_CG && resident_for(S);
  if (may_defer) {
    if (drain(kMaxInflight - 1)) return -1;
  } else if (drain()) {
    return -1;
  }
  const size_t g0 = pending.size();
  // the CG start rides on the MFMA Gram's accumulators (32 <= k <= 128)
  const bool fused = solver == MR_SOLVER_CG && fuse_start && k >= kMfmaMinK && k <= kMaxK;
  if (gram(S, fused)) return -1;
  const size_t c0 = pending.size();
  int its = 0;
  double rr = 0.0;
  if (solver == MR_SOLVER_CG) {
    its = cg(S, min_dec, max_it, &rr, fused, may_defer ? &dfr : nullptr);
    if (its < 0) return -1;
  } else {
    if (solve(S)) return -1;
  }
  if (allgather_side(user)) return -1;
  if (timing) {
    hipEvent_t end = nullptr;
    if (sharded()) {   // the RCCL exchange belongs to the solve phase
      if (ev_get(&end)) return -1;
      MR_HIP(hipEventRecord(end, stream));
    }
    spans.push_back({user ? 0 : 2, g0, c0, nullptr});
    spans.push_back({user ? 1 : 3, c0, pending.size(), end});
  }
  if (dfr.seq > 0) {
    inflight.push_back(dfr);
    return 0;
  }
  if (timing && pending.size() > 8192 && resolve_timing()) return -1;
  count_solve(user, its, rr);
  if (final_rr) *final_rr = rr;
  return its;
}

void Engine::count_solve(bool user, int its, double rr) {
  if (user) {
    stats.last_cg_users = its;
    stats.cg_users_total += its;
  } else {
    stats.last_cg_items = its;
    stats.cg_items_total += its;
    stats.last_final_rr = rr;
  }
}

int Engine::drain(size_t keep) {
  while (inflight.size() > keep) {
    const Inflight d = inflight.front();
    inflight.erase(inflight.begin());
    CgMirror ms{};
    if (wait_mirror(d.seq, &ms)) return -1;
    MR_CHECK(ms.ret >= 0, "peer all-reduce of the CG scalars timed out (a rank did not arrive)");
    if (d.pend >= 0 && d.pend < (long long)pending.size())
      pending[d.pend].units = ms.n_matvec - (d.started && ms.n_matvec > 0 ? 1 : 0);
    count_solve(d.user, ms.ret, ms.final_rr);
  }
  return 0;
}

// The reference outer loop (matrix.cpp:810-892).  The user half-step uses
// cg_least_squares' defaults (0.01, 200) as at :818; the item half-step passes
// (0.01, 200, &rr) as at :854; min_r_decrease only drives the outer test.
int Engine::run(double min_dec, int max_it) {
  if (drain()) return -1;
  int it = 0;
  double old_rr = 0.0;
  while (it < max_it) {
    if (half_step(true, 0.01, 200, nullptr) < 0) return -1;
    double rr = 0.0;
    if (half_step(false, 0.01, 200, &rr) < 0) return -1;
    stats.iterations += 1;
    if (it >= 3) {
      const double decrease = (old_rr - rr) / old_rr;
      if (decrease < min_dec) return it;
    }
    old_rr = rr;
    ++it;
  }
  return it;
}

// Exactly n iterations; nothing is reported per half-step, so resident
// solves are read back lazily (at most kMaxInflight in flight: the stream
// always holds the next half-step while the host waits for a solve); the
// next call that reads anything drains them.
int Engine::iterate(int n) {
  defer = true;
  int rc = 0;
  for (int i = 0; i < n && rc == 0; ++i) {
    if (half_step(true, 0.01, 200, nullptr) < 0 || half_step(false, 0.01, 200, nullptr) < 0)
      rc = -1;
    else
      stats.iterations += 1;
  }
  defer = false;
  if (rc) (void)drain();
  return rc;
}

int Engine::predict(int64_t n, const int* uid, const int* iid, double* out) {
  if (drain()) return -1;
  MR_HIP(hipSetDevice(device));
  int *du = nullptr, *di = nullptr;
  double* dout = nullptr;
  if (dalloc(&du, n, stream) || dalloc(&di, n, stream) || dalloc(&dout, n, stream)) return -1;
  if (n > 0) {
    MR_H2D(du, uid, n * 4, stream);
    MR_H2D(di, iid, n * 4, stream);
    MR_HIP(hipMemsetAsync(d_flag, 0, 8, stream));
    if (launch_validate_ids(stream, n, du, 0, (int32_t)U, d_flag)) return -1;
    if (launch_validate_ids(stream, n, di, 0, (int32_t)I, d_flag + 1)) return -1;
    int flags[2];
    MR_D2H(flags, d_flag, 8, stream);
    MR_HIP(hipStreamSynchronize(stream));
    MR_CHECK(!flags[0] && !flags[1], "predict: id out of range");
    if (launch_predict(stream, n, k, ldk, du, di, Ufac, Ubias, Vfac, dout)) return -1;
    MR_D2H(out, dout, n * 8, stream);
  }
  MR_HIP(hipStreamSynchronize(stream));
  dfree(du, stream); dfree(di, stream); dfree(dout, stream);
  return 0;
}

int Engine::get_normal_equations(bool user, int n, const int* ents, double* G, double* c) {
  if (drain()) return -1;
  MR_HIP(hipSetDevice(device));
  Side& S = user ? su : si;
  const int K = user ? k + 1 : k;
  const int nb = nb16_of(k);
  std::vector<float> g(gsize_of(k)), v(ldk), s(ldk);
  float cb = 0.f, gn = 0.f;
  for (int t = 0; t < n; ++t) {
    const int64_t e = ents[t];
    MR_CHECK(e >= 0 && e < S.E, "entity out of range");
    MR_D2H(g.data(), S.G + e * gsize_of(k), gsize_of(k) * 4, stream);
    MR_D2H(v.data(), S.C + e * ldk, ldk * 4, stream);
    if (user) {
      MR_D2H(s.data(), S.Gs + e * ldk, ldk * 4, stream);
      MR_D2H(&cb, S.Cb + e, 4, stream);
      MR_D2H(&gn, S.Gn + e, 4, stream);
    }
    MR_HIP(hipStreamSynchronize(stream));
    double* Ge = G + (size_t)t * K * K;
    double* ce = c + (size_t)t * K;
    for (int i = 0; i < K; ++i) {
      for (int j = 0; j < K; ++j) {
        double val;
        if (i < k && j < k) {
          val = g[packed_offset(i, j, nb)];
        } else if (i < k) val = s[i];
        else if (j < k) val = s[j];
        else val = gn;
        Ge[i * K + j] = val;
      }
      ce[i] = i < k ? v[i] : cb;
    }
  }
  return 0;
}

// The side's device CSR and Gram work list, for tests (a full-size check that
// the context build -- uploads, device sort, offsets, work list -- landed
// exactly).  Any pointer may be NULL.
int Engine::get_layout(bool user, long long* off, int* idx, float* val, long long* wbegin,
                       int* wlen, int* went, int* wslab) {
  MR_HIP(hipSetDevice(device));
  Side& S = user ? su : si;
  if (off) {
    std::vector<int64_t> o(S.E + 1);
    MR_D2H(o.data(), S.off, o.size() * 8, stream);
    for (int64_t e = 0; e <= S.E; ++e) off[e] = o[e];
  }
  if (idx) MR_D2H(idx, S.idx, S.nnz * 4, stream);
  if (val) MR_D2H(val, S.val, S.nnz * 4, stream);
  if (wbegin || wlen || went || wslab) {
    std::vector<WorkItem> w(S.n_work);
    MR_D2H(w.data(), S.work, w.size() * sizeof(WorkItem), stream);
    for (int64_t t = 0; t < S.n_work; ++t) {
      if (wbegin) wbegin[t] = w[t].begin;
      if (wlen) wlen[t] = w[t].len;
      if (went) went[t] = w[t].entity;
      if (wslab) wslab[t] = w[t].slab;
    }
  }
  return 0;
}

// CG vectors r, p, q of the side as left by the last solve (K = k+1 per user
// with the bias entry last, k per item), for tests.
int Engine::get_cg_vectors(bool user, double* r, double* p, double* q) {
  if (drain()) return -1;
  MR_HIP(hipSetDevice(device));
  Side& S = user ? su : si;
  const int K = user ? k + 1 : k;
  std::vector<double> v(S.E * ldk), b(user ? S.E : 0);
  double* outs[3] = {r, p, q};
  double* vecs[3] = {S.r, S.p, S.q};
  double* bvs[3] = {S.rb, S.pb, S.qb};
  for (int t = 0; t < 3; ++t) {
    if (!outs[t]) continue;
    MR_D2H(v.data(), vecs[t], v.size() * 8, stream);
    if (user) MR_D2H(b.data(), bvs[t], b.size() * 8, stream);
    MR_HIP(hipStreamSynchronize(stream));
    for (int64_t e = 0; e < S.E; ++e) {
      for (int j = 0; j < k; ++j) outs[t][e * K + j] = v[e * ldk + j];
      if (user) outs[t][e * K + k] = b[e];
    }
  }
  return 0;
}

}  // namespace mr
