// Host <-> device copies through pinned staging (Stager, mr_internal.h).
//
// Every caller buffer the library copies (ratings, ids, work lists, factor
// slices, results) is pageable host memory owned by Python / the caller.
// Instead of handing pageable pointers to hipMemcpyAsync -- whose staging is
// the runtime's business and whose completion semantics for pageable memory
// differ between copy sizes -- the library copies through two pinned chunks of
// its own: the host fills chunk b only after the DMA that last read it has
// completed (event), and a D2H result is copied out only after its DMA has
// completed.  The DMA engine reads / writes pinned memory only, and no host
// write can race a copy still in flight.  Both calls return with their DMAs
// complete (context builds and read-backs; nothing on the iteration path).
#include <cstring>

#include "mr_internal.h"

namespace mr {

Stager::~Stager() {
  for (int b = 0; b < 2; ++b)
    if (buf[b]) (void)hipHostFree(buf[b]);
}

int Stager::init() {
  for (int b = 0; b < 2; ++b)
    if (!buf[b]) MR_HIP(hipHostMalloc(&buf[b], kChunk, hipHostMallocDefault));
  return 0;
}

// Events live for one call only: a caller's stream may be destroyed between
// calls, and an event recorded on a destroyed stream cannot be waited on.
namespace {
struct CallEvents {
  hipEvent_t ev[2] = {nullptr, nullptr};
  ~CallEvents() {
    for (auto e : ev)
      if (e) {
        (void)hipEventSynchronize(e);
        (void)hipEventDestroy(e);
      }
  }
  int create() {
    for (auto& e : ev) MR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return 0;
  }
};
}  // namespace

int Stager::h2d(hipStream_t s, void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return 0;
  if (init()) return -1;
  CallEvents ce;
  if (ce.create()) return -1;
  bool used[2] = {false, false};
  int b = 0;
  for (size_t off = 0; off < bytes; off += kChunk, b ^= 1) {
    const size_t n = bytes - off < kChunk ? bytes - off : kChunk;
    if (used[b]) MR_HIP(hipEventSynchronize(ce.ev[b]));   // the DMA that read this chunk is done
    memcpy(buf[b], static_cast<const char*>(src) + off, n);
    MR_HIP(hipMemcpyAsync(static_cast<char*>(dst) + off, buf[b], n, hipMemcpyHostToDevice, s));
    MR_HIP(hipEventRecord(ce.ev[b], s));
    used[b] = true;
  }
  for (int t = 0; t < 2; ++t)
    if (used[t]) MR_HIP(hipEventSynchronize(ce.ev[t]));   // the staging may be reused
  return 0;
}

int Stager::d2h(hipStream_t s, void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return 0;
  if (init()) return -1;
  CallEvents ce;
  if (ce.create()) return -1;
  // chunk i's DMA is issued before chunk i-1 is copied out of its buffer
  size_t pend_off = 0, pend_n = 0;
  int pend_b = -1, b = 0;
  for (size_t off = 0; off < bytes; off += kChunk, b ^= 1) {
    const size_t n = bytes - off < kChunk ? bytes - off : kChunk;
    MR_HIP(hipMemcpyAsync(buf[b], static_cast<const char*>(src) + off, n, hipMemcpyDeviceToHost, s));
    MR_HIP(hipEventRecord(ce.ev[b], s));
    if (pend_b >= 0) {
      MR_HIP(hipEventSynchronize(ce.ev[pend_b]));
      memcpy(static_cast<char*>(dst) + pend_off, buf[pend_b], pend_n);
    }
    pend_b = b;
    pend_off = off;
    pend_n = n;
  }
  MR_HIP(hipEventSynchronize(ce.ev[pend_b]));
  memcpy(static_cast<char*>(dst) + pend_off, buf[pend_b], pend_n);
  return 0;
}

thread_local Stager t_stager;

}  // namespace mr
