// qd_runtime.hip — error reporting, device selection and the per-device
// workspace cache of libqdyn.
#include "qd_common.hpp"

#include <mutex>
#include <set>
#include <vector>

namespace qd {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Scratch is call-scoped: every workspace() call gets a stream-ordered buffer of the device's default memory pool
// (release threshold = max, so the pool keeps what is released reserved), live until the enclosing WsScope (one per
// entry point) ends.  At the end of a scope its buffers are PARKED for reuse rather than released: hipFreeAsync on
// this ROCm blocks the host until the stream has drained the work queued so far (median 1.1 ms, one 2DES grid, in the
// HIP API trace of profiles/r04/2des/hipfree_block.txt), which made every library call synchronous in effect (the
// bench's 2DES leg: 1.19 -> 0.035 ms of host time per grid, profiles/r04/2des/ws_park_ab.txt).  A parked buffer is
//   - reused by a later workspace() request on the SAME stream (stream order puts the new user behind every kernel
//     of the old one; the park happens after the old call queued its last kernel), the smallest parked buffer of at
//     least the requested size and at most 4x it;
//   - released when more than WS_PARK_CAP bytes are parked (first the buffers of other streams whose last users
//     have completed, by the event recorded behind them, then the oldest of the current stream), and, once their
//     last users have completed, by qd_workspace_stats and qd_shutdown.
// So two live calls never share scratch (a buffer is live for one call; parked buffers are shared by the host
// threads under g_park_mu), the reservation stays bounded by the peak concurrent use plus WS_PARK_CAP (not by the
// number of streams ever seen), and qd_workspace_stats reports nothing in use once the work has completed.
struct LiveBuf {
  void* ptr;
  size_t bytes;
  hipStream_t st;
};
struct ParkedBuf {
  void* ptr;
  size_t bytes;
  hipStream_t st;
  hipEvent_t done;   // recorded on st behind the buffer's last user
};
static thread_local std::vector<LiveBuf> g_live;
static std::mutex g_park_mu;                 // guards g_park / g_free_events (shared by every host thread)
static std::vector<ParkedBuf> g_park;
static std::vector<hipEvent_t> g_free_events;
static thread_local int g_depth = 0;
static std::mutex g_pool_mu;
static std::set<int> g_pool_ready;
static constexpr size_t WS_PARK_CAP = (size_t)8 << 30;

static int ensure_pool(int dev) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool_ready.count(dev)) return QD_OK;
  hipMemPool_t pool;
  QD_HIP(hipDeviceGetDefaultMemPool(&pool, dev));
  uint64_t thr = UINT64_MAX;
  QD_HIP(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
  g_pool_ready.insert(dev);
  return QD_OK;
}

static hipEvent_t take_event() {
  if (!g_free_events.empty()) {
    hipEvent_t e = g_free_events.back();
    g_free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

// release parked buffer k (its last user has completed, or `on` orders the release behind it: same stream)
static void release_parked(size_t k, hipStream_t on) {
  ParkedBuf b = g_park[k];
  g_park.erase(g_park.begin() + (long)k);
  (void)hipFreeAsync(b.ptr, on);
  if (b.done) g_free_events.push_back(b.done);
}

static bool parked_done(const ParkedBuf& b) { return !b.done || hipEventQuery(b.done) == hipSuccess; }

WsScope::WsScope(hipStream_t s) : st(s), mark(g_live.size()) { ++g_depth; }

WsScope::~WsScope() {
  std::lock_guard<std::mutex> lk(g_park_mu);
  // park this scope's buffers behind an event on their stream (every kernel that uses them is queued by now)
  for (size_t k = g_live.size(); k > mark; --k) {
    const LiveBuf& b = g_live[k - 1];
    hipEvent_t e = take_event();
    if (e && hipEventRecord(e, b.st) != hipSuccess) {
      g_free_events.push_back(e);
      e = nullptr;
    }
    if (!e) {   // no event: the old stream-ordered release
      (void)hipFreeAsync(b.ptr, b.st);
      continue;
    }
    g_park.push_back({b.ptr, b.bytes, b.st, e});
  }
  g_live.resize(mark);
  // bound what stays parked: first the buffers of other streams whose last users have completed (idle
  // memory, released on the null stream: their own stream may have been destroyed since), then the oldest of this
  // stream (ordered behind their users on it)
  size_t tot = 0;
  for (const ParkedBuf& b : g_park) tot += b.bytes;
  for (size_t k = g_park.size(); tot > WS_PARK_CAP && k-- > 0;)
    if (g_park[k].st != st && parked_done(g_park[k])) {
      tot -= g_park[k].bytes;
      release_parked(k, nullptr);
    }
  for (size_t k = 0; k < g_park.size() && tot > WS_PARK_CAP;) {
    if (g_park[k].st == st) {
      tot -= g_park[k].bytes;
      release_parked(k, st);
    } else {
      ++k;
    }
  }
  --g_depth;
}

int workspace(WsSlot slot, size_t bytes, void** ptr, hipStream_t st) {
  (void)slot;  // the slot names the buffer's role; every call gets its own buffer
  if (g_depth <= 0) {
    set_error("internal: workspace() outside a WsScope");
    return QD_EINVAL;
  }
  if (bytes == 0) bytes = 16;
  // a buffer parked on the same stream: the smallest of at least `bytes` and at most 4x that
  std::unique_lock<std::mutex> lk(g_park_mu);
  size_t best = g_park.size();
  for (size_t k = 0; k < g_park.size(); ++k) {
    const ParkedBuf& b = g_park[k];
    if (b.st == st && b.bytes >= bytes && b.bytes / 4 <= bytes && (best == g_park.size() || b.bytes < g_park[best].bytes))
      best = k;
  }
  if (best < g_park.size()) {
    ParkedBuf b = g_park[best];
    g_park.erase(g_park.begin() + (long)best);
    if (b.done) g_free_events.push_back(b.done);
    g_live.push_back({b.ptr, b.bytes, st});
    *ptr = b.ptr;
    return QD_OK;
  }
  lk.unlock();
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  int rc = ensure_pool(dev);
  if (rc) return rc;
  void* p = nullptr;
  hipError_t e = hipMallocAsync(&p, bytes, st);
  if (e != hipSuccess) {
    set_error("workspace allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return QD_ENOMEM;
  }
  g_live.push_back({p, bytes, st});
  *ptr = p;
  return QD_OK;
}

// parked buffers whose last users have completed go back to the pool (all of them after a device synchronisation
// when `all`)
void release_parked_workspaces(bool all) {
  if (all) (void)hipDeviceSynchronize();
  std::lock_guard<std::mutex> lk(g_park_mu);
  bool any = false;
  for (size_t k = g_park.size(); k-- > 0;)
    if (all || parked_done(g_park[k])) {
      release_parked(k, nullptr);
      any = true;
    }
  if (any) (void)hipStreamSynchronize(nullptr);
}

void free_workspaces() {
  release_parked_workspaces(true);
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (int dev : g_pool_ready) {
    hipMemPool_t pool;
    (void)hipSetDevice(dev);
    (void)hipDeviceSynchronize();
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
  }
  (void)hipSetDevice(cur);
}

int pool_stats(size_t* reserved, size_t* used) {
  release_parked_workspaces(false);
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  hipMemPool_t pool;
  QD_HIP(hipDeviceGetDefaultMemPool(&pool, dev));
  uint64_t r = 0, u = 0;
  QD_HIP(hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemCurrent, &r));
  QD_HIP(hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, &u));
  if (reserved) *reserved = (size_t)r;
  if (used) *used = (size_t)u;
  return QD_OK;
}

}  // namespace qd

extern "C" {

int qd_version(void) { return 100; }

const char* qd_last_error(void) { return qd::g_err; }

int qd_device_count(int* count) {
  QD_CHECK_ARG(count != nullptr, "qd_device_count: null pointer");
  QD_HIP(hipGetDeviceCount(count));
  return QD_OK;
}

int qd_init(int device) {
  int n = 0;
  QD_HIP(hipGetDeviceCount(&n));
  QD_CHECK_ARG(device >= 0 && device < n, "qd_init: device %d out of range (%d devices)", device, n);
  QD_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  QD_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    qd::set_error("qd_init: libqdyn is built for gfx950 only, device %d is %s", device,
                  prop.gcnArchName);
    return QD_EINVAL;
  }
  return QD_OK;
}

int qd_shutdown(void) {
  qd::free_workspaces();
  return QD_OK;
}

int qd_workspace_stats(size_t* reserved, size_t* used) { return qd::pool_stats(reserved, used); }

int qd_synchronize(void* stream) {
  QD_HIP(hipStreamSynchronize((hipStream_t)stream));
  return QD_OK;
}

}  // extern "C"
