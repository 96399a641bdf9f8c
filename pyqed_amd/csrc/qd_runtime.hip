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

// Scratch is call-scoped: every workspace() call takes a fresh stream-ordered allocation
// (hipMallocAsync on the call's stream) from the device's default memory pool, and the enclosing
// WsScope (one per entry point) returns it with hipFreeAsync on the same stream once every kernel
// that uses it has been enqueued.  The pool keeps released memory reserved (release threshold =
// max), so steady-state calls sub-allocate without touching the driver, any stream may reuse what
// another stream released (the pool orders the reuse), and the reserved total is bounded by the
// peak CONCURRENT use -- not by the number of streams ever seen.  qd_shutdown trims the pools.
struct LiveBuf {
  void* ptr;
  hipStream_t st;
};
static thread_local std::vector<LiveBuf> g_live;
static thread_local int g_depth = 0;
static std::mutex g_pool_mu;
static std::set<int> g_pool_ready;

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

WsScope::WsScope(hipStream_t s) : st(s), mark(g_live.size()) { ++g_depth; }

WsScope::~WsScope() {
  // stream-ordered release: runs after the work this call queued on `st`
  for (size_t k = g_live.size(); k > mark; --k) (void)hipFreeAsync(g_live[k - 1].ptr, g_live[k - 1].st);
  g_live.resize(mark);
  --g_depth;
}

int workspace(WsSlot slot, size_t bytes, void** ptr, hipStream_t st) {
  (void)slot;  // the slot names the buffer's role; every call gets its own allocation
  if (g_depth <= 0) {
    set_error("internal: workspace() outside a WsScope");
    return QD_EINVAL;
  }
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  int rc = ensure_pool(dev);
  if (rc) return rc;
  void* p = nullptr;
  hipError_t e = hipMallocAsync(&p, bytes ? bytes : 16, st);
  if (e != hipSuccess) {
    set_error("workspace allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return QD_ENOMEM;
  }
  g_live.push_back({p, st});
  *ptr = p;
  return QD_OK;
}

void free_workspaces() {
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
