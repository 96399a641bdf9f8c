// qd_runtime.hip — error reporting, device selection and the per-device
// workspace cache of libqdyn.
#include "qd_common.hpp"

#include <map>
#include <mutex>
#include <tuple>

namespace qd {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

struct Workspace {
  void* ptr = nullptr;
  size_t bytes = 0;
};

// (device, stream, slot) -> buffer.  See qd_common.hpp: distinct streams never share scratch.
static std::mutex g_ws_mu;
static std::map<std::tuple<int, uintptr_t, int>, Workspace> g_ws;

int workspace(WsSlot slot, size_t bytes, void** ptr, hipStream_t st) {
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Workspace& w = g_ws[std::make_tuple(dev, (uintptr_t)st, (int)slot)];
  if (w.bytes < bytes) {
    if (w.ptr) {
      // stream-ordered release: runs after the work already queued on `st` that uses the buffer,
      // without waiting for it here and without touching other streams
      QD_HIP(hipFreeAsync(w.ptr, st));
      w.ptr = nullptr;
      w.bytes = 0;
    }
    size_t want = bytes + bytes / 8;  // grow geometrically-ish
    hipError_t e = hipMallocAsync(&w.ptr, want, st);
    if (e != hipSuccess) {
      w.ptr = nullptr;
      set_error("workspace allocation of %zu bytes failed: %s", want, hipGetErrorString(e));
      return QD_ENOMEM;
    }
    w.bytes = want;
  }
  *ptr = w.ptr;
  return QD_OK;
}

void free_workspaces() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& kv : g_ws) {
    Workspace& w = kv.second;
    if (w.ptr) {
      // the owning stream may already be destroyed: wait for the device, then free
      (void)hipSetDevice(std::get<0>(kv.first));
      (void)hipDeviceSynchronize();
      (void)hipFree(w.ptr);
    }
  }
  g_ws.clear();
  (void)hipSetDevice(cur);
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

int qd_synchronize(void* stream) {
  QD_HIP(hipStreamSynchronize((hipStream_t)stream));
  return QD_OK;
}

}  // extern "C"
