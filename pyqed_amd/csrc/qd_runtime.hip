// qd_runtime.hip — error reporting, device selection and the per-device
// workspace cache of libqdyn.
#include "qd_common.hpp"

#include <mutex>
#include <vector>

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

static std::mutex g_ws_mu;
// [device][slot]
static std::vector<std::vector<Workspace>> g_ws;

int workspace(WsSlot slot, size_t bytes, void** ptr) {
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_ws_mu);
  if ((int)g_ws.size() <= dev) g_ws.resize(dev + 1, std::vector<Workspace>(WS_NSLOTS));
  Workspace& w = g_ws[dev][slot];
  if (w.bytes < bytes) {
    if (w.ptr) {
      // the previous buffer may still be in use by queued work
      QD_HIP(hipDeviceSynchronize());
      QD_HIP(hipFree(w.ptr));
      w.ptr = nullptr;
      w.bytes = 0;
    }
    size_t want = bytes + bytes / 8;  // grow geometrically-ish
    hipError_t e = hipMalloc(&w.ptr, want);
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
  for (size_t d = 0; d < g_ws.size(); ++d) {
    for (auto& w : g_ws[d]) {
      if (w.ptr) {
        (void)hipSetDevice((int)d);
        (void)hipDeviceSynchronize();
        (void)hipFree(w.ptr);
      }
      w.ptr = nullptr;
      w.bytes = 0;
    }
  }
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
