// qd_runtime.hip — error reporting, device selection and the library's scratch arena.
#include "qd_common.hpp"

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

namespace qd {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Scratch arena.  Every entry point that needs scratch opens a WsScope on its stream; workspace() hands it a SLAB
// (a plain hipMalloc buffer kept by the library) that no other live call holds, and the scope's end records the
// slab's `done` event on the call's stream behind the last kernel that uses it.  The next call that takes the slab --
// on any stream, from any host thread -- first queues hipStreamWaitEvent(its stream, done): the reuse is ordered on
// the DEVICE, so no library call waits on the host for earlier work (round 4's hipFreeAsync blocked the host until
// the stream drained, 1.1 ms per 2DES grid: profiles/r04/2des/hipfree_block.txt).  Ordering by event rather than by
// stream identity keeps reuse correct when a stream is destroyed and its handle recycled, and
// no stream-ordered pool is involved (round 4's parked pool buffers faulted under rocprofv3 --pmc).
//   - a request takes the smallest idle slab of at least the request and at most 4x it, else a new one (sizes are
//     rounded up to a power of two >= 64 KiB, so a call sequence of varying sizes settles on a few slabs);
//   - the reservation is bounded by the peak CONCURRENT scratch (two live calls never share a slab) -- not by the
//     number of streams seen -- plus idle slabs, which are released (hipFree) once more than kIdleCap bytes are
//     cached and the event says their last user has completed, on allocation failure, and by qd_shutdown.
struct Slab {
  void* ptr;
  size_t bytes;
  int dev;
  hipEvent_t done;   // recorded behind the slab's last user
  bool busy;         // held by a live WsScope
  bool recorded;     // `done` has been recorded at least once
};
struct LiveRef {
  Slab* slab;
  hipStream_t st;
};
static std::mutex g_mu;              // guards g_slabs and every Slab's busy / recorded fields
// Scratch of calls captured into a HIP graph: a plain hipMalloc buffer owned by the GRAPH (a user object retained by
// the graph being captured), since every replay reuses it; the graph's destruction queues it here and the next
// uncaptured workspace() call (or qd_shutdown) frees it.  Stream-ordered graph allocations (hipMallocAsync alloc /
// free nodes) gave non-reproducible replays on this ROCm (profiles/r06/graph/replay_diag.txt).
static std::mutex g_cap_mu;
static std::vector<std::pair<void*, int>> g_cap_dead;
static void cap_release(void* ud) {
  auto* b = static_cast<std::pair<void*, int>*>(ud);
  std::lock_guard<std::mutex> lk(g_cap_mu);
  g_cap_dead.push_back(*b);
  delete b;
}
static void free_dead_capture_buffers() {
  std::vector<std::pair<void*, int>> dead;
  {
    std::lock_guard<std::mutex> lk(g_cap_mu);
    dead.swap(g_cap_dead);
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& d : dead) {
    if (d.second != cur) (void)hipSetDevice(d.second);
    (void)hipFree(d.first);
    if (d.second != cur) (void)hipSetDevice(cur);
  }
}
// hipMalloc while `st` is captured (relaxed capture mode for this thread around the call), owned by the captured graph
static int capture_alloc(size_t bytes, void** ptr, hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(st, &cs, &id, &graph, &deps, &ndeps);
  if (e != hipSuccess || cs != hipStreamCaptureStatusActive || !graph) {
    set_error("workspace inside a graph capture: cannot query the graph being captured (%s)", hipGetErrorString(e));
    return QD_EHIP;
  }
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  void* p = nullptr;
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  e = hipMalloc(&p, bytes);
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  if (e != hipSuccess) {
    set_error("workspace allocation of %zu bytes inside a graph capture failed: %s", bytes, hipGetErrorString(e));
    return QD_ENOMEM;
  }
  auto* ud = new std::pair<void*, int>(p, dev);
  hipUserObject_t obj = nullptr;
  e = hipUserObjectCreate(&obj, ud, cap_release, 1, hipUserObjectNoDestructorSync);
  if (e == hipSuccess) e = hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove);
  if (e != hipSuccess) {
    if (obj) {
      (void)hipUserObjectRelease(obj, 1);   // its destructor queues the buffer for the next uncaptured call's free
    } else {
      delete ud;
      (void)hipFree(p);
    }
    set_error("workspace inside a graph capture: cannot attach the buffer to the graph (%s)", hipGetErrorString(e));
    return QD_EHIP;
  }
  *ptr = p;
  return QD_OK;
}
static std::vector<Slab*> g_slabs;
static thread_local std::vector<LiveRef> g_live;
static thread_local int g_depth = 0;
static constexpr size_t kIdleCapMiB = (size_t)16 << 10;   // QD_OPT_IDLE_CAP_MIB default: 16 GiB of idle slabs
static size_t idle_cap() {
  const int v = option(QD_OPT_IDLE_CAP_MIB);
  return v < 0 ? kIdleCapMiB << 20 : (size_t)v << 20;
}

static size_t slab_size(size_t bytes) {
  size_t s = (size_t)64 << 10;
  while (s < bytes) s <<= 1;
  return s;
}

static bool slab_idle_done(const Slab* s) {
  return !s->busy && (!s->recorded || hipEventQuery(s->done) == hipSuccess);
}

// frees slab k (caller holds g_mu; the slab is idle and its last user has completed)
static void drop_slab(size_t k) {
  Slab* s = g_slabs[k];
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != s->dev) (void)hipSetDevice(s->dev);
  (void)hipFree(s->ptr);
  (void)hipEventDestroy(s->done);
  if (cur != s->dev) (void)hipSetDevice(cur);
  delete s;
  g_slabs.erase(g_slabs.begin() + (long)k);
}

// releases idle, completed slabs until at most `keep` bytes are cached (caller holds g_mu)
static void trim_idle(size_t keep) {
  size_t tot = 0;
  for (const Slab* s : g_slabs) tot += s->bytes;
  for (size_t k = g_slabs.size(); tot > keep && k-- > 0;)
    if (slab_idle_done(g_slabs[k])) {
      tot -= g_slabs[k]->bytes;
      drop_slab(k);
    }
}

WsScope::WsScope(hipStream_t s) : st(s), mark(g_live.size()) { ++g_depth; }

WsScope::~WsScope() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t k = g_live.size(); k > mark; --k) {
    Slab* s = g_live[k - 1].slab;
    // every kernel of this call that touches the slab is queued on st by now
    if (hipEventRecord(s->done, g_live[k - 1].st) == hipSuccess) {
      s->recorded = true;
    } else {   // cannot order a later reuse behind this call: wait for the stream instead
      (void)hipStreamSynchronize(g_live[k - 1].st);
      s->recorded = false;
    }
    s->busy = false;
  }
  g_live.resize(mark);
  --g_depth;
}

int workspace(WsSlot slot, size_t bytes, void** ptr, hipStream_t st) {
  (void)slot;  // the slot names the buffer's role; every call gets its own slab
  if (g_depth <= 0) {
    set_error("internal: workspace() outside a WsScope");
    return QD_EINVAL;
  }
  int dev = 0;
  QD_HIP(hipGetDevice(&dev));
  const size_t want = slab_size(bytes ? bytes : 16);
  // A stream being captured into a HIP graph cannot wait on an event recorded outside the capture, and a slab handed
  // to a graph would be reused behind the graph's back at every replay: captured calls take a buffer the graph owns.
  if (stream_capturing(st)) return capture_alloc(want, ptr, st);
  free_dead_capture_buffers();
  (void)hipGetLastError();
  std::lock_guard<std::mutex> lk(g_mu);
  Slab* best = nullptr;
  for (Slab* s : g_slabs)
    if (!s->busy && s->dev == dev && s->bytes >= want && s->bytes / 4 <= want && (!best || s->bytes < best->bytes))
      best = s;
  if (best) {
    // device-side order behind the slab's previous user (no host wait)
    if (best->recorded) QD_HIP(hipStreamWaitEvent(st, best->done, 0));
  } else {
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      trim_idle(0);
      e = hipMalloc(&p, want);
    }
    if (e != hipSuccess) {
      set_error("workspace allocation of %zu bytes failed: %s", want, hipGetErrorString(e));
      return QD_ENOMEM;
    }
    hipEvent_t ev = nullptr;
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      (void)hipFree(p);
      set_error("workspace event creation failed: %s", hipGetErrorString(e));
      return QD_EHIP;
    }
    // the new slab is marked busy BEFORE the trim, which only releases idle slabs (a new slab pushed
    // idle was the first one trim_idle freed once the cache exceeded the cap)
    best = new Slab{p, want, dev, ev, true, false};
    g_slabs.push_back(best);
    trim_idle(idle_cap());
  }
  best->busy = true;
  g_live.push_back({best, st});
  *ptr = best->ptr;
  return QD_OK;
}

void free_workspaces() {
  free_dead_capture_buffers();
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t k = g_slabs.size(); k-- > 0;) {
    Slab* s = g_slabs[k];
    if (s->busy) continue;   // held by a call still running in another host thread
    if (s->recorded) (void)hipEventSynchronize(s->done);
    drop_slab(k);
  }
}

int pool_stats(size_t* reserved, size_t* used) {
  std::lock_guard<std::mutex> lk(g_mu);
  size_t r = 0, u = 0;
  for (const Slab* s : g_slabs) {
    r += s->bytes;
    if (!slab_idle_done(s)) u += s->bytes;
  }
  if (reserved) *reserved = r;
  if (used) *used = u;
  return QD_OK;
}

// ---------------------------------------------------------------- options and dispatch notes
static std::atomic<int> g_opt[QD_OPT_COUNT];
static const bool g_opt_init = [] {
  struct {
    int opt;
    const char* env;
    int dflt;
  } tab[] = {{QD_OPT_COOP_LAUNCH, "QD_COOP_LAUNCH", 1}, {QD_OPT_FAKE_TIMEOUT, "QD_TEST_FAKE_TIMEOUT", 0},
             {QD_OPT_GLF_PATH, "QD_GLF_PATH", QD_GLF_AUTO}, {QD_OPT_IDLE_CAP_MIB, nullptr, -1}};
  for (auto& t : tab) {
    const char* e = t.env ? std::getenv(t.env) : nullptr;
    g_opt[t.opt].store(e && *e ? std::atoi(e) : t.dflt);
  }
  return true;
}();

int option(int opt) { return (opt >= 0 && opt < QD_OPT_COUNT) ? g_opt[opt].load(std::memory_order_relaxed) : 0; }

bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cap) == hipSuccess && cap == hipStreamCaptureStatusActive;
}

// ---------------------------------------------------------------- fills, copies, uploads (qd_common.hpp)
__global__ void fill_bytes_kernel(unsigned char* __restrict__ d, unsigned char v, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t head = std::min<size_t>(n, (16 - ((uintptr_t)d & 15)) & 15);
  for (size_t i = i0; i < head; i += stride) d[i] = v;
  const unsigned w = 0x01010101u * v;
  uint4 q;
  q.x = q.y = q.z = q.w = w;
  uint4* d16 = (uint4*)(d + head);
  const size_t n16 = (n - head) / 16;
  for (size_t i = i0; i < n16; i += stride) d16[i] = q;
  for (size_t i = head + n16 * 16 + i0; i < n; i += stride) d[i] = v;
}

__global__ void copy_bytes_kernel(unsigned char* __restrict__ d, const unsigned char* __restrict__ s, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)d | (uintptr_t)s) & 15) == 0) {
    const size_t n16 = n / 16;
    for (size_t i = i0; i < n16; i += stride) ((uint4*)d)[i] = ((const uint4*)s)[i];
    for (size_t i = n16 * 16 + i0; i < n; i += stride) d[i] = s[i];
  } else {
    for (size_t i = i0; i < n; i += stride) d[i] = s[i];
  }
}

static int byte_grid(size_t n) { return (int)std::max<size_t>(1, std::min<size_t>((n / 16 + 255) / 256, 2048)); }

int fill_bytes(void* dst, unsigned char v, size_t n, hipStream_t st) {
  if (!n) return QD_OK;
  hipLaunchKernelGGL(fill_bytes_kernel, dim3(byte_grid(n)), dim3(256), 0, st, (unsigned char*)dst, v, n);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

int copy_device(void* dst, const void* src, size_t n, hipStream_t st) {
  if (!n) return QD_OK;
  hipLaunchKernelGGL(copy_bytes_kernel, dim3(byte_grid(n)), dim3(256), 0, st, (unsigned char*)dst,
                     (const unsigned char*)src, n);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

int upload(void* dst, const void* src, size_t n, hipStream_t st) {
  if (!n) return QD_OK;
  if (!stream_capturing(st)) {
    QD_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st));
    return QD_OK;
  }
  // dst is capture-owned scratch no kernel has touched yet: a blocking copy now, outside the capture
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  hipStream_t side = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, side);
  if (e == hipSuccess) e = hipStreamSynchronize(side);
  if (side) (void)hipStreamDestroy(side);
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  if (e != hipSuccess) {
    set_error("host upload of %zu bytes inside a graph capture failed: %s", n, hipGetErrorString(e));
    return QD_EHIP;
  }
  return QD_OK;
}

static thread_local std::string g_path;

void note_path(const char* name) {
  if (g_path.size() < 4096) {
    if (!g_path.empty()) g_path += ' ';
    g_path += name;
  }
}

}  // namespace qd

extern "C" {

int qd_set_option(int opt, int value) {
  QD_CHECK_ARG(opt >= 0 && opt < QD_OPT_COUNT, "qd_set_option: unknown option %d", opt);
  QD_CHECK_ARG(opt != QD_OPT_GLF_PATH || (value >= QD_GLF_AUTO && value <= QD_GLF_PERSISTENT),
               "qd_set_option: QD_OPT_GLF_PATH value %d", value);
  QD_CHECK_ARG(opt != QD_OPT_IDLE_CAP_MIB || value >= -1, "qd_set_option: QD_OPT_IDLE_CAP_MIB value %d", value);
  (void)qd::g_opt_init;
  qd::g_opt[opt].store(value);
  return QD_OK;
}

int qd_get_option(int opt, int* value) {
  QD_CHECK_ARG(opt >= 0 && opt < QD_OPT_COUNT && value, "qd_get_option: bad arguments");
  *value = qd::option(opt);
  return QD_OK;
}

int qd_take_path(char* buf, size_t len) {
  QD_CHECK_ARG(buf && len > 0, "qd_take_path: bad arguments");
  std::snprintf(buf, len, "%s", qd::g_path.c_str());
  qd::g_path.clear();
  return QD_OK;
}

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
