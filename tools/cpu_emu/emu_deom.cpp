// Host build of deom.hip through the flat-loop emulation shim: only the flat-loop kernels (deom_stage_tile_kernel,
// heom_chain_sweep_kernel, deom_trace_kernel, ...) can run here; the register / MFMA kernels are compiled, not run.
#include <vector>
#include <cstdarg>
#include "hip/hip_runtime.h"
thread_local emu_dim3 threadIdx, blockIdx, blockDim, gridDim;
#include "../../pyqed_amd/csrc/deom.hip"
namespace qd { namespace { c128 deom_lds[163840 / 16]; } }
namespace qd {
static thread_local std::vector<void*> g_bufs;
void set_error(const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap); fprintf(stderr, "\n");
}
WsScope::WsScope(hipStream_t s) : st(s), mark(g_bufs.size()) {}
WsScope::~WsScope() { while (g_bufs.size() > mark) { free(g_bufs.back()); g_bufs.pop_back(); } }
int workspace(WsSlot, size_t bytes, void** ptr, hipStream_t) { *ptr = calloc(1, bytes + 16); g_bufs.push_back(*ptr); return 0; }
}
