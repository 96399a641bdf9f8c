// Host build of spo_gen.hip through the flat-loop emulation shim (tools/cpu_emu/hip/hip_runtime.h).
#include <vector>
#include <cstdarg>
#include "hip/hip_runtime.h"
thread_local emu_dim3 threadIdx, blockIdx, blockDim, gridDim;
#include "../../pyqed_amd/csrc/spo_gen.hip"

namespace qd {
static thread_local std::vector<void*> g_bufs;
void set_error(const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap); fprintf(stderr, "\n");
}
WsScope::WsScope(hipStream_t s) : st(s), mark(g_bufs.size()) {}
WsScope::~WsScope() { while (g_bufs.size() > mark) { free(g_bufs.back()); g_bufs.pop_back(); } }
int workspace(WsSlot, size_t bytes, void** ptr, hipStream_t) { *ptr = calloc(1, bytes + 16); g_bufs.push_back(*ptr); return 0; }
}
namespace qd { namespace spog { c128 sm[163840 / 16]; } }
extern "C" {
int emu_spo_nd(void* psi, const void* Uh, const void* Uf, const void* K, const void* Ky, const int* dims, int D, int ns,
               int nsteps, int nout, void* snap) {
  return qd::spo_generic_run((qd::c128*)psi, (const qd::c128*)Uh, (const qd::c128*)Uf, (const qd::c128*)K,
                             (const qd::c128*)Ky, dims, D, ns, nsteps, nout, (qd::c128*)snap, nullptr);
}
int emu_spo1d(void* psi, const void* eV, const void* eVh, const void* eK, int nx, int B, int nt, int nout, void* snap) {
  return qd::spo1d_generic_run((qd::c128*)psi, (const qd::c128*)eV, (const qd::c128*)eVh, (const qd::c128*)eK, nx, B,
                               nt, nout, (qd::c128*)snap, nullptr);
}
}
