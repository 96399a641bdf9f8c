// CPU emulation shim for debugging libqdyn kernels WRITTEN IN FLAT-LOOP FORM (every phase is a
// `for (f = threadIdx.x; f < n; f += blockDim.x)` loop followed by __syncthreads()): with one thread per
// block (blockDim.x = 1) a block runs its phases in order and the barriers are no-ops, so the kernel's
// arithmetic and indexing run unchanged on the host.  Debug tool only (tools/cpu_emu); not part of the
// product library.
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__
#define __restrict__

struct emu_dim3 {
  unsigned x = 0, y = 0, z = 0;
};
struct dim3 {
  unsigned x, y, z;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
extern thread_local emu_dim3 threadIdx, blockIdx, blockDim, gridDim;
inline void __syncthreads() {}
using std::min;
using std::max;
inline void sincospi(double x, double* s, double* c) {
  // exact at multiples of 1/2 like the device sincospi
  double r = std::fmod(x, 2.0);
  *s = std::sin(M_PI * r);
  *c = std::cos(M_PI * r);
  double h = r * 2.0;
  if (h == std::floor(h)) {
    long k = ((long)h % 4 + 4) % 4;
    *s = (k == 1) ? 1.0 : (k == 3 ? -1.0 : 0.0);
    *c = (k == 0) ? 1.0 : (k == 2 ? -1.0 : 0.0);
  }
}
inline double __longlong_as_double(long long v) { double d; memcpy(&d, &v, 8); return d; }
inline long long __double_as_longlong(double v) { long long d; memcpy(&d, &v, 8); return d; }

typedef int hipError_t;
typedef void* hipStream_t;
enum { hipSuccess = 0, hipMemcpyDeviceToDevice = 3, hipFuncAttributeMaxDynamicSharedMemorySize = 8 };
inline hipError_t hipGetLastError() { return hipSuccess; }
inline const char* hipGetErrorString(hipError_t) { return "emu"; }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, int, hipStream_t) { memmove(d, s, n); return 0; }
inline hipError_t hipFuncSetAttribute(const void*, int, int) { return 0; }

#define hipLaunchKernelGGL(K, G, B, SH, ST, ...)                                   \
  do {                                                                             \
    dim3 g_ = (G);                                                                 \
    gridDim.x = g_.x; gridDim.y = g_.y; gridDim.z = g_.z;                          \
    blockDim.x = 1; blockDim.y = 1; blockDim.z = 1;                                \
    threadIdx.x = threadIdx.y = threadIdx.z = 0;                                   \
    for (unsigned bz = 0; bz < g_.z; ++bz)                                         \
      for (unsigned by = 0; by < g_.y; ++by)                                       \
        for (unsigned bx = 0; bx < g_.x; ++bx) {                                   \
          blockIdx.x = bx; blockIdx.y = by; blockIdx.z = bz;                       \
          K(__VA_ARGS__);                                                          \
        }                                                                          \
  } while (0)
// DPP intrinsics: declared for the templates in qd_common.hpp; kernels that use them do not run here
inline int __builtin_amdgcn_mov_dpp(int v, int, int, int, bool) { abort(); return v; }
inline int __builtin_amdgcn_update_dpp(int, int v, int, int, int, bool) { abort(); return v; }
typedef double emu_d4 __attribute__((ext_vector_type(4)));
inline emu_d4 __builtin_amdgcn_mfma_f64_16x16x4f64(double, double, emu_d4 c, int, int, int) { abort(); return c; }
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
template <typename T> T __shfl(T v, int, int = 64) { abort(); return v; }
#define __HIP_MEMORY_SCOPE_AGENT 0
