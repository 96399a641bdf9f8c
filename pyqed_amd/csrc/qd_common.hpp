// qd_common.hpp — shared device/host helpers for libqdyn (gfx950 only).
//
// Complex numbers are interleaved fp64 pairs (re, im), byte-compatible with
// torch.complex128 / numpy.complex128.  Every entry point in include/qdyn.h
// returns 0 on success and a negative QD_E* code otherwise; the message is
// kept in a thread-local buffer readable through qd_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include <cstring>
#include <algorithm>

#include "../../include/qdyn.h"

namespace qd {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);

#define QD_CHECK_ARG(cond, ...)                         \
  do {                                                  \
    if (!(cond)) {                                      \
      ::qd::set_error(__VA_ARGS__);                     \
      return QD_EINVAL;                                 \
    }                                                   \
  } while (0)

#define QD_TRY(call)        \
  do {                      \
    const int rc_ = (call); \
    if (rc_) return rc_;    \
  } while (0)
#define QD_HIP(call)                                                        \
  do {                                                                      \
    hipError_t _e = (call);                                                 \
    if (_e != hipSuccess) {                                                 \
      ::qd::set_error("HIP error %s at %s:%d (%s)", hipGetErrorString(_e),  \
                      __FILE__, __LINE__, #call);                           \
      return QD_EHIP;                                                       \
    }                                                                       \
  } while (0)

// Library-owned scratch, never handed to the caller (qd_runtime.hip).  Every entry point that needs
// scratch opens a WsScope on its stream; workspace() returns a slab of the library's arena that no other
// live call holds, ordered on the device behind the slab's previous user (hipStreamWaitEvent), and the
// scope's end records the slab's event on the stream -- no host wait anywhere.  Distinct streams / host
// threads never share live scratch (SURVEY.md §8(b) threading contract); the arena is bounded by the peak
// concurrent use plus a capped idle cache, not by the number of streams seen (qd_workspace_stats).
enum WsSlot { WS_LINDBLAD = 0, WS_LINDBLAD_OPS = 1, WS_SPO = 2, WS_DEOM = 3,
              WS_SUPEROP = 4, WS_2DES = 5, WS_MISC = 6, WS_2DES_OPS = 7, WS_TDSE_H = 8,
              WS_TDSE_GEMM = 9, WS_SUPEROP_OPS = 10, WS_NSLOTS = 11 };
struct WsScope {
  hipStream_t st;
  size_t mark;
  explicit WsScope(hipStream_t s);
  ~WsScope();
  WsScope(const WsScope&) = delete;
  WsScope& operator=(const WsScope&) = delete;
};
int workspace(WsSlot slot, size_t bytes, void** ptr, hipStream_t st);
int pool_stats(size_t* reserved, size_t* used);
void free_workspaces();

// Process options (qd_runtime.hip): the library's only run-time switches, read once from the environment when the
// library loads and changeable with qd_set_option (include/qdyn.h QD_OPT_*).  Dispatch is otherwise a function of
// the problem's shape alone.
int option(int opt);
// Records a dispatch decision of the current call for qd_take_path (tests assert which kernel a shape reaches).
void note_path(const char* name);
// true while `st` is being captured into a HIP graph
bool stream_capturing(hipStream_t st);
// Stream-ordered fills and copies of device memory done by kernels, not by hipMemsetAsync / hipMemcpyAsync: inside a
// graph capture those become memset / memcpy nodes, whose replays did not order reliably against the kernels around
// them on this ROCm (profiles/r06/graph/replay_diag.txt).  fill_bytes sets n bytes to `v`.
int fill_bytes(void* dst, unsigned char v, size_t n, hipStream_t st);
int copy_device(void* dst, const void* src, size_t n, hipStream_t st);
// Host array -> device scratch, stream-ordered.  Outside a capture a hipMemcpyAsync; inside one the bytes are copied
// at capture time (the replays reuse the values the host array held then, and never read the host pointer again).
int upload(void* dst, const void* src, size_t n, hipStream_t st);

// ---------------------------------------------------------------- complex
struct alignas(16) c128 {
  double re, im;
};

__host__ __device__ inline c128 cmk(double r, double i) { c128 z; z.re = r; z.im = i; return z; }
__host__ __device__ inline c128 cadd(c128 a, c128 b) { return cmk(a.re + b.re, a.im + b.im); }
__host__ __device__ inline c128 csub(c128 a, c128 b) { return cmk(a.re - b.re, a.im - b.im); }
__host__ __device__ inline c128 cmul(c128 a, c128 b) {
  return cmk(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
__host__ __device__ inline c128 cscale(c128 a, double s) { return cmk(a.re * s, a.im * s); }
__host__ __device__ inline c128 cconj(c128 a) { return cmk(a.re, -a.im); }
__host__ __device__ inline c128 cmuli(c128 a) { return cmk(-a.im, a.re); }     // i*a
__host__ __device__ inline c128 cmulmi(c128 a) { return cmk(a.im, -a.re); }    // -i*a

typedef double d4 __attribute__((ext_vector_type(4)));

// Quad-permute DPP move of a double / complex (gfx9 quad_perm: lane q of each group of 4 lanes reads
// lane (CTRL >> 2q) & 3 of its group); one VALU op per dword, no LDS traffic.
template <int CTRL>
__device__ __forceinline__ double dpp_qd(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ c128 dpp_qc(c128 v) { return cmk(dpp_qd<CTRL>(v.re), dpp_qd<CTRL>(v.im)); }
template <int CTRL>
__device__ __forceinline__ int dpp_qi(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }

// v + slab(s0) + ... + slab(S - 1) in that fixed order (deterministic split-K sums), with the loads of 16 slabs issued
// before their adds: a rolled load-add loop waits one memory round trip per slab (the 16 slabs of a 256 x 256 2DES
// grid took 14.3 us that way, 11.3 in batches of 8).
template <typename F>
__device__ __forceinline__ c128 slab_sum(c128 v, int s0, int S, F&& at) {
  constexpr int CH = 16;
  for (; s0 < S; s0 += CH) {
    c128 b[CH];
#pragma unroll
    for (int t = 0; t < CH; ++t) b[t] = s0 + t < S ? at(s0 + t) : cmk(0, 0);
#pragma unroll
    for (int t = 0; t < CH; ++t)
      if (s0 + t < S) v = cadd(v, b[t]);
  }
  return v;
}

// RK4 in Horner form for a linear generator L that is constant over the step (every propagator here except the
// driven DEOM stages): classical RK4 is then exactly the degree-4 Taylor polynomial
//   rho' = rho + dt L(rho + dt/2 L(rho + dt/3 L(rho + dt/4 L rho))),
// so stage m (0..3) reads s_m (s_0 = rho) and writes s_{m+1} = rho + c_m L s_m with c_m = dt / (4 - m), s_4 = rho'.
// No accumulator is read or written (phys.rk4, phys.py:1051-1064, up to rounding).
__device__ __forceinline__ double rk4_horner_coef(double dt, int stage) {
  return stage == 0 ? dt * 0.25 : stage == 1 ? dt / 3.0 : stage == 2 ? dt * 0.5 : dt;
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Split-K complex fp64 MFMA GEMM (response.hip): slabs[s] = A [Mp][Kp] x B [Kp][Np] over K slice s, S <= max_S
// slices (returned); Mp a multiple of 128, Np of 64 (64-wide column blocks) or 128, Kp of 16.
int cgemm_splitk_slabs(const c128* A, const c128* B, int Mp, int Kp, int Np, c128* slabs, int max_S, int* S_out,
                       hipStream_t st);

// Unnormalised DFT along the middle axis of the [O][L][I] grid x, in place, any L (spo_gen.hip).  *l2 != 0: four-step
// order, X[k1 + (L / *l2) k2] at slot *l2 k1 + k2; else natural order.  O L I < 2^31.
int fft_lines(c128* x, long O, int L, long I, bool inv, hipStream_t st, int* l2);

}  // namespace qd
