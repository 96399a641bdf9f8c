// handoff.hpp — in-launch hand-offs between workgroups of a persistent grid (MI355X_MICROARCH.md "Valid forms",
// table row 1): the producer stores every handed-off byte with 16-B write-through (sc1) buffer stores, every storing
// wave drains (s_waitcnt vmcnt(0)), a workgroup barrier, then one lane stores the epoch word (relaxed agent atomic);
// the consumer polls the epochs with relaxed agent loads from one wave, joins a workgroup barrier, and loads the
// handed-off bytes with 16-B sc1 buffer loads only (never a plain or flat load of them).  One workgroup per CU.
// Users: deom.hip (banded hierarchy; the pipelined stage kernel's plain buffer loads); glf_single.hip uses its
// loaders with the R2 form instead (the data is the flag, glf_single.hip header).
#pragma once
#include "qd_common.hpp"

namespace qd {

typedef unsigned int ho_u4 __attribute__((ext_vector_type(4)));

// 16-B sc1 buffer load of one complex element at byte offset `off`
__device__ __forceinline__ c128 ld16_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  const ho_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return cmk(__builtin_bit_cast(double, (unsigned long long)v.x | ((unsigned long long)v.y << 32)),
             __builtin_bit_cast(double, (unsigned long long)v.z | ((unsigned long long)v.w << 32)));
}
// 16-B write-through (sc1) buffer store of one complex element at byte offset `off`
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int off, c128 x) {
  const unsigned long long a = __builtin_bit_cast(unsigned long long, x.re);
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x.im);
  const ho_u4 v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// provably wave-uniform copy of a pointer (a buffer descriptor's base must be)
__device__ __forceinline__ void* wave_uniform_ptr(const void* q) {
  const unsigned long long v = (unsigned long long)q;
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)v), h = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (void*)(((unsigned long long)h << 32) | l);
}
// raw buffer descriptor over `bytes` bytes at `base` (the cache policy is the load / store's, not the descriptor's)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(wave_uniform_ptr(base), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sc1_rsrc(const void* base, int bytes) { return buf_rsrc(base, bytes); }

// plain (default cache policy) buffer loads with 32-bit byte offsets: an offset at or past the descriptor's size
// returns zeros (raw buffer range check), so a dead load needs no branch and no select
__device__ __forceinline__ c128 ld16_buf(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const ho_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return cmk(__builtin_bit_cast(double, (unsigned long long)v.x | ((unsigned long long)v.y << 32)),
             __builtin_bit_cast(double, (unsigned long long)v.z | ((unsigned long long)v.w << 32)));
}
__device__ __forceinline__ c128 ld16_buf_nt(__amdgpu_buffer_rsrc_t r, unsigned off) {   // non-temporal
  const ho_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2);
  return cmk(__builtin_bit_cast(double, (unsigned long long)v.x | ((unsigned long long)v.y << 32)),
             __builtin_bit_cast(double, (unsigned long long)v.z | ((unsigned long long)v.w << 32)));
}
// plain buffer store; an out-of-range offset drops it
__device__ __forceinline__ void st16_buf(__amdgpu_buffer_rsrc_t r, unsigned off, c128 x) {
  const unsigned long long a = __builtin_bit_cast(unsigned long long, x.re);
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x.im);
  const ho_u4 v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ int ld4_buf(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}
constexpr unsigned BUF_OOB = 0x7FFFFFF0u;   // an offset past every descriptor this library builds (sizes < 2^31 - 2^20)

}  // namespace qd
