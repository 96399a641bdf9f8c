// cgemm_block.hpp — workgroup-level complex-fp64 GEMM engine on
// v_mfma_f64_16x16x4_f64 (gfx950), used by the density-matrix kernels.
//
// One 512-thread workgroup (8 waves, 2 per SIMD) computes a BT x BT complex
// output block as a sum of "segments"  sum_s A_s[BT x K] * B_s[K x BT],
// with A_s, B_s row-major complex128 in global memory (L2/MALL resident).
//
// Data path per K-tile of 16 complex columns:
//   global --(16-B coalesced loads, register prefetch of tile t+1)--> LDS
//   (A tile row stride 18 complex: conflict-free ds_write_b128 staging and
//    ds_read_b128 fragment reads; B tile stride BT: natural and conflict-free)
//   LDS --(one complex = one ds_read_b128 per lane)--> MFMA fragments.
// A complex 16x16x4 MAC is 4 real f64 MFMAs:
//   Cr += Ar*Br ; Cr += (-Ai)*Bi ; Ci += Ar*Bi ; Ci += Ai*Br
// f64 MFMA operand / result maps (cdna_hip_programming.md §3):
//   A: lane l holds A[l&15][k=l>>4];  B: lane l holds B[k=l>>4][l&15]
//   D: 4 regs/lane, reg r = D[row=(l>>4)+4r][col=l&15]
#pragma once

#include "qd_common.hpp"

namespace qd {

constexpr int CG_WG = 512;       // threads per workgroup
constexpr int CG_KT = 16;        // complex K per LDS stage
constexpr int CG_SA = CG_KT + 2; // padded A-tile row stride (complex)

template <int BT> struct CgCfg;
// BT x BT block; wave grid WR x WC; each wave owns MW x NW MFMA tiles (16x16).
template <> struct CgCfg<128> { static constexpr int MW = 2, NW = 4, WR = 4, WC = 2; };
template <> struct CgCfg<64>  { static constexpr int MW = 1, NW = 2, WR = 4, WC = 2; };
template <> struct CgCfg<32>  { static constexpr int MW = 1, NW = 1, WR = 2, WC = 2; };

struct CgSeg {
  const c128* A;  // points at A[block_row0][0], leading dim lda
  const c128* B;  // points at B[0][block_col0], leading dim ldb
};

template <int BT>
struct CgLds {
  c128 a[2][BT * CG_SA];
  c128 b[2][CG_KT * BT];
};

template <int BT>
struct CgAcc {
  static constexpr int MW = CgCfg<BT>::MW, NW = CgCfg<BT>::NW;
  d4 re[MW][NW];
  d4 im[MW][NW];
};

// Number of complex elements per thread for one A (or B) tile.
template <int BT> constexpr int cg_nld() { return (BT * CG_KT) / CG_WG; }

// Staging registers are plain 16-B vectors and the loads go through an explicit
// global (address space 1) pointer: global_load_dwordx4 that stay in flight
// across the MFMA work of the current tile (no flat loads, no scratch round trip).
typedef double cg_v2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) cg_v2 cg_gv2;

__device__ __forceinline__ cg_v2 cg_ld(const c128* p) {
  return *(cg_gv2*)(p);  // generic -> global address-space cast (the pointer is a global buffer)
}
__device__ __forceinline__ void cg_st_lds(c128* p, cg_v2 v) { *reinterpret_cast<cg_v2*>(p) = v; }

#ifndef CG_STAGE_AT
#define CG_STAGE_AT 3  // k-step (of 4) before which the next tile's LDS stores are issued (4 = after compute)
#endif

#ifndef CG_SCHED_FENCE
#define CG_SCHED_FENCE 1
#endif
__device__ __forceinline__ void cg_sched_fence() {
#if CG_SCHED_FENCE
  __builtin_amdgcn_sched_barrier(0);
#endif
}

struct CgNoMid {
  __device__ __forceinline__ void operator()() const {}
};

// One K-tile of MFMA work from LDS buffer `buf`.  `mid()` runs before k-step CG_STAGE_AT: the caller puts
// the next tile's LDS stores there, so they issue while this tile's MFMAs are still in the pipe instead
// of between the last MFMA and the barrier (the double buffer keeps the two tiles apart).
// PIPE: the fragments of k-step q+1 are read from LDS into a second register set before the MFMAs
// of k-step q issue, so only the tile's first k-step waits on LDS latency (without it every k-step's
// first MFMA waits for its ds_read_b128s: the reads reuse the registers the previous MFMAs consume).
template <int BT, bool PIPE = false, typename Mid = CgNoMid>
__device__ __forceinline__ void cg_compute_tile(const CgLds<BT>& L, int buf, CgAcc<BT>& acc, int wr0, int wc0,
                                                Mid mid = Mid()) {
  constexpr int MW = CgCfg<BT>::MW, NW = CgCfg<BT>::NW;
  constexpr int NQ = CG_KT / 4;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = lane >> 4;
  constexpr int NS = PIPE ? 2 : 1;
  c128 a[NS][MW], b[NS][NW];
  auto frag = [&](int q, int slot) {
    const int kk = 4 * q;
#pragma unroll
    for (int mi = 0; mi < MW; ++mi) a[slot][mi] = L.a[buf][(wr0 + mi * 16 + lr) * CG_SA + kk + lk];
#pragma unroll
    for (int nj = 0; nj < NW; ++nj) b[slot][nj] = L.b[buf][(kk + lk) * BT + wc0 + nj * 16 + lr];
  };
  if (PIPE) frag(0, 0);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q == CG_STAGE_AT) {
      // keep the staging stores (and the vmcnt wait for their data) behind the MFMAs already issued:
      // without the fence the scheduler hoists them above the tile's MFMAs
      cg_sched_fence();
      mid();
      cg_sched_fence();
    }
    const int cs = PIPE ? (q & 1) : 0;
    if (PIPE) {
      if (q + 1 < NQ) frag(q + 1, (q + 1) & 1);
    } else {
      frag(q, 0);
    }
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        acc.re[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cs][mi].re, b[cs][nj].re, acc.re[mi][nj], 0, 0, 0);
        acc.im[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cs][mi].re, b[cs][nj].im, acc.im[mi][nj], 0, 0, 0);
      }
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        acc.re[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[cs][mi].im, b[cs][nj].im, acc.re[mi][nj], 0, 0, 0);
        acc.im[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cs][mi].im, b[cs][nj].re, acc.im[mi][nj], 0, 0, 0);
      }
  }
  if (CG_STAGE_AT >= NQ) {
    cg_sched_fence();
    mid();
  }
}

// Generic engine: T K-tiles; the operand tiles come from two policies with
//   Raw fetch(int t, int e, int q)           issued one tile ahead (global loads in flight during MFMA)
//   cg_v2 finish(const Raw&, int t, int e, int q)  run just before the LDS store (after the MFMA work)
// where e = tid + CG_WG*q is the element of the tile this thread stages (A: row e>>4, col e&15;
// B: row e/BT, col e%BT) and q < cg_nld<BT>() its compile-time slot.  A policy may fetch inputs and compute the operand in finish (generated operands).
// All threads of the workgroup must call it.  Ends with a workgroup barrier.
// zero = false accumulates onto acc (segment lists longer than an LDS table, run in chunks).
template <int BT, bool PIPE = false, typename APol, typename BPol>
__device__ __forceinline__ void cg_block_gemm_gen(int T, APol& pa, BPol& pb, CgLds<BT>& L, CgAcc<BT>& acc,
                                                  bool zero = true) {
  constexpr int MW = CgCfg<BT>::MW, NW = CgCfg<BT>::NW, WC = CgCfg<BT>::WC, WR = CgCfg<BT>::WR;
  const int wave = threadIdx.x >> 6;
  const bool active = wave < WR * WC;
  const int wr0 = (wave / WC) * (MW * 16);
  const int wc0 = (wave % WC) * (NW * 16);
  if (zero) {
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        acc.re[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
        acc.im[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
      }
  }
  constexpr int NLD = cg_nld<BT>();
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // staging address math stays per call (see cg_epilogue)
  typename APol::Raw ra[NLD];
  typename BPol::Raw rb[NLD];
  auto load = [&](int t) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = tid + CG_WG * q;
      ra[q] = pa.fetch(t, e, q);
      rb[q] = pb.fetch(t, e, q);
    }
  };
  auto store = [&](int t, int buf) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = tid + CG_WG * q;
      cg_st_lds(&L.a[buf][(e >> 4) * CG_SA + (e & 15)], pa.finish(ra[q], t, e, q));
      cg_st_lds(&L.b[buf][e], pb.finish(rb[q], t, e, q));
    }
  };
  load(0);
  store(0, 0);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const bool more = (t + 1) < T;
    if (more) load(t + 1);
    auto mid = [&]() {
      if (more) store(t + 1, (t + 1) & 1);
    };
    if (active) {
      cg_compute_tile<BT, PIPE>(L, t & 1, acc, wr0, wc0, mid);
    } else {
      mid();
    }
    __syncthreads();
  }
}

// The same engine with the global loads issued two K-tiles ahead (two register sets, loop unrolled by two so
// the set index is a compile-time constant): a tile's loads have two tiles of MFMA work to arrive instead of
// three k-steps, for blocks whose MFMA time per K-tile is short (BT = 64: 1.9 us per tile per SIMD) next to
// the fabric latency of operands served from the Infinity Cache.  Same results as cg_block_gemm_gen
// (identical MFMA order).
template <int BT, bool PIPE = false, typename APol, typename BPol>
__device__ __forceinline__ void cg_block_gemm_gen2(int T, APol& pa, BPol& pb, CgLds<BT>& L, CgAcc<BT>& acc) {
  constexpr int MW = CgCfg<BT>::MW, NW = CgCfg<BT>::NW, WC = CgCfg<BT>::WC, WR = CgCfg<BT>::WR;
  const int wave = threadIdx.x >> 6;
  const bool active = wave < WR * WC;
  const int wr0 = (wave / WC) * (MW * 16);
  const int wc0 = (wave % WC) * (NW * 16);
#pragma unroll
  for (int mi = 0; mi < MW; ++mi)
#pragma unroll
    for (int nj = 0; nj < NW; ++nj) {
      acc.re[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
      acc.im[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
    }
  constexpr int NLD = cg_nld<BT>();
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  typename APol::Raw ra[2][NLD];
  typename BPol::Raw rb[2][NLD];
  auto load = [&](int t, auto slot) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = tid + CG_WG * q;
      ra[slot()][q] = pa.fetch(t, e, q);
      rb[slot()][q] = pb.fetch(t, e, q);
    }
  };
  auto store = [&](int t, int buf, auto slot) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = tid + CG_WG * q;
      cg_st_lds(&L.a[buf][(e >> 4) * CG_SA + (e & 15)], pa.finish(ra[slot()][q], t, e, q));
      cg_st_lds(&L.b[buf][e], pb.finish(rb[slot()][q], t, e, q));
    }
  };
  struct S0 { constexpr int operator()() const { return 0; } };
  struct S1 { constexpr int operator()() const { return 1; } };
  load(0, S0{});
  if (T > 1) load(1, S1{});
  store(0, 0, S0{});
  __syncthreads();
  // iteration t: tile t+1 sits in register set (t+1)&1 and goes to LDS during tile t's MFMAs; tile t+2 is
  // loaded into set t&1 (tile t left it at iteration t-1)
  auto step = [&](int t, auto cur, auto nxt) {
    if (t + 2 < T) load(t + 2, cur);
    const bool more = (t + 1) < T;
    auto mid = [&]() {
      if (more) store(t + 1, (t + 1) & 1, nxt);
    };
    if (active) {
      cg_compute_tile<BT, PIPE>(L, t & 1, acc, wr0, wc0, mid);
    } else {
      mid();
    }
    __syncthreads();
  };
  int t = 0;
  for (; t + 1 < T; t += 2) {
    step(t, S0{}, S1{});
    step(t + 1, S1{}, S0{});
  }
  if (t < T) step(t, S0{}, S1{});
}

// Policies that read row-major complex tiles from memory through segment tables in LDS.
template <int BT>
struct CgSegA {
  using Raw = cg_v2;
  const CgSeg* segs;
  int tps, lda;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    const CgSeg sg = segs[t / tps];
    return cg_ld(sg.A + (size_t)(e >> 4) * lda + (t % tps) * CG_KT + (e & 15));
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int, int, int) const { return r; }
};
template <int BT>
struct CgSegB {
  using Raw = cg_v2;
  const CgSeg* segs;
  int tps, ldb;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    const CgSeg sg = segs[t / tps];
    return cg_ld(sg.B + (size_t)((t % tps) * CG_KT + e / BT) * ldb + (e % BT));
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int, int, int) const { return r; }
};

// Accumulate sum_s A_s * B_s over nseg segments of depth K (K % 16 == 0) into
// a zero-initialised accumulator.  All threads of the workgroup must call it.
// `segs` should live in LDS (or be uniform): it is indexed at run time, and a
// private array indexed at run time would be placed in scratch memory.
// Ends with a workgroup barrier, so LDS may be reused immediately after.
template <int BT, bool PIPE = false>
__device__ __forceinline__ void cg_block_gemm(const CgSeg* segs, int nseg, int K, int lda, int ldb, CgLds<BT>& L,
                                              CgAcc<BT>& acc, bool zero = true) {
  const int tps = K / CG_KT;
  CgSegA<BT> pa{segs, tps, lda};
  CgSegB<BT> pb{segs, tps, ldb};
  cg_block_gemm_gen<BT, PIPE>(nseg * tps, pa, pb, L, acc, zero);
}

// ---------------------------------------------------------------- Hermitian X GEMM (BT = 128)
// X = A r + B W over two K segments (A r: segment 0; B W: segment 1, W = C^+ / 2), for k = X + X^+ of a
// Hermitian right-hand side.  Only k on the upper triangle is used, and B W (= C r C^+ / 2) is itself Hermitian, so
// segment 1 need not reach the 16 x 16 tiles below the diagonal: there X = A r alone, and each tile above the diagonal
// takes the full C r C^+ instead of its half (A fragment doubled: 2 a x b / 2 is exact), so that
// k_ij = X_ij + conj(X_ji) = (A r)_ij + conj((A r)_ji) + (C r C^+)_ij for every i < j (diagonal tiles keep the half
// in both triangles).  Tile layout (16-tiles R, C in 0..7): wave w = 2 i + h owns row tiles {i, 7 - i} and the
// column tiles of kHermCols[w]; the two waves of a row pair split the 8 columns so that one holds 4 and the other 5
// of the pair's 9 tiles with R <= C, placed so that each SIMD's two waves (w, w + 4) hold 9: segment 1 is 36 tiles,
// 9 per SIMD, against 12 per SIMD when only the lower-left 64 x 64 block was skipped.
struct CgHermLayout {
  // column tiles of wave w, nibble nj (waves 0..3 in the low word, 4..7 in the high one)
  static __device__ __forceinline__ int ctile(int wave, int nj) {
    constexpr unsigned long long lo = 0x3210ULL | (0x7654ULL << 16) | (0x7610ULL << 32) | (0x5432ULL << 48);
    constexpr unsigned long long hi = 0x7432ULL | (0x6510ULL << 16) | (0x5410ULL << 32) | (0x7632ULL << 48);
    const unsigned long long t = wave < 4 ? lo : hi;
    return (int)((t >> ((wave & 3) * 16 + nj * 4)) & 15);
  }
  static __device__ __forceinline__ int rtile(int wave, int mi) { return mi == 0 ? (wave >> 1) : 7 - (wave >> 1); }
  static __device__ __forceinline__ int row0(int wave, int mi) { return rtile(wave, mi) * 16; }
  static __device__ __forceinline__ int col0(int wave, int nj) { return ctile(wave, nj) * 16; }
};

// Tile roles of wave w in the Hermitian segments, bit mi * 4 + nj: below the diagonal (skipped) / above it (A doubled).
constexpr int cg_herm_ctile(int w, int nj) {
  constexpr unsigned short cols[8] = {0x3210, 0x7654, 0x7610, 0x5432, 0x7432, 0x6510, 0x5410, 0x7632};
  return (cols[w] >> (nj * 4)) & 15;
}
constexpr unsigned cg_herm_mask(int w, bool below) {
  unsigned m = 0;
  for (int mi = 0; mi < 2; ++mi)
    for (int nj = 0; nj < 4; ++nj) {
      const int R = mi == 0 ? (w >> 1) : 7 - (w >> 1), C = cg_herm_ctile(w, nj);
      if (below ? R > C : R < C) m |= 1u << (mi * 4 + nj);
    }
  return m;
}

// k-steps [Q0, Q1) of one K-tile of the Hermitian X GEMM for a wave whose tile roles SK (skip) / DB (doubled A) are
// compile-time constants (segment 0 runs with SK = DB = 0): no per-tile selects or branches in the MFMA stream.
template <int W, unsigned SK, unsigned DB, int Q0, int Q1>
__device__ __forceinline__ void cg_herm_ksteps(const CgLds<128>& L, int buf, CgAcc<128>& acc, int wave) {
  constexpr int BT = 128, MW = 2, NW = 4;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = Q0; q < Q1; ++q) {
    const int kk = 4 * q;
    c128 a[MW], a2[MW], b[NW];
#pragma unroll
    for (int mi = 0; mi < MW; ++mi) {
      const int r0 = 16 * (mi == 0 ? (W >> 1) : 7 - (W >> 1));
      a[mi] = L.a[buf][(r0 + lr) * CG_SA + kk + lk];
      if ((DB >> (mi * 4)) & 15u) a2[mi] = cmk(a[mi].re + a[mi].re, a[mi].im + a[mi].im);   // doubled (exact)
    }
#pragma unroll
    for (int nj = 0; nj < NW; ++nj)
      b[nj] = L.b[buf][(kk + lk) * BT + 16 * cg_herm_ctile(W, nj) + lr];
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        if (SK & (1u << (mi * 4 + nj))) continue;   // below the diagonal: no Hermitian part
        const c128& av = (DB & (1u << (mi * 4 + nj))) ? a2[mi] : a[mi];
        acc.re[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.re, b[nj].re, acc.re[mi][nj], 0, 0, 0);
        acc.im[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.re, b[nj].im, acc.im[mi][nj], 0, 0, 0);
      }
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        if (SK & (1u << (mi * 4 + nj))) continue;
        const c128& av = (DB & (1u << (mi * 4 + nj))) ? a2[mi] : a[mi];
        acc.re[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.im, b[nj].im, acc.re[mi][nj], 0, 0, 0);
        acc.im[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.im, b[nj].re, acc.im[mi][nj], 0, 0, 0);
      }
  }
}

// K-tiles [t0, t1) of the X GEMM (of T in all) with the tile roles SK / DB fixed at compile time: tile t + 1's global
// loads are in flight during tile t's MFMAs and its LDS stores issue behind the first CG_STAGE_AT k-steps.
// The code path of wave W: its tile addresses are constants.
template <int W, unsigned SK, unsigned DB>
__device__ __forceinline__ void cg_herm_x_range(int t0, int t1, int T, const CgSegA<128>& pa, const CgSegB<128>& pb,
                                                CgLds<128>& L, CgAcc<128>& acc, int wave, int tid, cg_v2* ra,
                                                cg_v2* rb) {
  constexpr int NLD = cg_nld<128>(), NQ = CG_KT / 4, QS = CG_STAGE_AT < NQ ? CG_STAGE_AT : NQ;
  for (int t = t0; t < t1; ++t) {
    const bool more = (t + 1) < T;
    if (more) {
#pragma unroll
      for (int q = 0; q < NLD; ++q) {
        const int e = tid + CG_WG * q;
        ra[q] = pa.fetch(t + 1, e, q);
        rb[q] = pb.fetch(t + 1, e, q);
      }
    }
    cg_herm_ksteps<W, SK, DB, 0, QS>(L, t & 1, acc, wave);
    cg_sched_fence();
    if (more) {
#pragma unroll
      for (int q = 0; q < NLD; ++q) {
        const int e = tid + CG_WG * q;
        cg_st_lds(&L.a[(t + 1) & 1][(e >> 4) * CG_SA + (e & 15)], ra[q]);
        cg_st_lds(&L.b[(t + 1) & 1][e], rb[q]);
      }
    }
    cg_sched_fence();
    if constexpr (QS < NQ) cg_herm_ksteps<W, SK, DB, QS, NQ>(L, t & 1, acc, wave);
    __syncthreads();
  }
}

// segs[0] = (A, r), segs[1..nseg-1] = (B_c, W_c); K = the common depth (tps = K / 16 K-tiles per segment).
// sum_c B_c W_c must be Hermitian (segments >= 1 skip the tiles below the diagonal and double those above it,
// CgHermLayout; GLF operands without that property use cg_herm_x_gemm_q's plain X GEMM).  Each wave runs the
// Hermitian segments with its own compile-time tile roles (one code path per wave for the whole range, so the MFMA
// stream carries no selects or branches).  All threads call it; ends with a workgroup barrier.  Visit the result with
// cg_herm_epilogue.  Chunked segment lists (more Hermitian segments than an LDS table holds): the first chunk as
// above (nplain = 1, zero = true), every later one all Hermitian (nplain = 0) accumulated onto acc (zero = false).
__device__ __forceinline__ void cg_herm_x_gemm(const CgSeg* segs, int nseg, int K, int lda, int ldb, CgLds<128>& L,
                                               CgAcc<128>& acc, bool zero = true, int nplain = 1) {
  constexpr int BT = 128, MW = 2, NW = 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (zero) {
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        acc.re[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
        acc.im[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
      }
  }
  const int tps = K / CG_KT, T = nseg * tps;
  CgSegA<BT> pa{segs, tps, lda};
  CgSegB<BT> pb{segs, tps, ldb};
  constexpr int NLD = cg_nld<BT>();
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  cg_v2 ra[NLD], rb[NLD];
#pragma unroll
  for (int q = 0; q < NLD; ++q) {
    const int e = tid + CG_WG * q;
    cg_st_lds(&L.a[0][(e >> 4) * CG_SA + (e & 15)], pa.fetch(0, e, q));
    cg_st_lds(&L.b[0][e], pb.fetch(0, e, q));
  }
  __syncthreads();
  auto run = [&](auto wc) {
    constexpr int W = decltype(wc)::value;
    const int tp = nplain * tps;
    cg_herm_x_range<W, 0u, 0u>(0, tp, T, pa, pb, L, acc, wave, tid, ra, rb);
    cg_herm_x_range<W, cg_herm_mask(W, true), cg_herm_mask(W, false)>(tp, T, T, pa, pb, L, acc, wave, tid, ra, rb);
  };
#define QD_HT(w) \
  case w: run(std::integral_constant<int, w>{}); break;
  switch (wave) {
    QD_HT(0) QD_HT(1) QD_HT(2) QD_HT(3) QD_HT(4) QD_HT(5) QD_HT(6) default: QD_HT(7)
  }
#undef QD_HT
}

template <typename F>
__device__ __forceinline__ void cg_herm_epilogue(const CgAcc<128>& acc, F&& f) {
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) {
        const int row = CgHermLayout::row0(wave, mi) + (lane >> 4) + 4 * r;
        const int col = CgHermLayout::col0(wave, nj) + (lane & 15);
        f(row, col, cmk(acc.re[mi][nj][r], acc.im[mi][nj][r]));
      }
}

// Quadrant layout (the Redfield GLF operands, no Hermitian segment; and the round-2 first version of the Lindblad
// skip).  Hermitian right-hand side.  Only k on the upper blocks is used, and B W (= C r C^+ / 2) is itself Hermitian,
// so segment 1 need not reach the lower-left 64 x 64 block (1, 0): there X = A r alone, and the upper-right
// block (0, 1) takes the full C r C^+ instead of its half (A fragment doubled: 2 a x b / 2 is exact), so that
// k_ij = X_ij + conj(X_ji) = (A r)_ij + conj((A r)_ji) + (C r C^+)_ij on the off-diagonal blocks and as before on
// the diagonal ones.  The wave -> tile layout spreads block (1, 0) over every wave (each owns row tiles i and 4 + i
// and column tiles {2h, 2h+1, 4+2h, 5+2h}, i = wave / 2, h = wave % 2), so skipping its tiles in segment 1 takes
// 2 of 8 tiles from every wave alike: 1/4 of segment 1's MFMAs, 1/12 of a stage's.
struct CgHermLayoutQ {
  static __device__ __forceinline__ int row0(int wave, int mi) { return mi * 64 + (wave >> 1) * 16; }
  static __device__ __forceinline__ int col0(int wave, int nj) { return (nj >> 1) * 64 + (2 * (wave & 1) + (nj & 1)) * 16; }
};

template <typename Mid>
__device__ __forceinline__ void cg_herm_compute_tile_q(const CgLds<128>& L, int buf, CgAcc<128>& acc, int wave, bool seg1,
                                                     Mid mid) {
  constexpr int BT = 128, MW = 2, NW = 4, NQ = CG_KT / 4;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q == CG_STAGE_AT) {
      cg_sched_fence();
      mid();
      cg_sched_fence();
    }
    const int kk = 4 * q;
    c128 a[MW], b[NW];
#pragma unroll
    for (int mi = 0; mi < MW; ++mi) a[mi] = L.a[buf][(CgHermLayoutQ::row0(wave, mi) + lr) * CG_SA + kk + lk];
#pragma unroll
    for (int nj = 0; nj < NW; ++nj) b[nj] = L.b[buf][(kk + lk) * BT + CgHermLayoutQ::col0(wave, nj) + lr];
    // block (0, 1) in the Hermitian segments: the doubled fragment (exact); a[0] itself elsewhere
    const double s2 = seg1 ? 2.0 : 1.0;
    const c128 a2 = cmk(a[0].re * s2, a[0].im * s2);
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        if (mi == 1 && nj < 2 && seg1) continue;   // block (1, 0): no Hermitian part
        const c128& av = (mi == 0 && nj >= 2) ? a2 : a[mi];
        acc.re[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.re, b[nj].re, acc.re[mi][nj], 0, 0, 0);
        acc.im[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.re, b[nj].im, acc.im[mi][nj], 0, 0, 0);
      }
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        if (mi == 1 && nj < 2 && seg1) continue;
        const c128& av = (mi == 0 && nj >= 2) ? a2 : a[mi];
        acc.re[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.im, b[nj].im, acc.re[mi][nj], 0, 0, 0);
        acc.im[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.im, b[nj].re, acc.im[mi][nj], 0, 0, 0);
      }
  }
  if (CG_STAGE_AT >= NQ) {
    cg_sched_fence();
    mid();
  }
}

// segs[0] = (A, r), segs[1..nseg-1] = (B_c, W_c); K = the common depth (tps = K / 16 K-tiles per segment).
// hermitian_part: sum_c B_c W_c is Hermitian (segments >= 1 skip block (1, 0) and double block (0, 1)); otherwise
// every tile takes every segment (the plain X GEMM on this layout).  All threads call it; ends with a workgroup
// barrier.  Visit the result with cg_herm_epilogue_q.
__device__ __forceinline__ void cg_herm_x_gemm_q(const CgSeg* segs, int nseg, int K, int lda, int ldb, CgLds<128>& L,
                                               CgAcc<128>& acc, bool hermitian_part, bool zero = true, int nplain = 1) {
  constexpr int BT = 128, MW = 2, NW = 4;
  const int wave = threadIdx.x >> 6;
  if (zero) {
#pragma unroll
    for (int mi = 0; mi < MW; ++mi)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        acc.re[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
        acc.im[mi][nj] = d4{0.0, 0.0, 0.0, 0.0};
      }
  }
  const int tps = K / CG_KT, T = nseg * tps;
  CgSegA<BT> pa{segs, tps, lda};
  CgSegB<BT> pb{segs, tps, ldb};
  constexpr int NLD = cg_nld<BT>();
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  cg_v2 ra[NLD], rb[NLD];
  auto load = [&](int t) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = tid + CG_WG * q;
      ra[q] = pa.fetch(t, e, q);
      rb[q] = pb.fetch(t, e, q);
    }
  };
  auto store = [&](int t, int buf) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = tid + CG_WG * q;
      cg_st_lds(&L.a[buf][(e >> 4) * CG_SA + (e & 15)], ra[q]);
      cg_st_lds(&L.b[buf][e], rb[q]);
    }
  };
  load(0);
  store(0, 0);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const bool more = (t + 1) < T;
    if (more) load(t + 1);
    auto mid = [&]() {
      if (more) store(t + 1, (t + 1) & 1);
    };
    cg_herm_compute_tile_q(L, t & 1, acc, wave, hermitian_part && t >= nplain * tps, mid);
    __syncthreads();
  }
}

template <typename F>
__device__ __forceinline__ void cg_herm_epilogue_q(const CgAcc<128>& acc, F&& f) {
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) {
        const int row = CgHermLayoutQ::row0(wave, mi) + (lane >> 4) + 4 * r;
        const int col = CgHermLayoutQ::col0(wave, nj) + (lane & 15);
        f(row, col, cmk(acc.re[mi][nj][r], acc.im[mi][nj][r]));
      }
}

// Visit every accumulator element: f(row, col, value) with row/col inside the block.
template <int BT, typename F>
__device__ __forceinline__ void cg_epilogue(const CgAcc<BT>& acc, F&& f) {
  constexpr int MW = CgCfg<BT>::MW, NW = CgCfg<BT>::NW, WC = CgCfg<BT>::WC, WR = CgCfg<BT>::WR;
  // The thread index goes through an empty asm so the compiler cannot hoist the per-element
  // address math of an epilogue out of a persistent kernel's step loop (it would spill it).
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int wave = tid >> 6;
  if (wave >= WR * WC) return;
  const int lane = tid & 63;
  const int wr0 = (wave / WC) * (MW * 16);
  const int wc0 = (wave % WC) * (NW * 16);
#pragma unroll
  for (int mi = 0; mi < MW; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nj = 0; nj < NW; ++nj) {
        const int row = wr0 + mi * 16 + (lane >> 4) + 4 * r;
        const int col = wc0 + nj * 16 + (lane & 15);
        f(row, col, cmk(acc.re[mi][nj][r], acc.im[mi][nj][r]));
      }
}

}  // namespace qd
