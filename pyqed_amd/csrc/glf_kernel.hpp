// glf_kernel.hpp — the persistent GLF / Lindblad RK4 kernel (lindblad_rk4_kernel) and its parameter block,
// shared by glf.hip (every nc <= MAX_NC instantiation) and glf_chunk.hip (the CHUNK instantiations for longer
// collapse-operator lists).  The CHUNK kernels live in their own translation unit: instantiated next to the
// headline kernel they changed its register allocation (12 B per lane of scratch instead of 0).
// See glf.hip for the algorithm.
#pragma once
#include "cgemm_block.hpp"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace qd {

struct LindbladParams {
  const c128* Cop;  // [nc][Np][Np]  L_c   (Lindblad: C_c)
  const c128* mK;   // [Np][Np]      P     (Lindblad: -iK)
  const c128* iKd;  // [Np][Np]      Q     (Lindblad: iH - S/2)
  const c128* Cd;   // [nc][Np][Np]  R_c   (Lindblad: C_c^+)
  const c128* eT;   // [ne][Np][Np]  E_m^T
  c128* rho;        // [B][Np][Np]   state (in/out)
  c128* ws;         // [B][3+nc][Np][Np] scratch
  c128* obs;        // [B][nsteps+1][ne]
  c128* snap;       // [B][nsave][N][N]
  int N, Np, nc, ne, nsteps, save_every, nsave;
  int step0, total_steps;  // this launch runs global steps step0 .. step0+nsteps-1 of total_steps
  int herm;                // Hermitian fast path (Lindblad, rho exactly Hermitian, single block)
  int hseg;                // Hermitian path: sum_c L_c r W_c is itself Hermitian (Lindblad C r C^+ / 2; not Redfield's
                           // sum A r Lam^+), so its redundant tiles below the diagonal may be skipped (cg_herm_x_gemm)
  double dt;
  unsigned long long* tbuf;  // [B][8] per-phase wall-clock ticks (QD_PHASE_TIMING diagnostics) or null
  int stage, rin, rout;        // split path: RK4 stage; stage input / output buffer (0 = rho, 1/2 = scratch 0/1)
  int ks, ys;                  // split path: K-splits of the k / Y phases (1 = none)
  c128* kslab;                 // [B][nb^2][ks][BT^2] partial k blocks
  c128* yslab;                 // [B][nc][nb^2][ys][BT^2] partial Y blocks
  unsigned* ticket;            // [B][1 + nc][nb^2] arrival counters (zero between launches)
  const int* guard;            // persistent kernel: run only if *guard != 0 (the single launch's fallback), or null
};

namespace {

constexpr int MAX_NC = 256;  // collapse-operator / GLF pair segments held in the kernels' LDS segment tables (4 KB);
                             // longer lists run the persistent kernels' CHUNK instantiations (chunks of MAX_NC)


// Per-matrix scratch slots of Np x Np: stage buffer(s), Y_c.
__host__ __device__ inline int glf_slots(int Np, int nc, int herm) {
  (void)herm;
  return (Np <= 128 ? 1 : 2) + nc;
}

// Horner coefficient of RK4 stage m (0..3): s_{m+1} = rho + dt / (4 - m) L s_m  (see the file header)
__device__ __forceinline__ double glf_horner_coef(double dt, int stage) { return rk4_horner_coef(dt, stage); }

#ifdef QD_PHASE_TIMING
// Diagnostics only (p.tbuf != null): barrier, then thread 0 charges the ticks since the last mark to `slot`.
#define QD_TMARK(slot)                                   \
  if (p.tbuf) {                                          \
    __syncthreads();                                     \
    if (threadIdx.x == 0) {                              \
      const unsigned long long now_ = wall_clock64();    \
      tacc[slot] += now_ - tlast;                        \
      tlast = now_;                                      \
    }                                                    \
  }
#define QD_TIMING_DECL                                                                \
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tlast = p.tbuf ? wall_clock64() : 0; \
  const unsigned long long t0w_ = tlast, t0c_ = clock64();
#define QD_TIMING_FLUSH                                                     \
  if (p.tbuf && threadIdx.x == 0) {                                         \
    for (int q = 0; q < 6; ++q) p.tbuf[(size_t)b * 8 + q] += tacc[q];      \
    p.tbuf[(size_t)b * 8 + 6] += clock64() - t0c_;                          \
    p.tbuf[(size_t)b * 8 + 7] += wall_clock64() - t0w_;                     \
  }
#else
#define QD_TMARK(slot)
#define QD_TIMING_DECL
#define QD_TIMING_FLUSH
#endif

// Tr(E_m rho) = sum_ij rho_ij E_m[j][i] = sum_ij rho_ij eT_m[i][j]; fixed
// reduction order (per-thread strided partials, wave butterfly, 8-wave sum).
__device__ void wg_observables(const c128* rho, const c128* eT, int ne, size_t NN, c128* out, c128* sred) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int m = 0; m < ne; ++m) {
    const c128* e = eT + (size_t)m * NN;
    double sr = 0.0, si = 0.0;
    for (size_t i = tid; i < NN; i += CG_WG) {
      c128 r = rho[i], x = e[i];
      sr += r.re * x.re - r.im * x.im;
      si += r.re * x.im + r.im * x.re;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      sr += __shfl_xor(sr, off, 64);
      si += __shfl_xor(si, off, 64);
    }
    if (lane == 0) sred[wave] = cmk(sr, si);
    __syncthreads();
    if (tid == 0) {
      c128 s = sred[0];
      for (int w = 1; w < CG_WG / 64; ++w) s = cadd(s, sred[w]);
      out[m] = s;
    }
    __syncthreads();
  }
}

#ifndef GLF_HERM_X
#define GLF_HERM_X 1   // Hermitian kernel at BT = 128: X GEMM on the CgHermLayout tiles (Lindblad: no Hermitian part below the diagonal; A/B: 0)
#endif
#ifndef GLF_EPI_PRE
#define GLF_EPI_PRE 4   // Hermitian epilogue: this many rho loads of round 0's first chunk issued before the LDS passes
#endif
#ifndef GLF_SPLIT_DEPTH
#define GLF_SPLIT_DEPTH 2   // split-path GEMMs: K-tiles of global loads in flight ahead of the MFMAs (1 or 2)
#endif
// the split-path GEMM engine: tile loads one (cg_block_gemm_gen) or two (cg_block_gemm_gen2) K-tiles ahead; same
// MFMA order, bit-identical results
// (measured and rejected: 32-blocks with the even / odd K-tiles on the two wave halves of a single-buffered K-tile
// pair, all eight waves issuing MFMAs: 64 matrices 204k vs 218-223k DM-steps/s, profiles/r03/lindblad/split_halves_ab.txt)
template <int BT, typename APol, typename BPol>
__device__ __forceinline__ void split_gemm(int T, APol& pa, BPol& pb, CgLds<BT>& L, CgAcc<BT>& acc) {
  if constexpr (GLF_SPLIT_DEPTH >= 2) cg_block_gemm_gen2<BT>(T, pa, pb, L, acc);
  else cg_block_gemm_gen<BT>(T, pa, pb, L, acc);
}
template <int BT>
__device__ __forceinline__ void split_block_gemm(const CgSeg* segs, int nseg, int K, int lda, int ldb, CgLds<BT>& L,
                                                 CgAcc<BT>& acc) {
  const int tps = K / CG_KT;
  CgSegA<BT> pa{segs, tps, lda};
  CgSegB<BT> pb{segs, tps, ldb};
  split_gemm<BT>(nseg * tps, pa, pb, L, acc);
}
#ifndef GLF_HERM_PIPE
#define GLF_HERM_PIPE false   // fragment double-buffering in the Hermitian kernel's GEMMs (A/B builds)
#endif

#ifndef GLF_KW
#define GLF_KW 1   // Hermitian kernel (HSEG): k = X + X^+ passes with the wave's tile roles as compile-time constants
#endif

// Pass A (PB = false) / pass B (PB = true) of k = X + X^+ into the LDS k buffers (see the kernel) for wave W of the
// CgHermLayout tiles.  Tile (R, C) of 16 x 16 lies in 64 x 64 quadrant (R / 4, C / 4); only the diagonal 16 x 16 tiles
// need per-element tests, every other tile is wholly upper (pass A stores), wholly lower (pass B adds the conjugate
// at the mirror slot) or in the lower-left quadrant (pass B into T01 transposed).  Same stores / adds as the generic
// visitor, without its per-element index arithmetic and branches.
template <int W, bool PB, typename Slot>
__device__ __forceinline__ void herm_k_pass(const CgAcc<128>& A, c128* T01, c128* Tt, int lane, Slot&& slot) {
  constexpr int TS = 64, LD = TS + 1, TRI = TS * (TS + 1) / 2;
  const int lr = lane >> 4, lc = lane & 15;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      const int R = mi == 0 ? (W >> 1) : 7 - (W >> 1), C = cg_herm_ctile(W, nj);   // constants after unrolling
      const int QR = R >> 2, QC = C >> 2, rr = (R & 3) * 16, c0 = (C & 3) * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const c128 v = cmk(A.re[mi][nj][r], A.im[mi][nj][r]);
        const int ra = rr + lr + 4 * r, cc = c0 + lc;
        if (QR < QC) {
          if (!PB) T01[ra * LD + cc] = v;
        } else if (QR > QC) {
          if (PB) {
            c128* t = &T01[cc * LD + ra];
            *t = cadd(*t, cconj(v));
          }
        } else if ((R & 3) < (C & 3)) {
          if (!PB) Tt[QR * TRI + slot(ra, cc)] = v;
        } else if ((R & 3) > (C & 3)) {
          if (PB) {
            c128* t = &Tt[QR * TRI + slot(cc, ra)];
            *t = cadd(*t, cconj(v));
          }
        } else if (!PB) {
          if (ra < cc) Tt[QR * TRI + slot(ra, cc)] = v;
          else if (ra == cc) Tt[QR * TRI + slot(ra, cc)] = cadd(v, cconj(v));
        } else if (ra > cc) {
          c128* t = &Tt[QR * TRI + slot(cc, ra)];
          *t = cadd(*t, cconj(v));
        }
      }
    }
}

// HSEG (Hermitian kernel only): sum_c L_c r W_c is itself Hermitian (Lindblad C r C^+ / 2), so the X GEMM skips its
// tiles below the diagonal (cg_herm_x_gemm); without it (Redfield's GLF operands) the plain X GEMM (cg_herm_x_gemm_q).
// CHUNK (nc > MAX_NC only; the nc <= MAX_NC instantiations are compiled without it): the segment lists of the X / k
// GEMMs run in chunks of MAX_NC collapse-operator segments through the LDS table, accumulating in registers.
template <int BT, bool HERM, bool HSEG = false, bool CHUNK = false>
__global__ __launch_bounds__(CG_WG) void lindblad_rk4_kernel(LindbladParams p) {
  if (p.guard && __hip_atomic_load(p.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  __shared__ CgLds<BT> L;
  __shared__ c128 sred[CG_WG / 64];
  __shared__ CgSeg segs[2 + MAX_NC];   // segment table in LDS (no scratch)

  const int b = blockIdx.x;
  const int Np = p.Np, nc = p.nc;
  const size_t NN = (size_t)Np * Np;
  c128* rho = p.rho + (size_t)b * NN;
  // single block (Np <= 128): every stage input is fully consumed by the GEMMs before the epilogue
  // overwrites it, so one stage buffer is updated in place; else two alternate.
  const bool single = (Np / BT) == 1;
  c128* ws = p.ws + (size_t)b * glf_slots(Np, nc, HERM) * NN;
  c128* rbuf1 = single ? ws : ws + NN;
  c128* Y = single ? ws + NN : ws + 2 * NN;
  c128* obs = p.obs ? p.obs + (size_t)b * (p.total_steps + 1) * p.ne : nullptr;

  if (p.ne > 0 && p.step0 == 0) wg_observables(rho, p.eT, p.ne, NN, obs, sred);
  __syncthreads();

  const int nb = Np / BT;
  const double dt = p.dt;
  CgAcc<BT> A;
  QD_TIMING_DECL

  for (int step = 0; step < p.nsteps; ++step) {
    for (int stage = 0; stage < 4; ++stage) {
      // Horner stages (glf_horner_coef): rho -> s1 -> s2 -> s3 -> rho; single block: s_m in place in ws
      const c128* r = stage == 0 ? rho : ((stage - 1) & 1) ? rbuf1 : ws;
      c128* rn = stage == 3 ? rho : (stage & 1) ? rbuf1 : ws;
      const double hc = glf_horner_coef(dt, stage);
      auto rk4_update = [&](size_t idx, c128 k) { rn[idx] = cadd(rho[idx], cscale(k, hc)); };
      if constexpr (HERM) {
        // Hermitian rho: L[rho] = X + X^+ with X = (-iK) r + sum_c (C_c r)(C_c^+ / 2)   (single block, nb == 1;
        // p.Cd holds C_c^+ / 2 on this path).  phase 1: Y_c = C_c r
        for (int c = 0; c < nc; ++c) {
          if (threadIdx.x == 0) {
            segs[0].A = p.Cop + (size_t)c * NN;
            segs[0].B = r;
          }
          __syncthreads();
          cg_block_gemm<BT, GLF_HERM_PIPE>(segs, 1, Np, Np, Np, L, A);
          QD_TMARK(0);
          c128* Yc = Y + (size_t)c * NN;
          cg_epilogue<BT>(A, [&](int row, int col, c128 v) { Yc[(size_t)row * Np + col] = v; });
          QD_TMARK(1);
        }
        __syncthreads();
        // phase 2: X in registers (one accumulator over 1 + nc segments); k_ij = X_ij + conj(X_ji) is
        // formed from the accumulator and an LDS transpose: exactly Hermitian, fused RK4 epilogue
        constexpr bool HX = BT == 128 && GLF_HERM_X;   // tiles without the Hermitian part (cgemm_block.hpp)
        if constexpr (!CHUNK) {
          if (threadIdx.x == 0) {
            segs[0].A = p.mK;
            segs[0].B = r;
            for (int c = 0; c < nc; ++c) {
              segs[1 + c].A = Y + (size_t)c * NN;
              segs[1 + c].B = p.Cd + (size_t)c * NN;
            }
          }
          __syncthreads();
          if constexpr (HX && HSEG) cg_herm_x_gemm(segs, 1 + nc, Np, Np, Np, L, A);
          else if constexpr (HX) cg_herm_x_gemm_q(segs, 1 + nc, Np, Np, Np, L, A, false);
          else cg_block_gemm<BT, GLF_HERM_PIPE>(segs, 1 + nc, Np, Np, Np, L, A);
        } else {
          for (int c0 = 0; c0 < nc; c0 += MAX_NC) {   // (P r) + the first MAX_NC segments, then MAX_NC at a time
            const int first = c0 == 0 ? 1 : 0, cn = min(MAX_NC, nc - c0);
            if (threadIdx.x == 0) {
              segs[0].A = p.mK;
              segs[0].B = r;
              for (int c = 0; c < cn; ++c) {
                segs[first + c].A = Y + (size_t)(c0 + c) * NN;
                segs[first + c].B = p.Cd + (size_t)(c0 + c) * NN;
              }
            }
            __syncthreads();
            if constexpr (HX && HSEG) cg_herm_x_gemm(segs, first + cn, Np, Np, Np, L, A, first, first);
            else if constexpr (HX) cg_herm_x_gemm_q(segs, first + cn, Np, Np, Np, L, A, false, first, first);
            else cg_block_gemm<BT, GLF_HERM_PIPE>(segs, first + cn, Np, Np, Np, L, A, first);
          }
        }
        auto visit = [&](auto&& f) {
          if constexpr (HX && HSEG) cg_herm_epilogue(A, f);
          else if constexpr (HX) cg_herm_epilogue_q(A, f);
          else cg_epilogue<BT>(A, f);
        };
        QD_TMARK(2);
        // k = X + X^+ formed in LDS on the upper triangle only (TS = BT/2; the GEMM staging buffers are free).
        // Every stage quantity is exactly Hermitian (k_ji = conj(k_ij) bit for bit, and the RK4 updates are
        // elementwise with real coefficients), so each (i, j), i <= j, is computed once and its mirror written as
        // the conjugate.  Pass A stores the accumulator's upper elements: tile (0, 1) into T01 [TS][TS + 1] and the
        // diagonal tiles' upper triangles into Tt (packed, folded: rows u and TS - 1 - u of a tile share one run of
        // TS + 1 slots); pass B adds the conjugate of every lower element at its mirror slot.  The accumulator
        // stays in registers through both passes (no global round trip of the diagonal tiles).  The Horner update then
        // reads rho on the upper triangle only and writes the next stage input (rho at stage 3) in full (the GEMMs,
        // observables and the caller read it).
        {
          constexpr int TS = BT / 2, LD = TS + 1, TRI = TS * (TS + 1) / 2;
          static_assert((TS * LD + 2 * TRI) * sizeof(c128) <= sizeof(CgLds<BT>), "LDS k buffers");
#ifndef QD_EPI_CH
#define QD_EPI_CH 8   // rho loads per thread in flight per chunk of the Horner update
#endif
          c128* T01 = reinterpret_cast<c128*>(&L);
          c128* Tt = T01 + TS * LD;
          int tid = threadIdx.x;
          asm volatile("" : "+v"(tid));  // keep the per-element index math inside the stage loop (no LICM + spill)
          // folded packed slot of (ra, cc), ra <= cc, within a diagonal tile
          auto slot = [&](int ra, int cc) {
            const bool top = ra < TS / 2;
            const int u = top ? ra : TS - 1 - ra;
            return u * (TS + 1) + (top ? 0 : TS - u) + (cc - ra);
          };
          constexpr int NPER0 = (TS * TS + CG_WG - 1) / CG_WG;
          constexpr int CH0 = NPER0 < QD_EPI_CH ? NPER0 : QD_EPI_CH;
          constexpr int NPRE = GLF_EPI_PRE < CH0 ? GLF_EPI_PRE : CH0;   // prefetched elements per thread
          c128 pre[NPRE ? NPRE : 1];
          if constexpr (GLF_EPI_PRE) {   // round 0's first chunk (tile (0, 1): e -> (e / TS, TS + e % TS))
#pragma unroll
            for (int q = 0; q < NPRE; ++q) {
              const int e = tid + CG_WG * q;
              if (e < TS * TS) pre[q] = rho[(e / TS) * Np + TS + e % TS];
            }
          }
          if constexpr (HX && HSEG && GLF_KW) {
            const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = tid & 63;
            auto pass = [&](auto pbc) {
              constexpr bool PB = decltype(pbc)::value;
#define QD_KW(w) \
  case w: herm_k_pass<w, PB>(A, T01, Tt, lane, slot); break;
              switch (wave) { QD_KW(0) QD_KW(1) QD_KW(2) QD_KW(3) QD_KW(4) QD_KW(5) QD_KW(6) default: QD_KW(7) }
#undef QD_KW
            };
            pass(std::false_type{});
            __syncthreads();
            pass(std::true_type{});
            __syncthreads();
          } else {
          visit([&](int row, int col, c128 v) {
            const int ti = row / TS, tj = col / TS, ra = row - ti * TS, cc = col - tj * TS;
            if (ti < tj) T01[ra * LD + cc] = v;
            else if (ti == tj && ra < cc) Tt[ti * TRI + slot(ra, cc)] = v;
            else if (ti == tj && ra == cc) Tt[ti * TRI + slot(ra, cc)] = cadd(v, cconj(v));
          });
          __syncthreads();
          visit([&](int row, int col, c128 v) {
            const int ti = row / TS, tj = col / TS, ra = row - ti * TS, cc = col - tj * TS;
            c128* t = ti > tj ? &T01[cc * LD + ra] : (ti == tj && ra > cc) ? &Tt[ti * TRI + slot(cc, ra)] : nullptr;
            if (t) *t = cadd(*t, cconj(v));
          });
          __syncthreads();
          }
          QD_TMARK(5);
          // round 0: tile (0, 1), element e -> (e / TS, TS + e % TS), k at T01; round 1: the two folded diagonal
          // triangles, element e -> k at Tt[e]
          auto place_rd = [&](auto rdc, int e, int& gi, int& gj) -> const c128* {
            constexpr int rd = decltype(rdc)::value;
            if (rd == 0) {
              gi = e / TS;
              gj = TS + e % TS;
              return &T01[gi * LD + e % TS];
            }
            const int ts = e / TRI, ff = e % TRI, u = ff / (TS + 1), v = ff % (TS + 1);
            const bool lo = v < TS - u;
            const int ra = lo ? u : TS - 1 - u;
            gi = ts * TS + ra;
            gj = ts * TS + (lo ? u + v : ra + v - (TS - u));
            return &Tt[e];
          };
          // Horner update of one upper element (i, j) with k, writing the mirror (j, i) as the conjugate
          auto update = [&](int gi, int gj, c128 k, c128 r0v) {
            const int id = gi * Np + gj, mid = gj * Np + gi;
            const c128 v = cadd(r0v, cscale(k, hc));
            rn[id] = v;
            if (gi != gj) rn[mid] = cconj(v);
          };
          auto round = [&](auto rdc) {
            constexpr int rd = decltype(rdc)::value;
            constexpr int NE = rd == 0 ? TS * TS : 2 * TRI;
            constexpr int NPER = (NE + CG_WG - 1) / CG_WG;
            constexpr int CH = NPER < QD_EPI_CH ? NPER : QD_EPI_CH;
            for (int q0 = 0; q0 < NPER; q0 += CH) {
              c128 r0[CH];
#pragma unroll
              for (int q = 0; q < CH; ++q) {
                const int e = tid + CG_WG * (q0 + q);
                if (q0 + q < NPER && (NE % CG_WG == 0 || e < NE)) {
                  int gi, gj;
                  place_rd(rdc, e, gi, gj);
                  if (NPRE && rd == 0 && q0 == 0 && q < NPRE) r0[q] = pre[q < NPRE ? q : 0];
                  else r0[q] = rho[gi * Np + gj];
                }
              }
#pragma unroll
              for (int q = 0; q < CH; ++q) {
                const int e = tid + CG_WG * (q0 + q);
                if (q0 + q >= NPER || (NE % CG_WG != 0 && e >= NE)) continue;
                int gi, gj;
                const c128 k = *place_rd(rdc, e, gi, gj);
                update(gi, gj, k, r0[q]);
              }
            }
          };
          round(std::integral_constant<int, 0>{});
          round(std::integral_constant<int, 1>{});
          __syncthreads();
        }
        QD_TMARK(3);
        continue;
      } else {
      // ---- phase 1: Y_c = C_c r
      for (int c = 0; c < nc; ++c) {
        for (int bm = 0; bm < nb; ++bm)
          for (int bn = 0; bn < nb; ++bn) {
            if (threadIdx.x == 0) {
              segs[0].A = p.Cop + (size_t)c * NN + (size_t)bm * BT * Np;
              segs[0].B = r + bn * BT;
            }
            __syncthreads();
            cg_block_gemm<BT>(segs, 1, Np, Np, Np, L, A);
            QD_TMARK(0);
            c128* Yc = Y + (size_t)c * NN;
            cg_epilogue<BT>(A, [&](int row, int col, c128 v) {
              Yc[(size_t)(bm * BT + row) * Np + bn * BT + col] = v;
            });
            QD_TMARK(1);
          }
      }
      __syncthreads();
      // ---- phase 2: k = (-iK) r + r (iK^+) + sum_c Y_c C_c^+ ; RK4 epilogue
      for (int bm = 0; bm < nb; ++bm)
        for (int bn = 0; bn < nb; ++bn) {
          if constexpr (!CHUNK) {
            if (threadIdx.x == 0) {
              segs[0].A = p.mK + (size_t)bm * BT * Np;
              segs[0].B = r + bn * BT;
              segs[1].A = r + (size_t)bm * BT * Np;
              segs[1].B = p.iKd + bn * BT;
              for (int c = 0; c < nc; ++c) {
                segs[2 + c].A = Y + (size_t)c * NN + (size_t)bm * BT * Np;
                segs[2 + c].B = p.Cd + (size_t)c * NN + bn * BT;
              }
            }
            __syncthreads();
            cg_block_gemm<BT>(segs, 2 + nc, Np, Np, Np, L, A);
          } else {
            for (int c0 = 0; c0 < nc; c0 += MAX_NC) {   // (P r, r Q) + the first MAX_NC pairs, then MAX_NC at a time
              const int first = c0 == 0 ? 2 : 0, cn = min(MAX_NC, nc - c0);
              if (threadIdx.x == 0) {
                segs[0].A = p.mK + (size_t)bm * BT * Np;
                segs[0].B = r + bn * BT;
                segs[1].A = r + (size_t)bm * BT * Np;
                segs[1].B = p.iKd + bn * BT;
                for (int c = 0; c < cn; ++c) {
                  segs[first + c].A = Y + (size_t)(c0 + c) * NN + (size_t)bm * BT * Np;
                  segs[first + c].B = p.Cd + (size_t)(c0 + c) * NN + bn * BT;
                }
              }
              __syncthreads();
              cg_block_gemm<BT>(segs, first + cn, Np, Np, Np, L, A, first != 0);
            }
          }
          QD_TMARK(2);
          cg_epilogue<BT>(A, [&](int row, int col, c128 k) {
            rk4_update((size_t)(bm * BT + row) * Np + bn * BT + col, k);
          });
          QD_TMARK(3);
        }
      __syncthreads();
      }
    }
    const int gs = p.step0 + step + 1;  // global step count after this step
    if (p.ne > 0) wg_observables(rho, p.eT, p.ne, NN, obs + (size_t)gs * p.ne, sred);
    if (p.snap && p.save_every > 0 && (gs % p.save_every) == 0) {
      const int s = gs / p.save_every - 1;
      if (s < p.nsave) {
        const int N = p.N;
        c128* out = p.snap + ((size_t)b * p.nsave + s) * N * N;
        for (size_t i = threadIdx.x; i < (size_t)N * N; i += CG_WG) {
          const int ii = (int)(i / N), jj = (int)(i % N);
          out[i] = rho[(size_t)ii * Np + jj];
        }
      }
    }
    __syncthreads();
    QD_TMARK(4);
  }
  QD_TIMING_FLUSH
}


}  // namespace
}  // namespace qd

namespace qd {
// The CHUNK instantiations of lindblad_rk4_kernel (nc > MAX_NC), one workgroup per matrix (glf_chunk.hip).
int glf_launch_chunk(const LindbladParams& p, int B, hipStream_t st);
// Few matrices as one persistent launch, a workgroup per 16 x 16 output tile (glf_single.hip).
int glf_single_max_batch(int Np, int nc, int herm = 0);
int glf_single_run(const c128* P, const c128* Q, const c128* Lop, const c128* Rop, int nc, const c128* eT, int ne,
                   c128* rho, int B, int N, int Np, double dt, int nsteps, c128* obs, c128* snap, int save_every,
                   const int** status_out, hipStream_t st, int herm = 0);
}  // namespace qd
