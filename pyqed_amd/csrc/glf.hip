// glf.hip — batched RK4 propagation of density matrices whose equation of
// motion has the "generalised Lindblad form" (GLF)
//     d rho/dt = P rho + rho Q + sum_c L_c rho R_c .
// Entry points: qd_glf_rk4 (caller supplies P, Q, L_c, R_c) and
// qd_lindblad_rk4 (builds P, Q, R_c from H and the collapse operators).
//
// Lindblad (replaces pyqed/oqs.py:1682-1690 _lindblad, RHS oqs.py:697-714,
// integrator phys.rk4 phys.py:1051-1064), mathematically identical to the
// reference RHS:
//   K    = H - (i/2) sum_c C_c^+ C_c ,  P = -iK , Q = iK^+ , L_c = C_c , R_c = C_c^+
//   L[r] = -i(H r - r H) + sum_c ( C_c r C_c^+ - 1/2 {C_c^+ C_c, r} )
// so one RHS costs 2 + 2*nc complex N^3 GEMMs (the reference spends 2 + 4*nc).
// Redfield in the H eigenbasis (oqs.py:519-570, R vec(rho) of oqs.py:462) is
// also GLF: P = -iE - sum_k A_k Lam_k, Q = iE - sum_k Lam_k^+ A_k, pairs
// (A_k, Lam_k^+) and (Lam_k, A_k) — see pyqed_amd/oqs.py.
//
// Kernel layout: one 512-thread workgroup owns one density matrix for the
// whole run (persistent over nsteps RK4 steps; only workgroup barriers, no
// inter-workgroup communication).  Per RK4 stage:
//   phase 1: Y_c = L_c * s                        (block GEMM, K = N)
//   phase 2: k   = P s + s Q + sum_c Y_c R_c      (one accumulator,
//            2+nc segments), fused epilogue s' = rho + c_m k.
// RK4 in Horner form: for a generator L that is constant over the step (every
// path here: H(t) of the driven runs is frozen per step, oqs.py:1780-1786),
// the classical RK4 update equals the degree-4 Taylor polynomial
//   rho' = rho + dt L(rho + dt/2 L(rho + dt/3 L(rho + dt/4 L rho)))
// so stage m reads s_m (s_0 = rho) and writes s_{m+1} = rho + dt/(4-m) L s_m,
// s_4 = rho'.  No RK4 accumulator: the epilogue reads rho and writes s_{m+1}
// (round 2 also read and wrote acc).  Equal to phys.rk4 (phys.py:1051-1064)
// in exact arithmetic; the tests hold it to the oracle's RK4 at 1e-12.
// s (one buffer for a single GEMM block, else two alternating) and Y_c live
// in a per-workgroup scratch slab in HBM (L2/MALL resident in practice).
// Matrices are zero-padded to Np = 32, 64 or a multiple of 128 so every GEMM
// tile is full; the padding stays exactly zero through the propagation.
// The complex GEMM engine's next-tile LDS stores issue before k-step 2 of 4 in this file's kernels (cgemm_block.hpp
// default 3): with the Hermitian epilogue's round-0 loads issued before its LDS passes (GLF_EPI_PRE 4) and 8-element
// Horner chunks, 351.5k -> 357.6k DM-steps/s on the headline batch (profiles/r06/lindblad/epilogue_knobs.txt)
#define CG_STAGE_AT 2
#include "glf_kernel.hpp"

namespace qd {
namespace {

// ---------------------------------------------------------------- operator prep
// S = sum_c C_c^+ C_c, K = H - (i/2) S.  Writes P = -iK, Q = iH - S/2 = i(H + (i/2) S), padded C, C^+, E^T,
// so that P rho + rho Q + sum_c C rho C^+ is oqs.liouvillian (oqs.py:697-714) term by term:
// -i(H rho - rho H) - (1/2)(S rho + rho S) + sum_c C rho C^+.  Q is formed from H itself (not from K^+), so
// a non-Hermitian H gives the reference's -i[H, rho] exactly.
__global__ void lindblad_prep_kernel(const c128* H, const c128* C, int nc, const c128* E, int ne, int N, int Np,
                                     c128* Cop, c128* mK, c128* iKd, c128* Cd, c128* eT) {
  const size_t NN = (size_t)Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / Np), j = (int)(e % Np);
    const bool in = (i < N) && (j < N);
    c128 K = cmk(0, 0), Qv = cmk(0, 0);
    if (in) {
      const c128 h = H[(size_t)i * N + j];
      c128 s = cmk(0, 0);
      for (int c = 0; c < nc; ++c) {
        const c128* Cc = C + (size_t)c * N * N;
        for (int k = 0; k < N; ++k) s = cadd(s, cmul(cconj(Cc[(size_t)k * N + i]), Cc[(size_t)k * N + j]));
      }
      K = csub(h, cmuli(cscale(s, 0.5)));    // H - (i/2) S
      Qv = csub(cmuli(h), cscale(s, 0.5));   // iH - S/2
    }
    mK[e] = cmulmi(K);  // P[i][j] = (-iK)[i][j]
    iKd[e] = Qv;        // Q[i][j]
    for (int c = 0; c < nc; ++c) {
      const c128 v = in ? C[(size_t)c * N * N + (size_t)i * N + j] : cmk(0, 0);
      Cop[c * NN + e] = v;
      Cd[c * NN + (size_t)j * Np + i] = cconj(v);
    }
    for (int m = 0; m < ne; ++m) {
      const c128 v = in ? E[(size_t)m * N * N + (size_t)j * N + i] : cmk(0, 0);
      eT[m * NN + e] = v;  // eT[i][j] = E[j][i]
    }
  }
}

// GLF operators supplied by the caller: pad/copy P, Q, L_c, R_c and E^T into
// the kernel's operator workspace.
__global__ void glf_prep_kernel(const c128* P, const c128* Q, const c128* Lop, const c128* Rop, int nc,
                                const c128* E, int ne, int N, int Np, c128* Cop, c128* mK, c128* iKd, c128* Cd,
                                c128* eT) {
  const size_t NN = (size_t)Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / Np), j = (int)(e % Np);
    const bool in = (i < N) && (j < N);
    const size_t src = (size_t)i * N + j;
    mK[e] = in ? P[src] : cmk(0, 0);
    iKd[e] = in ? Q[src] : cmk(0, 0);
    for (int c = 0; c < nc; ++c) {
      Cop[c * NN + e] = in ? Lop[(size_t)c * N * N + src] : cmk(0, 0);
      Cd[c * NN + e] = in ? Rop[(size_t)c * N * N + src] : cmk(0, 0);
    }
    for (int m = 0; m < ne; ++m) eT[m * NN + e] = in ? E[(size_t)m * N * N + (size_t)j * N + i] : cmk(0, 0);
  }
}

__global__ void pad_kernel(const c128* src, c128* dst, int B, int N, int Np) {
  const size_t tot = (size_t)B * Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const size_t b = e / ((size_t)Np * Np);
    const int r = (int)((e / Np) % Np), c = (int)(e % Np);
    dst[e] = (r < N && c < N) ? src[(b * N + r) * N + c] : cmk(0, 0);
  }
}

// dst = src when *guard != 0 (restores the saved state behind a single-trajectory launch that timed out)
__global__ void guarded_copy_kernel(const c128* src, c128* dst, size_t n, const int* guard) {
  if (__hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    dst[e] = src[e];
}

__global__ void unpad_kernel(const c128* src, c128* dst, int B, int N, int Np) {
  const size_t tot = (size_t)B * N * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const size_t b = e / ((size_t)N * N);
    const int r = (int)((e / N) % N), c = (int)(e % N);
    dst[e] = src[(b * Np + r) * Np + c];
  }
}

// Batched basis transform, one workgroup per matrix:
//   mode 0: A <- V^+ A V   (phys.transform(A, V), pyqed/phys.py:1121-1137)
//   mode 1: A <- V A V^+   (transform(A, dag(V)), the back-transform of oqs.py:450)
template <int BT>
__global__ __launch_bounds__(CG_WG) void basis_transform_kernel(const c128* Vl, const c128* Vr, c128* A, c128* T,
                                                                int Np) {
  __shared__ CgLds<BT> L;
  const size_t NN = (size_t)Np * Np;
  c128* Ab = A + (size_t)blockIdx.x * NN;
  c128* Tb = T + (size_t)blockIdx.x * NN;
  const int nb = Np / BT;
  CgAcc<BT> acc;
  __shared__ CgSeg seg[1];
  for (int bm = 0; bm < nb; ++bm)
    for (int bn = 0; bn < nb; ++bn) {  // T = Vl * A
      if (threadIdx.x == 0) {
        seg[0].A = Vl + (size_t)bm * BT * Np;
        seg[0].B = Ab + bn * BT;
      }
      __syncthreads();
      cg_block_gemm<BT>(seg, 1, Np, Np, Np, L, acc);
      cg_epilogue<BT>(acc, [&](int r, int c, c128 v) { Tb[(size_t)(bm * BT + r) * Np + bn * BT + c] = v; });
    }
  __syncthreads();
  for (int bm = 0; bm < nb; ++bm)
    for (int bn = 0; bn < nb; ++bn) {  // A = T * Vr
      if (threadIdx.x == 0) {
        seg[0].A = Tb + (size_t)bm * BT * Np;
        seg[0].B = Vr + bn * BT;
      }
      __syncthreads();
      cg_block_gemm<BT>(seg, 1, Np, Np, Np, L, acc);
      cg_epilogue<BT>(acc, [&](int r, int c, c128 v) { Ab[(size_t)(bm * BT + r) * Np + bn * BT + c] = v; });
    }
}

// Vl, Vr (padded) from V: mode 0 -> Vl = V^+, Vr = V ; mode 1 -> Vl = V, Vr = V^+
__global__ void transform_prep_kernel(const c128* V, int N, int Np, int mode, c128* Vl, c128* Vr) {
  const size_t NN = (size_t)Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / Np), j = (int)(e % Np);
    const bool in = i < N && j < N;
    const c128 v = in ? V[(size_t)i * N + j] : cmk(0, 0);          // V[i][j]
    const c128 vd = in ? cconj(V[(size_t)j * N + i]) : cmk(0, 0);  // V^+[i][j]
    Vl[e] = mode == 0 ? vd : v;
    Vr[e] = mode == 0 ? v : vd;
  }
}

// Vl = L, Vr = R (padded), for the general two-sided product A <- L A R
__global__ void sandwich_prep_kernel(const c128* Lm, const c128* Rm, int N, int Np, c128* Vl, c128* Vr) {
  const size_t NN = (size_t)Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / Np), j = (int)(e % Np);
    const bool in = i < N && j < N;
    Vl[e] = in ? Lm[(size_t)i * N + j] : cmk(0, 0);
    Vr[e] = in ? Rm[(size_t)i * N + j] : cmk(0, 0);
  }
}

// ---------------------------------------------------------------- split path (small batches)
// A persistent workgroup per density matrix leaves most of the chip idle when B is small (one
// trajectory = one CU).  Here every BT x BT output block of a stage phase is a workgroup of its own,
// and the phases are kernel launches:
//   glf_split_y_kernel  grid (nb^2, nc, B):  Y_c[bm, bn] = L_c[bm, :] r[:, bn]
//   glf_split_k_kernel  grid (nb^2, 1, B):   k[bm, bn] = P r + r Q + sum_c Y_c R_c (2 + nc segments),
//                                            fused RK4 epilogue of the block (same order as the
//                                            persistent kernel's rk4_update)
// Stage buffers: stage 0 reads rho, then scratch 0 / 1 alternate; stage 3 writes rho only, which is the
// next step's stage-0 input (Horner stages, see the file header).  Scratch per matrix: [buf0, buf1, Y_0 .. Y_nc-1].
__device__ __forceinline__ c128* split_buf(const LindbladParams& p, int b, int which) {
  const size_t NN = (size_t)p.Np * p.Np;
  if (which == 0) return p.rho + (size_t)b * NN;
  return p.ws + (size_t)b * (2 + p.nc) * NN + (size_t)(which - 1) * NN;
}

// Split-K (small batches): the k-phase (2 + nc segments) and Y-phase K-tiles of one output block are dealt
// to `S` workgroups; each writes its partial block to a slab and takes an arrival ticket, and the last to
// arrive sums the S slabs in the fixed order s = 0 .. S-1 (deterministic) and runs the block's epilogue.
// No workgroup waits on another (no co-residency needed); the last arriver resets the ticket for the next
// launch.  Visibility without L2 write-back fences (MI355X_MICROARCH.md "Valid forms",
// cdna_hip_programming.md §6 G16): every slab store is an agent-scope relaxed atomic store (write-through
// `sc1`), drained (vmcnt(0)) before the workgroup barrier and the ticket, and every slab load of the last
// arriver an agent-scope relaxed atomic load (`sc1`).  (Plain stores + __threadfence() per thread measured
// 1.5-2x slower than no split at all: each release fence writes back the L2.)
// Invariant this relies on (MI355X_MICROARCH.md "Valid forms", hand-off table row 1 -- the sc1 form that
// replaces an agent release/acquire pair; keep ALL of these when editing):
//   (1) every store of a slab is slab_st (agent-scope atomic store = global_store ... sc1, write-through);
//   (2) every load of a slab by the last arriver is slab_ld (agent-scope atomic load = global_load ... sc1),
//       never a plain or flat load, so no stale L1/L2 line can serve it;
//   (3) every storing wave drains its stores (s_waitcnt vmcnt(0)) before the workgroup barrier, and ONE lane
//       takes the ticket behind that barrier for all the workgroup's stores;
//   (4) the consumer is the workgroup whose fetch_add returned S-1; its other waves load only after the second
//       __syncthreads(), which they join after lane 0's add has returned.
// __syncthreads() is also the compiler barrier that keeps the slab stores above, and the slab loads below, the
// ticket; the asm's "memory" clobber keeps the stores above the drain.
__device__ __forceinline__ void slab_st(c128* p, c128 v) {
  __hip_atomic_store(&p->re, v.re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&p->im, v.im, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ c128 slab_ld(const c128* p) {
  return cmk(__hip_atomic_load(&p->re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_load(&p->im, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <typename Pol>
struct CgOffset {  // a K-tile policy shifted by t0 tiles
  using Raw = typename Pol::Raw;
  Pol pol;
  int t0;
  __device__ __forceinline__ Raw fetch(int t, int e, int q) const { return pol.fetch(t + t0, e, q); }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int t, int e, int q) const {
    return pol.finish(r, t + t0, e, q);
  }
};

// tiles [T s / S, T (s+1) / S) of the segment list `segs` (each segment tps tiles deep) into A
template <int BT>
__device__ __forceinline__ void split_gemm_range(const CgSeg* segs, int tps, int ld, int T, int s, int S, CgLds<BT>& L,
                                                 CgAcc<BT>& A) {
  const int t0 = (int)((long)T * s / S), t1 = (int)((long)T * (s + 1) / S);
  CgOffset<CgSegA<BT>> pa{CgSegA<BT>{segs, tps, ld}, t0};
  CgOffset<CgSegB<BT>> pb{CgSegB<BT>{segs, tps, ld}, t0};
  split_gemm<BT>(t1 - t0, pa, pb, L, A);
}

// Publish this workgroup's partial block and return true in the last arriver (all threads agree).
template <int BT>
__device__ __forceinline__ bool split_arrive(const CgAcc<BT>& A, c128* slab_s, unsigned* ticket, int S) {
  __shared__ int last;
  cg_epilogue<BT>(A, [&](int row, int col, c128 v) { slab_st(slab_s + row * BT + col, v); });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores are complete
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (old == (unsigned)(S - 1));
    if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last;
}

template <int BT>
__global__ __launch_bounds__(CG_WG) void glf_split_y_kernel(LindbladParams p) {
  __shared__ CgLds<BT> L;
  __shared__ CgSeg segs[1];
  const int nb = p.Np / BT, bm = blockIdx.x / nb, bn = blockIdx.x % nb, c = blockIdx.y;
  const int S = p.ys, b = blockIdx.z / S, s = blockIdx.z % S;
  const int Np = p.Np;
  const size_t NN = (size_t)Np * Np;
  const c128* r = split_buf(p, b, p.rin);
  c128* Yc = p.ws + (size_t)b * (2 + p.nc) * NN + (size_t)(2 + c) * NN;
  if (threadIdx.x == 0) {
    segs[0].A = p.Cop + (size_t)c * NN + (size_t)bm * BT * Np;
    segs[0].B = r + bn * BT;
  }
  __syncthreads();
  CgAcc<BT> A;
  auto store = [&](int row, int col, c128 v) { Yc[(size_t)(bm * BT + row) * Np + bn * BT + col] = v; };
  if (S == 1) {
    split_block_gemm<BT>(segs, 1, Np, Np, Np, L, A);
    cg_epilogue<BT>(A, store);
    return;
  }
  split_gemm_range<BT>(segs, Np / CG_KT, Np, Np / CG_KT, s, S, L, A);
  const size_t blk = ((size_t)b * p.nc + c) * nb * nb + blockIdx.x;
  c128* slab = p.yslab + blk * S * BT * BT;
  if (!split_arrive<BT>(A, slab + (size_t)s * BT * BT, p.ticket + (size_t)(gridDim.z / S) * nb * nb + blk, S)) return;
  for (int e = threadIdx.x; e < BT * BT; e += CG_WG) {
    c128 v = slab_ld(slab + e);
    for (int q = 1; q < S; ++q) v = cadd(v, slab_ld(slab + (size_t)q * BT * BT + e));
    store(e / BT, e % BT, v);
  }
}

// Horner epilogue of one element of the block (the persistent kernel's rk4_update): rn = rho + dt / (4 - stage) k,
// rn = rho at stage 3
__device__ __forceinline__ void split_rk4(const LindbladParams& p, c128* rho, c128* rn, size_t idx, c128 k) {
  (p.stage == 3 ? rho : rn)[idx] = cadd(rho[idx], cscale(k, glf_horner_coef(p.dt, p.stage)));
}

template <int BT>
__global__ __launch_bounds__(CG_WG) void glf_split_k_kernel(LindbladParams p) {
  __shared__ CgLds<BT> L;
  __shared__ CgSeg segs[2 + MAX_NC];
  const int nb = p.Np / BT, bm = blockIdx.x / nb, bn = blockIdx.x % nb;
  const int S = p.ks, b = blockIdx.y / S, s = blockIdx.y % S;
  const int Np = p.Np, nc = p.nc;
  const size_t NN = (size_t)Np * Np;
  const c128* r = split_buf(p, b, p.rin);
  c128* rn = p.rout ? split_buf(p, b, p.rout) : nullptr;
  c128* rho = p.rho + (size_t)b * NN;
  const c128* Y = p.ws + (size_t)b * (2 + nc) * NN + 2 * NN;
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
  CgAcc<BT> A;
  if (S == 1) {
    split_block_gemm<BT>(segs, 2 + nc, Np, Np, Np, L, A);
    cg_epilogue<BT>(A, [&](int row, int col, c128 k) {
      split_rk4(p, rho, rn, (size_t)(bm * BT + row) * Np + bn * BT + col, k);
    });
    return;
  }
  split_gemm_range<BT>(segs, Np / CG_KT, Np, (2 + nc) * (Np / CG_KT), s, S, L, A);
  const size_t blk = (size_t)b * nb * nb + blockIdx.x;
  c128* slab = p.kslab + blk * S * BT * BT;
  if (!split_arrive<BT>(A, slab + (size_t)s * BT * BT, p.ticket + blk, S)) return;
  for (int e = threadIdx.x; e < BT * BT; e += CG_WG) {
    c128 k = slab_ld(slab + e);
    for (int q = 1; q < S; ++q) k = cadd(k, slab_ld(slab + (size_t)q * BT * BT + e));
    split_rk4(p, rho, rn, (size_t)(bm * BT + e / BT) * Np + bn * BT + e % BT, k);
  }
}

// ---- Hermitian split path (Lindblad, exactly Hermitian rho, batches below the persistent kernel's range)
// k = X + X^+ with X = P r + sum_c Y_c (C_c^+ / 2) (the persistent Hermitian kernel's form), one workgroup per block
// PAIR (bm <= bn) of the upper block triangle instead of one per block: the pair's workgroup computes
//   X(bm, bn) with the Hermitian part C r C^+ in full (A operand Y doubled in the staging, exact), and
//   X(bn, bm) = (P r)(bn, bm) only (C r C^+ is Hermitian, so its lower block is redundant),
// and forms k on the upper block, k_ij = X_ij + conj(X_ji), through an LDS transpose; a diagonal block takes the
// half-weighted X and its own transpose.  The Horner update runs on the upper elements (rho read there) and writes each mirror as the conjugate.  Work per stage at n_c = 1 and nb x nb blocks: nb^2 Y blocks
// + nb(nb-1)/2 x 3 + nb x 2 X segment-blocks, against nb^2 x 4 for the general split path (nb = 4: 42 vs 64).
template <int BT>
struct CgSegAScaled {   // CgSegA with the segments >= 1 multiplied by `scale` as they are staged
  using Raw = cg_v2;
  const CgSeg* segs;
  int tps, lda;
  double scale;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    const CgSeg sg = segs[t / tps];
    return cg_ld(sg.A + (size_t)(e >> 4) * lda + (t % tps) * CG_KT + (e & 15));
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int t, int, int) const {
    return t >= tps ? cg_v2{r.x * scale, r.y * scale} : r;
  }
};

__device__ __forceinline__ void split_herm_rk4(const LindbladParams& p, c128* rho, c128* rn, int gi, int gj, c128 k) {
  const int Np = p.Np;
  const size_t id = (size_t)gi * Np + gj, mid = (size_t)gj * Np + gi;
  c128* out = p.stage == 3 ? rho : rn;
  const c128 v = cadd(rho[id], cscale(k, glf_horner_coef(p.dt, p.stage)));
  out[id] = v;
  if (gi != gj) out[mid] = cconj(v);
}

// Each off-diagonal pair's two GEMMs run on two workgroups (grid x = pairs + off-diagonal pairs): the pair's
// workgroup computes XU (16 K-tiles at N_p = 128, n_c = 1), an extra workgroup XL (8 K-tiles), so the longest
// workgroup does not run all 24 (round 3's one-workgroup-per-pair form, removed in round 5).  Both publish their
// block to a slab (write-through) and take the pair's arrival ticket (split_arrive, the split-K hand-off); the last
// arriver forms k from its own accumulator and the other's slab and runs the update.  A diagonal block takes the
// half-weighted X and its own transpose.
template <int BT>
__global__ __launch_bounds__(CG_WG) void glf_split_hk2_kernel(LindbladParams p) {
  __shared__ CgLds<BT> L;
  __shared__ CgSeg segs[1 + MAX_NC];
  const int nb = p.Np / BT, npairs = nb * (nb + 1) / 2, noff = nb * (nb - 1) / 2;
  // grid (B, pairs + off-diagonal pairs): the linear dispatch order runs every matrix's 16-K-tile workgroups (XU and
  // diagonal blocks) before the 8-K-tile XL ones, so the short workgroups fill the launch's tail
  const int role = blockIdx.y;
  const bool xl_role = role >= npairs;
  int bm = 0, bn, oj = -1;   // (bm, bn) block pair; oj = its index among the off-diagonal pairs (row-major)
  if (!xl_role) {
    int pi = role;
    while (pi >= nb - bm) {
      pi -= nb - bm;
      ++bm;
    }
    bn = bm + pi;
    if (bm < bn) oj = bm * (nb - 1) - bm * (bm - 1) / 2 + (bn - bm - 1);
  } else {
    oj = role - npairs;
    int j = oj;
    while (j >= nb - 1 - bm) {
      j -= nb - 1 - bm;
      ++bm;
    }
    bn = bm + 1 + j;
  }
  const int b = blockIdx.x;
  const int Np = p.Np, nc = p.nc;
  const size_t NN = (size_t)Np * Np;
  const c128* r = split_buf(p, b, p.rin);
  c128* rn = p.rout ? split_buf(p, b, p.rout) : nullptr;
  c128* rho = p.rho + (size_t)b * NN;
  const c128* Y = p.ws + (size_t)b * (2 + nc) * NN + 2 * NN;
  const int tps = Np / CG_KT;
  constexpr int LD = BT + 1;
  static_assert(BT * LD * sizeof(c128) <= sizeof(CgLds<BT>), "LDS transpose buffer");
  c128* T = reinterpret_cast<c128*>(&L);
  auto put = [&](int row, int col, c128 v) { T[row * LD + col] = v; };
  auto update = [&](int row, int col, c128 v) {
    if (bm == bn && row > col) return;
    split_herm_rk4(p, rho, rn, bm * BT + row, bn * BT + col, cadd(v, cconj(T[col * LD + row])));
  };
  c128* slab = oj >= 0 ? p.kslab + ((size_t)b * (noff > 0 ? noff : 1) + oj) * 2 * BT * BT : nullptr;   // [XU, XL]
  unsigned* ticket = p.ticket + (size_t)b * nb * nb + (oj >= 0 ? oj : 0);
  CgAcc<BT> X;
  if (!xl_role) {
    if (threadIdx.x == 0) {
      segs[0].A = p.mK + (size_t)bm * BT * Np;
      segs[0].B = r + bn * BT;
      for (int c = 0; c < nc; ++c) {
        segs[1 + c].A = Y + (size_t)c * NN + (size_t)bm * BT * Np;
        segs[1 + c].B = p.Cd + (size_t)c * NN + bn * BT;
      }
    }
    __syncthreads();
    CgSegAScaled<BT> pa{segs, tps, Np, bm < bn ? 2.0 : 1.0};
    CgSegB<BT> pb{segs, tps, Np};
    split_gemm<BT>((1 + nc) * tps, pa, pb, L, X);
    if (bm == bn) {   // diagonal block: its own transpose
      cg_epilogue<BT>(X, put);
      __syncthreads();
      cg_epilogue<BT>(X, update);
      return;
    }
    if (!split_arrive<BT>(X, slab, ticket, 2)) return;
    for (int e = threadIdx.x; e < BT * BT; e += CG_WG) T[(e / BT) * LD + e % BT] = slab_ld(slab + BT * BT + e);
    __syncthreads();
    cg_epilogue<BT>(X, update);
    return;
  }
  if (threadIdx.x == 0) {
    segs[0].A = p.mK + (size_t)bn * BT * Np;
    segs[0].B = r + bm * BT;
  }
  __syncthreads();
  CgSegA<BT> pa{segs, tps, Np};
  CgSegB<BT> pb{segs, tps, Np};
  split_gemm<BT>(tps, pa, pb, L, X);
  if (!split_arrive<BT>(X, slab + BT * BT, ticket, 2)) return;
  cg_epilogue<BT>(X, put);
  __syncthreads();
  for (int e = threadIdx.x; e < BT * BT; e += CG_WG) update(e / BT, e % BT, slab_ld(slab + e));
}

// Observables / snapshot of global step gs (after it; gs = 0: the initial state), one workgroup per matrix.
__global__ __launch_bounds__(CG_WG) void glf_split_obs_kernel(LindbladParams p, int gs) {
  __shared__ c128 sred[CG_WG / 64];
  const int b = blockIdx.x;
  const size_t NN = (size_t)p.Np * p.Np;
  const c128* rho = p.rho + (size_t)b * NN;
  if (p.ne > 0) wg_observables(rho, p.eT, p.ne, NN, p.obs + ((size_t)b * (p.total_steps + 1) + gs) * p.ne, sred);
  if (gs > 0 && p.snap && p.save_every > 0 && (gs % p.save_every) == 0) {
    const int s = gs / p.save_every - 1;
    if (s < p.nsave) {
      const int N = p.N;
      c128* out = p.snap + ((size_t)b * p.nsave + s) * N * N;
      for (size_t i = threadIdx.x; i < (size_t)N * N; i += CG_WG) {
        const int ii = (int)(i / N), jj = (int)(i % N);
        out[i] = rho[(size_t)ii * p.Np + jj];
      }
    }
  }
}

int padded_dim(int N) {
  if (N <= 32) return 32;
  if (N <= 64) return 64;
  return ((N + 127) / 128) * 128;
}

}  // namespace
}  // namespace qd

using namespace qd;

namespace {

enum GlfSource { GLF_FROM_LINDBLAD = 0, GLF_FROM_OPERATORS = 1 };

// Shared driver of qd_lindblad_rk4 / qd_glf_rk4.
// H(t) = H0 - sum_d f_d Hd_d (time-dependent Hamiltonian of _lindblad_driven, oqs.py:1725-1732, constant
// within a step; f is complex, so H(t) need not be Hermitian):  P = P0 + i sum_d f_d Hd_d,
// Q = Q0 - i sum_d f_d Hd_d, with P0 = -iK0 and Q0 = iH0 - S/2 saved at the start of the run.
__global__ void driven_update_kernel(const c128* P0, const c128* Q0, const c128* Hd, int nd, const c128* f, int N,
                                     int Np, c128* mK, c128* iKd) {
  const size_t NN = (size_t)Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / Np), j = (int)(e % Np);
    c128 fh = cmk(0, 0);
    if (i < N && j < N)
      for (int d = 0; d < nd; ++d) fh = cadd(fh, cmul(f[d], Hd[(size_t)d * N * N + (size_t)i * N + j]));
    mK[e] = cadd(P0[e], cmuli(fh));
    iKd[e] = csub(Q0[e], cmuli(fh));
  }
}

__global__ void save_pq0_kernel(const c128* mK, const c128* iKd, size_t NN, c128* P0, c128* Q0) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    P0[e] = mK[e];
    Q0[e] = iKd[e];
  }
}

__global__ void scale_kernel(c128* a, size_t n, double s) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    a[e] = cscale(a[e], s);
}

int glf_run(GlfSource src, const c128* H, const c128* C, const c128* P, const c128* Q, const c128* Lop,
            const c128* Rop, int nc, c128* rho, int B, int N, double dt, int nsteps, const c128* E, int ne,
            c128* obs, c128* snap, int save_every, hipStream_t st, const c128* Hd = nullptr, int nd = 0,
            const qd_c128* fvals = nullptr, int herm = 0) {
  WsScope wss_(st);  // call-scoped scratch (qd_runtime.hip)
  const int Np = padded_dim(N);
  const size_t NN = (size_t)Np * Np;
  // operator workspace: Cop(L), mK(P), iKd(Q), Cd(R), eT, [P0, Q0, f scratch for driven runs]
  const size_t ops_elems = (size_t)(2 + 2 * nc + ne + (nd ? 2 : 0)) * NN + (size_t)nd * nsteps;
  void* wops = nullptr;
  int rc = workspace(WS_LINDBLAD_OPS, ops_elems * sizeof(c128), &wops, st);
  if (rc) return rc;
  c128* Cop = (c128*)wops;
  c128* mK = Cop + (size_t)nc * NN;
  c128* iKd = mK + NN;
  c128* Cd = iKd + NN;
  c128* eT = Cd + (size_t)nc * NN;
  c128* P0 = eT + (size_t)ne * NN;
  c128* Q0 = P0 + (nd ? NN : 0);
  c128* fdev = Q0 + (nd ? NN : 0);
  // state workspace: per-matrix scratch (+ padded rho when N != Np)
  const bool pad = (Np != N);
  if (Np > 128) herm = 0;  // the Hermitian path is single-block
  // Paths (QD_OPT_GLF_PATH forces one where it applies; otherwise the batch shape decides):
  //  - single-trajectory launch (glf_single.hip) for few undriven non-Hermitian matrices, below;
  //  - split path (glf_split_*): each output block of a phase is a workgroup, for batches too small to occupy the chip
  //    with one persistent workgroup per matrix.  Measured (tools/glf_split_bench.py, N = 128 / 256, B = 1 .. 256):
  //    it wins below ~192 matrices at Np <= 128 (6.6x at one trajectory) and at every batch size above Np = 128; the
  //    block is the largest BT < Np that still gives >= 512 workgroups, else 32.  nc > MAX_NC: the persistent
  //    kernels' chunked segment lists (the split kernels hold one LDS table);
  //  - Hermitian Lindblad batches at Np = 128 below 208 matrices: the pair-block split path (glf_split_hk2_kernel,
  //    32-blocks; tools/glf_hsplit_sweep.sh: 198k / 233k / 258k / 264k DM-steps/s at 64 / 128 / 192 / 224 matrices
  //    against 82k / 164k / 242k / 278k for the persistent kernel);
  //  - else the persistent kernel (a workgroup per matrix).
#ifndef GLF_HSPLIT_Y64
#define GLF_HSPLIT_Y64 1
#endif
  const int force = option(QD_OPT_GLF_PATH);
  int split_bt = 0;
  bool hsplit = false;
  {
#ifndef GLF_SPLIT_MINWG
#define GLF_SPLIT_MINWG 512
#endif
    int bt = 32;
    for (int v : {128, 64}) {
      if (v < Np && Np % v == 0 && (long)B * (Np / v) * (Np / v) >= GLF_SPLIT_MINWG) {
        bt = v;
        break;
      }
    }
    const bool split_ok = !herm && Np >= 64 && nc <= MAX_NC;
    const bool hsplit_ok = herm && src == GLF_FROM_LINDBLAD && Np == 128 && nc <= MAX_NC;
    const bool want_split = force == QD_GLF_SPLIT || (force == QD_GLF_AUTO && (Np > 128 || B < (herm ? 208 : 192)));
    if (want_split && split_ok) split_bt = bt;
    if (want_split && hsplit_ok) {
      hsplit = true;
      split_bt = 32;
    }
  }
  // Split-K of the (general) split path when its blocks leave the chip under-filled: up to 256 workgroups per phase,
  // >= 3 K-tiles each, at most 4 (k phase) / 8 (Y phase) partial slabs per block.  Measured (N = 128 / 256, one
  // trajectory, tools/ks_sweep.sh): 4 k-splits 12.0k / 6.9k steps/s, 8: 11.8k / 6.6k, 16: 9.8k / 5.8k, none: 8.4k / 4.2k.
  int ks = 1, ys = 1;
  // the Hermitian pair path's Y launch takes 64-blocks (all eight waves of a workgroup issuing MFMAs) from two per CU:
  // 128 matrices 288k -> 293k DM-steps/s, 64 matrices (one per CU) 255k -> 254k (profiles/r05/lindblad/y64_ab.txt)
  const int y_bt = (hsplit && GLF_HSPLIT_Y64 && (long)B * (Np / 64) * (Np / 64) >= 512) ? 64 : split_bt;
  if (split_bt) {
    const long blocks = (long)B * (Np / split_bt) * (Np / split_bt);
    const long yblocks = (long)B * (Np / y_bt) * (Np / y_bt);
    const int Tk = (2 + nc) * (Np / CG_KT), Ty = Np / CG_KT;
    ks = hsplit ? 1 : (int)std::max(1L, std::min<long>({4L, 256L / blocks, (long)Tk / 3}));
    ys = nc ? (int)std::max(1L, std::min<long>({8L, 256L / (yblocks * nc), (long)Ty / 3})) : 1;
  }
  // Hermitian pairs on two workgroups each: one N_p^2 slab slot per matrix holds the off-diagonal pairs' XU / XL blocks
  const bool hk2 = hsplit;
  const int kslots = (ks > 1 ? ks : 0) + (hk2 ? 1 : 0);
  const size_t per = (size_t)(split_bt ? 2 + nc + kslots + (ys > 1 ? nc * ys : 0)
                                       : glf_slots(Np, nc, herm)) * NN;
  const size_t nticket = split_bt ? (size_t)B * (1 + nc) * (Np / std::min(split_bt, y_bt)) * (Np / std::min(split_bt, y_bt)) : 0;
  const size_t st_elems = (size_t)B * per + (pad ? (size_t)B * NN : 0) + (nticket + 3) / 4;
  void* wst = nullptr;
  rc = workspace(WS_LINDBLAD, st_elems * sizeof(c128), &wst, st);
  if (rc) return rc;
  c128* scratch = (c128*)wst;
  c128* rho_p = pad ? scratch + (size_t)B * per : rho;

  const int threads = 256;
  const int blocks = (int)std::min<size_t>((NN + threads - 1) / threads, 4096);
  if (src == GLF_FROM_LINDBLAD)
    hipLaunchKernelGGL(lindblad_prep_kernel, dim3(blocks), dim3(threads), 0, st, H, C, nc, E, ne, N, Np, Cop, mK,
                       iKd, Cd, eT);
  else
    hipLaunchKernelGGL(glf_prep_kernel, dim3(blocks), dim3(threads), 0, st, P, Q, Lop, Rop, nc, E, ne, N, Np, Cop,
                       mK, iKd, Cd, eT);
  QD_HIP(hipGetLastError());
  if (herm && nc > 0 && src == GLF_FROM_LINDBLAD) {  // the Hermitian kernel consumes C_c^+ / 2
    hipLaunchKernelGGL(scale_kernel, dim3(blocks), dim3(threads), 0, st, Cd, (size_t)nc * NN, 0.5);
    QD_HIP(hipGetLastError());
  }
  if (nd) {
    hipLaunchKernelGGL(save_pq0_kernel, dim3(blocks), dim3(threads), 0, st, (const c128*)mK, (const c128*)iKd, NN,
                       P0, Q0);
    QD_HIP(hipGetLastError());
    if (nsteps > 0)
      if ((rc = upload(fdev, fvals, (size_t)nd * nsteps * sizeof(c128), st))) return rc;
  }
  if (pad) {
    const size_t tot = (size_t)B * NN;
    const int pb = (int)std::min<size_t>((tot + threads - 1) / threads, 65535);
    hipLaunchKernelGGL(pad_kernel, dim3(pb), dim3(threads), 0, st, rho, rho_p, B, N, Np);
    QD_HIP(hipGetLastError());
  }

  // Few undriven matrices: one persistent launch with a workgroup per 16 x 16 output tile (glf_single.hip; the split
  // path takes eight dependent launches per step).  A refused cooperative launch re-runs on the path the shape selects
  // (split, or persistent when the single path was forced).  A hand-off timeout is only known on the device: behind the
  // single launch the call queues a guarded restore of the saved initial state and a guarded run of the persistent
  // kernel (a workgroup per matrix), both no-ops unless the launch's status word reports the timeout -- no host wait.
  const int* single_guard = nullptr;
  void* wsave = nullptr;
  {
    // Hermitian Lindblad states at N_p = 128 (B <= 2, nc in {1, 2}) take the Hermitian single launch
    const bool hsingle = herm && src == GLF_FROM_LINDBLAD && B <= glf_single_max_batch(Np, nc, 1);
    const bool fits = !nd && (herm ? hsingle : B <= glf_single_max_batch(Np, nc));
    if (fits && (force == QD_GLF_AUTO || force == QD_GLF_SINGLE)) {
      if ((rc = workspace(WS_MISC, (size_t)B * NN * sizeof(c128), &wsave, st))) return rc;
      if ((rc = copy_device(wsave, rho_p, (size_t)B * NN * sizeof(c128), st))) return rc;
      rc = glf_single_run(mK, iKd, Cop, Cd, nc, eT, ne, rho_p, B, N, Np, dt, nsteps, obs,
                          save_every > 0 ? snap : nullptr, save_every, &single_guard, st, hsingle ? 1 : 0);
      if (rc == QD_OK && !single_guard) {   // nothing to run
        note_path("glf_single");
        return QD_OK;
      }
      if (rc == QD_OK) {
        note_path("glf_single");
        hipLaunchKernelGGL(guarded_copy_kernel, dim3(std::min<size_t>((B * NN + 255) / 256, 1024)), dim3(256), 0, st,
                           (const c128*)wsave, rho_p, (size_t)B * NN, single_guard);
        QD_HIP(hipGetLastError());
        split_bt = 0;   // the guarded re-run takes the persistent kernel
      } else {
        if (rc != QD_EBUSY) return rc;
        std::fprintf(stderr, "[libqdyn] glf single-trajectory launch refused; re-running on the split path\n");
      }
    }
  }

  LindbladParams p{};
  p.Cop = Cop;
  p.mK = mK;
  p.iKd = iKd;
  p.Cd = Cd;
  p.eT = eT;
  p.rho = rho_p;
  p.ws = scratch;
  p.obs = obs;
  p.snap = (save_every > 0) ? snap : nullptr;
  p.N = N;
  p.Np = Np;
  p.nc = nc;
  p.ne = ne;
  p.nsteps = nsteps;
  p.save_every = save_every;
  p.nsave = (save_every > 0) ? nsteps / save_every : 0;
  p.dt = dt;
  p.step0 = 0;
  p.total_steps = nsteps;
  p.herm = herm;
  p.hseg = herm && src == GLF_FROM_LINDBLAD;
  p.tbuf = nullptr;
  p.stage = p.rin = p.rout = 0;
  p.ks = ks;
  p.ys = ys;
  // split-K slabs after the per-matrix scratch of all B matrices; tickets after the padded copy
  p.kslab = split_bt ? scratch + (size_t)B * (2 + nc) * NN : nullptr;
  p.yslab = split_bt ? p.kslab + (size_t)B * kslots * NN : nullptr;
  p.ticket = split_bt ? (unsigned*)(scratch + (size_t)B * per + (pad ? (size_t)B * NN : 0)) : nullptr;
  p.guard = single_guard;
  if (split_bt && (ks > 1 || ys > 1 || hk2) && (rc = fill_bytes(p.ticket, 0, nticket * sizeof(unsigned), st))) return rc;
#ifdef QD_PHASE_TIMING
  const bool timing = true;  // diagnostics build: per-phase clocks to stderr
#else
  const bool timing = false;
#endif
  if (timing) {
    QD_HIP(hipMalloc(&p.tbuf, (size_t)B * 8 * sizeof(unsigned long long)));
    QD_HIP(hipMemsetAsync(p.tbuf, 0, (size_t)B * 8 * sizeof(unsigned long long), st));
  }

  auto launch_split = [&]() -> int {
    const int nb = Np / split_bt;
    auto obs_at = [&](int gs) -> int {
      hipLaunchKernelGGL(glf_split_obs_kernel, dim3(B), dim3(CG_WG), 0, st, p, gs);
      QD_HIP(hipGetLastError());
      return QD_OK;
    };
    int rc2;
    if (p.ne > 0 && p.step0 == 0 && (rc2 = obs_at(0))) return rc2;
    for (int s = 0; s < p.nsteps; ++s) {
      for (int stage = 0; stage < 4; ++stage) {
        p.stage = stage;
        p.rin = stage == 0 ? 0 : ((stage - 1) & 1) + 1;
        p.rout = stage == 3 ? 0 : (stage & 1) + 1;
#define QD_SPLIT(KERN, GRID)                                                                   \
  switch (split_bt) {                                                                            \
    case 32: hipLaunchKernelGGL(KERN<32>, GRID, dim3(CG_WG), 0, st, p); break;                   \
    case 64: hipLaunchKernelGGL(KERN<64>, GRID, dim3(CG_WG), 0, st, p); break;                   \
    default: hipLaunchKernelGGL(KERN<128>, GRID, dim3(CG_WG), 0, st, p); break;                  \
  }
        if (nc > 0) {
          const int ynb = Np / y_bt;
          if (y_bt == 64) hipLaunchKernelGGL(glf_split_y_kernel<64>, dim3(ynb * ynb, nc, B * ys), dim3(CG_WG), 0, st, p);
          else QD_SPLIT(glf_split_y_kernel, dim3(nb * nb, nc, B * ys));
          QD_HIP(hipGetLastError());
        }
        if (hk2) {   // split_bt is 32 here
          const unsigned np2 = nb * (nb + 1) / 2 + nb * (nb - 1) / 2;
          hipLaunchKernelGGL(glf_split_hk2_kernel<32>, dim3(B, np2), dim3(CG_WG), 0, st, p);
        } else {
          QD_SPLIT(glf_split_k_kernel, dim3(nb * nb, B * ks));
        }
        QD_HIP(hipGetLastError());
#undef QD_SPLIT
      }
      const int gs = p.step0 + s + 1;
      if ((p.ne > 0 || (p.snap && p.save_every > 0 && gs % p.save_every == 0)) && (rc2 = obs_at(gs))) return rc2;
    }
    return QD_OK;
  };
  note_path(single_guard ? "glf_single_guarded" : split_bt ? (hsplit ? "glf_split_pairs" : "glf_split")
                                                 : nc > MAX_NC ? "glf_persistent_chunk" : "glf_persistent");
  auto launch = [&]() -> int {
    if (split_bt) return launch_split();
    if (nc > MAX_NC) return glf_launch_chunk(p, B, st);   // glf_chunk.hip
    if (Np == 32) {
      if (herm) hipLaunchKernelGGL((lindblad_rk4_kernel<32, true>), dim3(B), dim3(CG_WG), 0, st, p);
      else hipLaunchKernelGGL((lindblad_rk4_kernel<32, false>), dim3(B), dim3(CG_WG), 0, st, p);
    } else if (Np == 64) {
      if (herm) hipLaunchKernelGGL((lindblad_rk4_kernel<64, true>), dim3(B), dim3(CG_WG), 0, st, p);
      else hipLaunchKernelGGL((lindblad_rk4_kernel<64, false>), dim3(B), dim3(CG_WG), 0, st, p);
    } else {
      if (herm && p.hseg) hipLaunchKernelGGL((lindblad_rk4_kernel<128, true, true>), dim3(B), dim3(CG_WG), 0, st, p);
      else if (herm) hipLaunchKernelGGL((lindblad_rk4_kernel<128, true>), dim3(B), dim3(CG_WG), 0, st, p);
      else hipLaunchKernelGGL((lindblad_rk4_kernel<128, false>), dim3(B), dim3(CG_WG), 0, st, p);
    }
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  if (!nd) {
    if ((rc = launch())) return rc;
  } else {
    // one launch per step: H(t_k) is constant within a step (oqs.py:1780-1786 evaluates it once per step)
    p.nsteps = 1;
    for (int k = 0; k < nsteps; ++k) {
      hipLaunchKernelGGL(driven_update_kernel, dim3(blocks), dim3(threads), 0, st, (const c128*)P0, (const c128*)Q0, Hd, nd,
                         (const c128*)fdev + (size_t)k * nd, N, Np, mK, iKd);
      QD_HIP(hipGetLastError());
      p.step0 = k;
      if ((rc = launch())) return rc;
    }
  }

  if (pad) {
    const size_t tot = (size_t)B * N * N;
    const int pb = (int)std::min<size_t>((tot + threads - 1) / threads, 65535);
    hipLaunchKernelGGL(unpad_kernel, dim3(pb), dim3(threads), 0, st, rho_p, rho, B, N, Np);
    QD_HIP(hipGetLastError());
  }
  if (timing) {
    std::vector<unsigned long long> t((size_t)B * 8);
    QD_HIP(hipStreamSynchronize(st));
    QD_HIP(hipMemcpy(t.data(), p.tbuf, t.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    (void)hipFree(p.tbuf);
    int dev = 0, khz = 100000;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    const char* names[6] = {"gemm1", "epi1", "gemm2", "epi2", "obs/snap", "epi2-lds"};
    std::fprintf(stderr, "[qd phase timing] N=%d B=%d herm=%d nsteps=%d, us per step (mean over workgroups):", N, B,
                 herm, nsteps);
    for (int q = 0; q < 6; ++q) {
      double s = 0;
      for (int b = 0; b < B; ++b) s += (double)t[(size_t)b * 8 + q];
      std::fprintf(stderr, " %s %.2f", names[q], s / B / (khz * 1e-3) / std::max(1, nsteps));
    }
    double cyc = 0, wt = 0;
    for (int b = 0; b < B; ++b) {
      cyc += (double)t[(size_t)b * 8 + 6];
      wt += (double)t[(size_t)b * 8 + 7];
    }
    std::fprintf(stderr, " | shader clock %.0f MHz\n", wt > 0 ? cyc / (wt / (khz * 1e3)) / 1e6 : 0.0);
  }
  return QD_OK;
}

int check_common(const char* fn, const void* rho, int B, int N, int nc, int ne, const void* E, const void* obs,
                 int nsteps) {
  QD_CHECK_ARG(rho, "%s: rho must be non-null", fn);
  QD_CHECK_ARG(N >= 1 && N <= 16384, "%s: N=%d outside [1, 16384]", fn, N);
  QD_CHECK_ARG(B >= 1, "%s: B=%d must be >= 1", fn, B);
  QD_CHECK_ARG(nc >= 0, "%s: nc=%d < 0", fn, nc);
  QD_CHECK_ARG(ne >= 0, "%s: ne=%d < 0", fn, ne);
  QD_CHECK_ARG(ne == 0 || (E && obs), "%s: E/obs null but ne=%d", fn, ne);
  QD_CHECK_ARG(nsteps >= 0, "%s: nsteps=%d < 0", fn, nsteps);
  return QD_OK;
}

}  // namespace

extern "C" int qd_lindblad_rk4(const qd_c128* H, const qd_c128* C, int nc, qd_c128* rho, int B, int N, double dt,
                               int nsteps, const qd_c128* E, int ne, qd_c128* obs, qd_c128* snap, int save_every,
                               void* stream) {
  QD_CHECK_ARG(H && rho, "qd_lindblad_rk4: H and rho must be non-null");
  int rc = check_common("qd_lindblad_rk4", rho, B, N, nc, ne, E, obs, nsteps);
  if (rc) return rc;
  QD_CHECK_ARG(nc == 0 || C, "qd_lindblad_rk4: C is null but nc=%d", nc);
  return glf_run(GLF_FROM_LINDBLAD, (const c128*)H, (const c128*)C, nullptr, nullptr, nullptr, nullptr, nc,
                 (c128*)rho, B, N, dt, nsteps, (const c128*)E, ne, (c128*)obs, (c128*)snap, save_every,
                 (hipStream_t)stream);
}

extern "C" int qd_lindblad_rk4_herm(const qd_c128* H, const qd_c128* C, int nc, qd_c128* rho, int B, int N,
                                    double dt, int nsteps, const qd_c128* E, int ne, qd_c128* obs, qd_c128* snap,
                                    int save_every, void* stream) {
  QD_CHECK_ARG(H && rho, "qd_lindblad_rk4_herm: H and rho must be non-null");
  int rc = check_common("qd_lindblad_rk4_herm", rho, B, N, nc, ne, E, obs, nsteps);
  if (rc) return rc;
  QD_CHECK_ARG(nc == 0 || C, "qd_lindblad_rk4_herm: C is null but nc=%d", nc);
  return glf_run(GLF_FROM_LINDBLAD, (const c128*)H, (const c128*)C, nullptr, nullptr, nullptr, nullptr, nc,
                 (c128*)rho, B, N, dt, nsteps, (const c128*)E, ne, (c128*)obs, (c128*)snap, save_every,
                 (hipStream_t)stream, nullptr, 0, nullptr, 1);
}

extern "C" int qd_glf_rk4(const qd_c128* P, const qd_c128* Q, const qd_c128* L, const qd_c128* R, int npairs,
                          qd_c128* rho, int B, int N, double dt, int nsteps, const qd_c128* E, int ne, qd_c128* obs,
                          qd_c128* snap, int save_every, void* stream) {
  QD_CHECK_ARG(P && Q && rho, "qd_glf_rk4: P, Q and rho must be non-null");
  int rc = check_common("qd_glf_rk4", rho, B, N, npairs, ne, E, obs, nsteps);
  if (rc) return rc;
  QD_CHECK_ARG(npairs == 0 || (L && R), "qd_glf_rk4: L/R null but npairs=%d", npairs);
  return glf_run(GLF_FROM_OPERATORS, nullptr, nullptr, (const c128*)P, (const c128*)Q, (const c128*)L,
                 (const c128*)R, npairs, (c128*)rho, B, N, dt, nsteps, (const c128*)E, ne, (c128*)obs, (c128*)snap,
                 save_every, (hipStream_t)stream);
}

extern "C" int qd_glf_rk4_herm(const qd_c128* P, const qd_c128* L, const qd_c128* W, int npairs, qd_c128* rho, int B,
                               int N, double dt, int nsteps, const qd_c128* E, int ne, qd_c128* obs, qd_c128* snap,
                               int save_every, void* stream) {
  QD_CHECK_ARG(P && rho, "qd_glf_rk4_herm: P and rho must be non-null");
  int rc = check_common("qd_glf_rk4_herm", rho, B, N, npairs, ne, E, obs, nsteps);
  if (rc) return rc;
  QD_CHECK_ARG(npairs == 0 || (L && W), "qd_glf_rk4_herm: L/W null but npairs=%d", npairs);
  QD_CHECK_ARG(N <= 128, "qd_glf_rk4_herm: N=%d > 128 (the Hermitian kernel is single-block)", N);
  // the Hermitian kernel reads X = P r + sum_c L_c r W_c from the mK / Cop / Cd slots; Q is not used
  return glf_run(GLF_FROM_OPERATORS, nullptr, nullptr, (const c128*)P, (const c128*)P, (const c128*)L,
                 (const c128*)W, npairs, (c128*)rho, B, N, dt, nsteps, (const c128*)E, ne, (c128*)obs, (c128*)snap,
                 save_every, (hipStream_t)stream, nullptr, 0, nullptr, 1);
}

namespace {
// shared driver: A[b] <- Vl A[b] Vr for b < B; mode 0/1 = V^+ . V / V . V^+, mode 2 = L . R
int sandwich_run(const c128* V, const c128* Lm, const c128* Rm, c128* A, int B, int N, int mode, hipStream_t st) {
  WsScope wss_(st);  // call-scoped scratch (qd_runtime.hip)
  const int Np = padded_dim(N);
  const size_t NN = (size_t)Np * Np;
  const bool pad = Np != N;
  void* w = nullptr;
  int rc = workspace(WS_MISC, (2 * NN + (size_t)B * NN * (pad ? 2 : 1)) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* Vl = (c128*)w;
  c128* Vr = Vl + NN;
  c128* T = Vr + NN;
  c128* Ap = pad ? T + (size_t)B * NN : A;
  const int threads = 256;
  const int pb = (int)std::min<size_t>((NN + 255) / 256, 4096);
  if (mode == 2)
    hipLaunchKernelGGL(sandwich_prep_kernel, dim3(pb), dim3(threads), 0, st, Lm, Rm, N, Np, Vl, Vr);
  else
    hipLaunchKernelGGL(transform_prep_kernel, dim3(pb), dim3(threads), 0, st, V, N, Np, mode, Vl, Vr);
  QD_HIP(hipGetLastError());
  if (pad) {
    hipLaunchKernelGGL(pad_kernel, dim3((int)std::min<size_t>((B * NN + 255) / 256, 65535)), dim3(threads), 0, st, A,
                       Ap, B, N, Np);
    QD_HIP(hipGetLastError());
  }
  if (Np == 32)
    hipLaunchKernelGGL(basis_transform_kernel<32>, dim3(B), dim3(CG_WG), 0, st, Vl, Vr, Ap, T, Np);
  else if (Np == 64)
    hipLaunchKernelGGL(basis_transform_kernel<64>, dim3(B), dim3(CG_WG), 0, st, Vl, Vr, Ap, T, Np);
  else
    hipLaunchKernelGGL(basis_transform_kernel<128>, dim3(B), dim3(CG_WG), 0, st, Vl, Vr, Ap, T, Np);
  QD_HIP(hipGetLastError());
  if (pad) {
    hipLaunchKernelGGL(unpad_kernel, dim3((int)std::min<size_t>(((size_t)B * N * N + 255) / 256, 65535)),
                       dim3(threads), 0, st, Ap, A, B, N, Np);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}
}  // namespace

extern "C" int qd_basis_transform(const qd_c128* V, qd_c128* A, int B, int N, int mode, void* stream) {
  QD_CHECK_ARG(V && A, "qd_basis_transform: null pointer");
  QD_CHECK_ARG(N >= 1 && N <= 16384 && B >= 1, "qd_basis_transform: bad sizes N=%d B=%d", N, B);
  QD_CHECK_ARG(mode == 0 || mode == 1, "qd_basis_transform: mode must be 0 or 1");
  return sandwich_run((const c128*)V, nullptr, nullptr, (c128*)A, B, N, mode, (hipStream_t)stream);
}

extern "C" int qd_sandwich(const qd_c128* Lm, const qd_c128* Rm, qd_c128* A, int B, int N, void* stream) {
  QD_CHECK_ARG(Lm && Rm && A, "qd_sandwich: null pointer");
  QD_CHECK_ARG(N >= 1 && N <= 16384 && B >= 1, "qd_sandwich: bad sizes N=%d B=%d", N, B);
  return sandwich_run(nullptr, (const c128*)Lm, (const c128*)Rm, (c128*)A, B, N, 2, (hipStream_t)stream);
}

extern "C" int qd_lindblad_driven_rk4(const qd_c128* H0, const qd_c128* Hd, int nd, const qd_c128* fvals,
                                      const qd_c128* C, int nc, qd_c128* rho, int B, int N, double dt, int nsteps,
                                      const qd_c128* E, int ne, qd_c128* obs, qd_c128* snap, int save_every,
                                      void* stream) {
  QD_CHECK_ARG(H0 && rho, "qd_lindblad_driven_rk4: H0 and rho must be non-null");
  int rc = check_common("qd_lindblad_driven_rk4", rho, B, N, nc, ne, E, obs, nsteps);
  if (rc) return rc;
  QD_CHECK_ARG(nc == 0 || C, "qd_lindblad_driven_rk4: C is null but nc=%d", nc);
  QD_CHECK_ARG(nd >= 1 && Hd && fvals, "qd_lindblad_driven_rk4: need nd >= 1 drive terms");
  return glf_run(GLF_FROM_LINDBLAD, (const c128*)H0, (const c128*)C, nullptr, nullptr, nullptr, nullptr, nc,
                 (c128*)rho, B, N, dt, nsteps, (const c128*)E, ne, (c128*)obs, (c128*)snap, save_every,
                 (hipStream_t)stream, (const c128*)Hd, nd, fvals);
}
