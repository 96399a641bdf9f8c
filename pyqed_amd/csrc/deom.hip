// deom.hip — DEOM / HEOM auxiliary-density-operator (ADO) hierarchy, RK4.
//
// Replaces DEOMSolver.run's loop (pyqed/heom/deom.py:1107-1113) over rk4
// (deom.py:725-766) whose RHS is rem_cal / generate_dot_element
// (deom.py:641-673) with the time-dependent H(t), Q(t) of generate_time
// (deom.py:676-688).  Per ADO n with index vector key_n:
//   d rho_n = damp_n rho_n - i[H(t), rho_n]
//           + sum_{k: n_k>0} ( cL_nk Q_m rho_{n-e_k} + cR_nk rho_{n-e_k} Q_m )
//           + sum_{k: tier<L} cP_nk [Q_m, rho_{n+e_k}]
// with damp_n = -sum_k n_k expn_k, cL = -i sqrt(n_k)/sqrt(etaa_k) etal_k,
// cR = +i sqrt(n_k)/sqrt(etaa_k) etar_k, cP = -i sqrt(n_k+1) sqrt(etaa_k),
// m = mode[k].  The host builds the bit-exact neighbour tables minus/plus
// (hash of key -/+ e_k, -1 when absent) and the coefficient tables once.
//
// One launch per RK4 stage (the stage needs every ADO of the previous stage);
// one thread per matrix element (b, n, i, j); H(t)/Q(t) are assembled in LDS
// per workgroup from H + f_sys(t) Hdip, Q + f_coup(t) Qdip.  The fused
// epilogue does the RK4 bookkeeping (deom_rk4_next: the classic acc form for
// driven runs, the accumulator-free Horner form when the generator is constant
// over the step) and records rho_0 (the system density matrix) after every step.
#include "handoff.hpp"
#include "qd_common.hpp"

#include <cstdlib>
#include <vector>

namespace qd {
namespace {

constexpr int DEOM_MAX_NS = 16;
constexpr int DEOM_MAX_NMOD = 8;
constexpr int DEOM_TPB = 256;

struct DeomParams {
  const c128* rho;     // [B][nmax][ns][ns]   state at step start (stage 0 input)
  c128* rho_out;       // same buffer as rho (written at stage 3 only)
  const c128* xin;     // stage input (stage 0: rho)
  c128* xout;          // next-stage input
  c128* acc;           // RK4 accumulator
  const int* minus;    // [nmax][K]
  const int* plus;     // [nmax][K]
  const c128* coef;    // [nmax][K][3] : cL, cR, cP
  const c128* damp;    // [nmax]
  const int* mode;     // [K]
  const c128* H;       // [ns][ns]
  const c128* Hdip;    // [ns][ns] or null
  const c128* Q;       // [nmod][ns][ns]
  const c128* Qdip;    // [nmod][ns][ns] or null
  c128 fs, fc;         // pulse values at this stage's time
  c128* snap;          // [B][nsteps+1][ns][ns] (rho_0 after each step) or null
  int B, nmax, K, ns, nmod, stage, step, nsteps;
  double dt;
  int bminor;  // ADO-major layout [nmax][B][ns][ns] (hierarchy index fastest; group kernel only)
  int xsplit;  // group kernel: 0 = flat lane numbering; X in {1, 2, 4, 8} = hierarchies dealt to X block classes
  int ntst;    // group kernel: non-temporal rho / acc accesses (host: state beyond the Infinity Cache's share)
  int bchunk;  // group kernel, ADO-major: hierarchies of a class walked in chunks of bchunk (0 = all at once)
  int horner;  // RK4 in Horner form (no pulse: the generator is constant over the step; acc unused)
};

// RK4 stage epilogue: returns the next stage input (stage < 3) or the new rho (stage 3); `acc` is the lane's RK4
// accumulator (in: its value after the previous stage, out: after this one).
//   classic (driven runs, H(t) / Q(t) at t, t + dt/2, t + dt): deom.py:735-766's order, ddos1 = k1; += 2 k2;
//     += 2 k3; += k4; ddos += ddos1 dt / 6, each stage input rho + c k;
//   Horner (no pulse): for a generator L constant over the step RK4 is exactly the degree-4 Taylor polynomial,
//     rho' = rho + dt L(rho + dt/2 L(rho + dt/3 L(rho + dt/4 L rho))), so stage m writes rho + dt / (4 - m) L s_m
//     and needs no accumulator (glf.hip header): one state row less read and written per stage.
__device__ __forceinline__ c128 deom_rk4_next(int stage, bool horner, double dt, c128 r0, c128& acc, c128 d) {
  if (horner) {   // explicit fma: the same rounding in every kernel whatever the compiler contracts around it
    const double c = rk4_horner_coef(dt, stage);
    return cmk(__builtin_fma(d.re, c, r0.re), __builtin_fma(d.im, c, r0.im));
  }
  if (stage == 0) {
    acc = d;
    return cadd(r0, cscale(d, dt / 2));
  }
  if (stage < 3) {
    acc = cadd(acc, cscale(d, 2.0));
    return cadd(r0, cscale(d, stage == 1 ? dt / 2 : dt));
  }
  return cadd(r0, cscale(cscale(cadd(acc, d), dt), 1.0 / 6.0));
}


// One element e of a stage (any B, ns <= DEOM_MAX_NS, nmod <= DEOM_MAX_NMOD, driven or not) with H(t), Q(t) of the
// stage in sH / sQ: the generic stage kernel and the banded launch's stream-ordered fallback run this.
__device__ __forceinline__ void deom_stage_element(const DeomParams& p, size_t e, const c128* sH, const c128* sQ) {
  const int ns = p.ns, ns2 = ns * ns;
  const int j = (int)(e % ns), i = (int)((e / ns) % ns);
  const size_t bn = e / ns2;                  // b * nmax + n
  const int n = (int)(bn % p.nmax);
  const size_t bbase = (bn - n) * ns2;        // start of batch member b
  const c128* X = p.xin + bbase;
  const c128* xn = X + (size_t)n * ns2;

  // damping + coherent part: damp_n x - i (H x - x H)
  c128 d = cmul(p.damp[n], xn[i * ns + j]);
  c128 comm = cmk(0, 0);
  for (int l = 0; l < ns; ++l)
    comm = cadd(comm, csub(cmul(sH[i * ns + l], xn[l * ns + j]), cmul(xn[i * ns + l], sH[l * ns + j])));
  d = cadd(d, cmulmi(comm));

  const int* mi = p.minus + (size_t)n * p.K;
  const int* pl = p.plus + (size_t)n * p.K;
  const c128* cf = p.coef + (size_t)n * p.K * 3;
  for (int k = 0; k < p.K; ++k) {
    const c128* Qm = sQ + p.mode[k] * ns2;
    const int nm = mi[k];
    if (nm >= 0) {
      const c128* y = X + (size_t)nm * ns2;
      c128 qy = cmk(0, 0), yq = cmk(0, 0);
      for (int l = 0; l < ns; ++l) {
        qy = cadd(qy, cmul(Qm[i * ns + l], y[l * ns + j]));
        yq = cadd(yq, cmul(y[i * ns + l], Qm[l * ns + j]));
      }
      d = cadd(d, cadd(cmul(cf[3 * k + 0], qy), cmul(cf[3 * k + 1], yq)));
    }
    const int np = pl[k];
    if (np >= 0) {
      const c128* y = X + (size_t)np * ns2;
      c128 c = cmk(0, 0);
      for (int l = 0; l < ns; ++l)
        c = cadd(c, csub(cmul(Qm[i * ns + l], y[l * ns + j]), cmul(y[i * ns + l], Qm[l * ns + j])));
      d = cadd(d, cmul(cf[3 * k + 2], c));
    }
  }

  // RK4 bookkeeping (deom_rk4_next)
  const c128 r0 = p.rho ? p.rho[e] : cmk(0, 0);   // rho == nullptr: qd_deom_apply
  c128 a = (p.stage > 0 && !p.horner) ? p.acc[e] : cmk(0, 0);
  const c128 v = deom_rk4_next(p.stage, p.horner, p.dt, r0, a, d);
  if (p.stage < 3) {
    if (!p.horner) p.acc[e] = a;
    p.xout[e] = v;
  } else {
    p.rho_out[e] = v;
    if (p.snap && n == 0) {
      const size_t b = bn / p.nmax;
      p.snap[(b * (p.nsteps + 1) + p.step + 1) * ns2 + i * ns + j] = v;
    }
  }
}

__device__ __forceinline__ void deom_stage_ops(const DeomParams& p, c128* sH, c128* sQ) {
  const int ns2 = p.ns * p.ns;
  for (int e = threadIdx.x; e < ns2; e += blockDim.x)
    sH[e] = p.Hdip ? cadd(p.H[e], cmul(p.Hdip[e], p.fs)) : p.H[e];
  for (int e = threadIdx.x; e < p.nmod * ns2; e += blockDim.x)
    sQ[e] = p.Qdip ? cadd(p.Q[e], cmul(p.Qdip[e], p.fc)) : p.Q[e];
}

__global__ __launch_bounds__(DEOM_TPB) void deom_stage_kernel(DeomParams p) {
  __shared__ c128 sH[DEOM_MAX_NS * DEOM_MAX_NS];
  __shared__ c128 sQ[DEOM_MAX_NMOD * DEOM_MAX_NS * DEOM_MAX_NS];
  deom_stage_ops(p, sH, sQ);
  __syncthreads();
  const size_t tot = (size_t)p.B * p.nmax * p.ns * p.ns;
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e < tot) deom_stage_element(p, e, sH, sQ);
}

// Stream-ordered fallback of qd_deom_rk4_banded called without a status word: queued behind the banded launch, it
// returns at once unless that launch reported a hand-off timeout in *stat; then ONE workgroup restores the saved
// initial ADOs and runs the whole propagation on deom_stage_element (the stage launches' arithmetic), stage by stage
// with a device-scope fence and a workgroup barrier between stages (slow -- one CU -- but no host wait: the banded
// entry point stays asynchronous).  x0 / x1: stage buffers, acc: the classic-form accumulator (driven runs).
// The band tables' local neighbour rows (lminus / lplus: a band's own rows first, then its halo rows) are mapped back
// to global ADO rows into gminus / gplus first.
__global__ __launch_bounds__(1024) void deom_banded_fallback_kernel(DeomParams p, const int* stat, const c128* saved,
                                                                     c128* ados, c128* x0, c128* x1,
                                                                     const c128* fsv, const c128* fcv,
                                                                     const int* lminus, const int* lplus,
                                                                     const int* band_lo, const int* halo_off,
                                                                     const int* halo_idx, int nbands, int* gminus,
                                                                     int* gplus) {
  if (__hip_atomic_load(stat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  __shared__ c128 sH[DEOM_MAX_NS * DEOM_MAX_NS];
  __shared__ c128 sQ[DEOM_MAX_NMOD * DEOM_MAX_NS * DEOM_MAX_NS];
  const size_t tot = (size_t)p.nmax * p.ns * p.ns;
  for (size_t e = threadIdx.x; e < tot; e += blockDim.x) ados[e] = saved[e];
  for (int e = threadIdx.x; e < p.nmax * p.K; e += blockDim.x) {
    const int n = e / p.K;
    int lo = 0, hi = nbands;   // band b with band_lo[b] <= n < band_lo[b + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) / 2;
      if (band_lo[mid] <= n) lo = mid;
      else hi = mid;
    }
    const int own = band_lo[lo + 1] - band_lo[lo];
    auto glob = [&](int r) { return r < 0 ? -1 : r < own ? band_lo[lo] + r : halo_idx[halo_off[lo] + r - own]; };
    gminus[e] = glob(lminus[e]);
    gplus[e] = glob(lplus[e]);
  }
  __threadfence();
  __syncthreads();
  p.minus = gminus;
  p.plus = gplus;
  p.rho = ados;
  p.rho_out = ados;
  for (int s = 0; s < p.nsteps; ++s) {
    p.step = s;
    for (int stage = 0; stage < 4; ++stage) {
      p.stage = stage;
      p.xin = stage == 0 ? (const c128*)ados : ((stage - 1) & 1 ? x1 : x0);
      p.xout = stage & 1 ? x1 : x0;
      const int ti = s * 3 + (stage + 1) / 2;   // pulse values at t, t + dt/2, t + dt
      p.fs = fsv ? fsv[ti] : cmk(0, 0);
      p.fc = fcv ? fcv[ti] : cmk(0, 0);
      deom_stage_ops(p, sH, sQ);
      __syncthreads();
      for (size_t e = threadIdx.x; e < tot; e += blockDim.x) deom_stage_element(p, e, sH, sQ);
      __threadfence();   // agent-scope release / acquire: the next stage's loads see these stores, not stale L1 lines
      __syncthreads();
    }
  }
}

// Group kernel: G = next pow2 >= ns^2 lanes per ADO, one lane per matrix element, so every
// neighbour ADO is read once per group as one coalesced ns^2 x 16-B row (not once per row/column
// it touches).  The ADO's neighbour indices and prefactors are loaded ONCE per group: lane e loads
// entries e, e + G, ... of the ADO's rows (contiguous across the group) and the group broadcasts them
// (quad DPP for G = 4, lane shuffles otherwise), so a lane issues ~2K/G + 3K/G of these loads instead
// of 5K.  All of them are issued together with the lane's own element and RK4 state (round trip 1),
// then every neighbour element (round trip 2).  NS2: ns = 2 (G = 4) with every exchange of the
// 2 x 2 products a quad DPP move.  Every lane of a group follows the same branches (they share the
// ADO), so no exchange reads an inactive lane.  H(t), Q(t) go to dynamic LDS ((1 + nmod) ns^2).
typedef double deom_d2 __attribute__((ext_vector_type(2)));
// The RK4 state rho / acc is read and written once per stage by its own lane.  p.ntst: non-temporal accesses for
// those streams, so that they do not evict the stage input rows the 2K neighbour reads hit in the caches (set by
// the host for batches whose state outgrows the Infinity Cache; below that the plain accesses keep acc resident
// there from one stage to the next).
__device__ __forceinline__ c128 ld_once(const c128* q, bool nt) {
  if (nt) {
    const deom_d2 v = __builtin_nontemporal_load((const deom_d2*)q);
    return cmk(v.x, v.y);
  }
  return *q;
}
__device__ __forceinline__ void st_once(c128* q, c128 v, bool nt) {
  if (nt) __builtin_nontemporal_store(deom_d2{v.re, v.im}, (deom_d2*)q);
  else *q = v;
}

// a load through the constant address space: wave-uniform addresses become scalar loads (s_load) of tables the
// stage kernels never write
template <typename T>
__device__ __forceinline__ T ld_uniform(const T* q) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(4))) T*)q;
#else
  return *q;   // host pass of the device function only (never executed)
#endif
}

// UNI: every wave holds lanes of ONE ADO (ADO-major layout, B / xsplit a multiple of 64 / G), so the ADO's
// neighbour indices, prefactors and damping are wave-uniform scalar loads instead of per-group vector loads
// broadcast by DPP moves.
// HM: 1 = Horner-form stages fixed at compile time (no accumulator registers or code; the undriven ns = 2 launches),
// 0 = p.horner at run time.
template <int G, int KMAX, bool NS2, bool UNI = false, int HM = 0>
__device__ __forceinline__ void deom_stage_grp_body(const DeomParams& p) {
  const bool horner = HM ? true : (bool)p.horner;
  extern __shared__ c128 deom_lds[];
  c128* sH = deom_lds;
  c128* sQ = deom_lds + p.ns * p.ns;
  const int ns = NS2 ? 2 : p.ns, ns2 = ns * ns, K = p.K;
  // [B][nmax] layout: an ADO's neighbours are rows of its own hierarchy;
  // [nmax][B] layout (bminor): a wave holds one ADO of up to 64 / G hierarchies, so its index / prefactor loads
  // are one request per wave and each neighbour read is one contiguous run of 64-B rows.
  // xsplit = X > 0: block class c = blockIdx % 8 < X owns hierarchies [c B/X, (c+1) B/X) for every ADO, classes
  // >= X exit at once.  Blocks b and b + 8 share an XCD (round-robin dispatch, MI355X_MICROARCH.md "Workgroup
  // dispatch"), so one XCD reads only its own hierarchies' rows and the 2K neighbour reads of an ADO hit that
  // XCD's L2 instead of coming from the Infinity Cache eight times over.  Placement is a speed matter only.
  // 32-bit lane arithmetic (the host checks B nmax G < 2^31): one integer division per lane
  unsigned cls = 0, u;
  if (p.xsplit > 0) {
    cls = blockIdx.x & 7;
    if (cls >= (unsigned)p.xsplit) return;  // whole block exits before any barrier
    u = (blockIdx.x >> 3) * blockDim.x + threadIdx.x;
  } else {
    u = blockIdx.x * blockDim.x + threadIdx.x;
  }
  const unsigned Bx = p.xsplit > 0 ? (unsigned)(p.B / p.xsplit) : (unsigned)p.B;
  const unsigned lgrp = u / G;              // b nmax + n, or n B + b (bminor), within the class
  const int e = (int)(u % G);
  const bool live = lgrp < Bx * (unsigned)p.nmax;   // uniform within a group
  // bchunk = C > 0 (ADO-major): the class's hierarchies are walked in chunks of C, every ADO of one chunk before
  // the next chunk, so the neighbour rows the resident waves read (tiers l - 1 .. l + 1 of C hierarchies) stay
  // within the XCD's L2 instead of spanning all Bx hierarchies of the class
  unsigned lch = lgrp, boff = 0;
  if (p.bminor && p.bchunk > 0) {
    const unsigned per = (unsigned)p.bchunk * (unsigned)p.nmax;
    const unsigned ch = lgrp / per;
    lch = lgrp - ch * per;
    boff = ch * (unsigned)p.bchunk;
  }
  const unsigned q = p.bminor ? (p.bchunk > 0 ? (unsigned)p.bchunk : Bx) : (unsigned)p.nmax;
  const unsigned hi = lch / q, lo = lch - hi * q;
  const int n = live ? (int)(p.bminor ? hi : lo) : 0;
  const size_t hb = (size_t)cls * Bx + (live ? (p.bminor ? boff + lo : hi) : 0);   // hierarchy b
  const size_t grp = p.bminor ? (size_t)n * p.B + hb : hb * p.nmax + n;     // flat row of rho / acc / xout
  const bool valid = live && e < ns2;
  const size_t rs = p.bminor ? (size_t)p.B * ns2 : (size_t)ns2;         // ADO row stride
  const int ee = e < ns2 ? e : 0;           // padding lanes shadow element 0
  const c128* X = p.xin + (p.bminor ? hb * ns2 : hb * p.nmax * ns2);
  const int base = (int)(threadIdx.x & 63) & ~(G - 1);
  auto shfl = [&](c128 v, int src) { return cmk(__shfl(v.re, base + src, 64), __shfl(v.im, base + src, 64)); };
  // value of v held by lane `src` of this group (src is a compile-time constant after unrolling)
  auto bc = [&](c128 v, int src) -> c128 {
    if constexpr (G == 4) {
      switch (src) {
        case 0: return dpp_qc<0x00>(v);
        case 1: return dpp_qc<0x55>(v);
        case 2: return dpp_qc<0xAA>(v);
        default: return dpp_qc<0xFF>(v);
      }
    } else {
      return shfl(v, src);
    }
  };
  auto bci = [&](int v, int src) -> int {
    if constexpr (G == 4) {
      switch (src) {
        case 0: return dpp_qi<0x00>(v);
        case 1: return dpp_qi<0x55>(v);
        case 2: return dpp_qi<0xAA>(v);
        default: return dpp_qi<0xFF>(v);
      }
    } else {
      return __shfl(v, base + src, 64);
    }
  };

  // round trip 1: this lane's share of the indices and prefactors, own element, RK4 state, H/Q -> LDS
  constexpr int NI = UNI ? 1 : (KMAX + G - 1) / G;
  constexpr int NC = UNI ? 1 : (3 * KMAX + G - 1) / G;
  const int nu = UNI ? __builtin_amdgcn_readfirstlane(n) : n;
  int lm[NI], lp[NI];
  c128 lc[NC];
  if constexpr (!UNI) {
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int k = e + G * q;
      lm[q] = (live && k < K) ? p.minus[(size_t)n * K + k] : -1;
      lp[q] = (live && k < K) ? p.plus[(size_t)n * K + k] : -1;
    }
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = e + G * q;
      lc[q] = (live && c < 3 * K) ? p.coef[(size_t)n * K * 3 + c] : cmk(0, 0);
    }
  }
  const c128 own = live ? X[(size_t)n * rs + ee] : cmk(0, 0);
  const c128 dmp = UNI ? ld_uniform(p.damp + nu) : (live ? p.damp[n] : cmk(0, 0));
  const size_t idx = grp * ns2 + e;
  // stage 0 of the Horner form: the stage input is rho itself (own == rho[idx] for a valid lane)
  const c128 r0 = !valid ? cmk(0, 0) : (horner && p.stage == 0) ? own : p.rho ? ld_once(p.rho + idx, p.ntst) : cmk(0, 0);
  c128 a0 = (valid && p.stage > 0 && !horner) ? ld_once(p.acc + idx, p.ntst) : cmk(0, 0);
  for (int q = threadIdx.x; q < ns2; q += blockDim.x)
    sH[q] = p.Hdip ? cadd(p.H[q], cmul(p.Hdip[q], p.fs)) : p.H[q];
  for (int q = threadIdx.x; q < p.nmod * ns2; q += blockDim.x)
    sQ[q] = p.Qdip ? cadd(p.Q[q], cmul(p.Qdip[q], p.fc)) : p.Q[q];
  int im[KMAX], ip[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if constexpr (UNI) {
      im[k] = k < K ? ld_uniform(p.minus + (size_t)nu * K + k) : -1;
      ip[k] = k < K ? ld_uniform(p.plus + (size_t)nu * K + k) : -1;
    } else {
      im[k] = bci(lm[k / G], k % G);
      ip[k] = bci(lp[k / G], k % G);
    }
  }

  // round trip 2: every neighbour element this lane owns
  c128 ym[KMAX], yp[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    ym[k] = (k < K && im[k] >= 0) ? X[(size_t)im[k] * rs + ee] : cmk(0, 0);
    yp[k] = (k < K && ip[k] >= 0) ? X[(size_t)ip[k] * rs + ee] : cmk(0, 0);
  }
  __syncthreads();

  const int i = ee / ns, j = ee % ns;
  // v[l][j] and v[i][l] of this lane's group (v[i][j] held by lane i ns + j)
  auto colv = [&](c128 v, int l) -> c128 {
    if constexpr (NS2) return l == 0 ? dpp_qc<0x44>(v) : dpp_qc<0xEE>(v);   // lanes (0,1,0,1) / (2,3,2,3)
    else return shfl(v, l * ns + j);
  };
  auto rowv = [&](c128 v, int l) -> c128 {
    if constexpr (NS2) return l == 0 ? dpp_qc<0xA0>(v) : dpp_qc<0xF5>(v);   // lanes (0,0,2,2) / (1,1,3,3)
    else return shfl(v, i * ns + l);
  };
  auto for_l = [&](auto&& f) {   // l = 0 .. ns-1 (two literal calls for ns = 2)
    if constexpr (NS2) {
      f(0);
      f(1);
    } else {
      for (int l = 0; l < ns; ++l) f(l);
    }
  };

  // damping + coherent part: damp_n x - i (H x - x H)
  c128 d = cmul(dmp, own);
  c128 comm = cmk(0, 0);
  for_l([&](int l) {
    comm = cadd(comm, csub(cmul(sH[i * ns + l], colv(own, l)), cmul(rowv(own, l), sH[l * ns + j])));
  });
  d = cadd(d, cmulmi(comm));
  // Dissipaton terms regrouped by bath mode m (as the MFMA tile kernel below):
  //   sum_{k: mode m} cL y_- Q.. = Q_m SL_m + SR_m Q_m,  SL_m = sum_k (cL_k y_{n-e_k} + cP_k y_{n+e_k}),
  //   SR_m = sum_k (cR_k y_{n-e_k} - cP_k y_{n+e_k}),
  // so a lane scales its own neighbour elements per k (absent neighbours were loaded as 0) and the 2 x 2 ... ns x ns
  // products and their lane exchanges run once per run of equal modes instead of three times per k.
  c128 SL = cmk(0, 0), SR = cmk(0, 0);
  auto flush = [&](int m) {
    const c128* Qm = sQ + m * ns2;
    c128 t = cmk(0, 0);
    for_l([&](int l) { t = cadd(t, cadd(cmul(Qm[i * ns + l], colv(SL, l)), cmul(rowv(SR, l), Qm[l * ns + j]))); });
    d = cadd(d, t);
  };
  int mcur = p.mode[0];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k >= K) break;
    const int m = p.mode[k];
    if (m != mcur) {   // wave-uniform
      flush(mcur);
      SL = SR = cmk(0, 0);
      mcur = m;
    }
    c128 cL, cR, cP;
    if constexpr (UNI) {
      const c128* cf = p.coef + ((size_t)nu * K + k) * 3;
      cL = ld_uniform(cf);
      cR = ld_uniform(cf + 1);
      cP = ld_uniform(cf + 2);
    } else {
      cL = bc(lc[(3 * k) / G], (3 * k) % G);
      cR = bc(lc[(3 * k + 1) / G], (3 * k + 1) % G);
      cP = bc(lc[(3 * k + 2) / G], (3 * k + 2) % G);
    }
    const c128 py = cmul(cP, yp[k]);
    SL = cadd(SL, cadd(cmul(cL, ym[k]), py));
    SR = cadd(SR, csub(cmul(cR, ym[k]), py));
  }
  flush(mcur);
  if (!valid) return;

  const c128 v = deom_rk4_next(p.stage, horner, p.dt, r0, a0, d);
  if (p.stage < 3) {
    if (!horner) st_once(p.acc + idx, a0, p.ntst);
    p.xout[idx] = v;
  } else {
    p.rho_out[idx] = v;
    if (p.snap && n == 0) p.snap[(hb * (p.nsteps + 1) + p.step + 1) * ns2 + e] = v;
  }
}

template <int G, int KMAX, bool NS2, bool UNI = false, int HM = 0>
__global__ __launch_bounds__(DEOM_TPB) void deom_stage_grp_kernel(DeomParams p) {
  deom_stage_grp_body<G, KMAX, NS2, UNI, HM>(p);
}
// The same body held to five waves per SIMD (96 VGPRs, 12 B of spill at K = 5): the undriven ns = 2 batches of >= 64
// hierarchies whose XCD classes are not wave-uniform (64 hierarchies: 30.5 -> 29.8 us per stage; at 16 hierarchies
// it is slower, 11.2 vs 10.3: profiles/r03/deom/horner_compile_time_ab.txt)
template <int G, int KMAX, bool NS2, bool UNI, int HM>
__global__ __launch_bounds__(DEOM_TPB) __attribute__((amdgpu_waves_per_eu(5))) void deom_stage_grp_w5_kernel(DeomParams p) {
  deom_stage_grp_body<G, KMAX, NS2, UNI, HM>(p);
}

// Software-pipelined persistent form of the ns = 2 group kernel for undriven ADO-major batches (Horner stages, XCD
// classes of B / 8 hierarchies, no hierarchy chunks): a fixed grid whose waves walk the class's lane groups with a
// stride, and while one group's neighbour rows are in flight the NEXT group's neighbour indices, own element and
// stage state are loaded.  The stage kernels above spend two dependent memory round trips per wave (tables + own
// rows, then the neighbour rows the tables point at), once per wave generation; here a wave pays about one per group
// after the first.  Same per-element arithmetic in the same order as deom_stage_grp_body<4, KMAX, true, false, 1>,
// so the result is bit-identical (tests/test_deom_gpu.py); H / Q go to LDS once per workgroup.  Every gather and the
// state accesses are buffer loads / stores at 32-bit byte offsets, a dead lane's at BUF_OOB (zeros / dropped), and the
// lane-group coordinates advance by a carry step: against 64-bit global addresses with a branch around each
// conditional load and a division per group, 64 hierarchies 28.9 -> 26.0 us per stage
// (profiles/r04/deom/deom_buf_ab.txt, deom_buf2_ab.txt).
template <int KMAX>
__global__ __launch_bounds__(DEOM_TPB) void deom_stage_pipe_kernel(DeomParams p) {
  constexpr int G = 4, NI = (KMAX + G - 1) / G, NC = (3 * KMAX + G - 1) / G;
  extern __shared__ c128 deom_lds[];
  c128* sH = deom_lds;
  c128* sQ = deom_lds + 4;
  for (int q = threadIdx.x; q < 4; q += blockDim.x) sH[q] = p.H[q];
  for (int q = threadIdx.x; q < p.nmod * 4; q += blockDim.x) sQ[q] = p.Q[q];
  __syncthreads();
  const int K = p.K;
  const unsigned cls = blockIdx.x & 7;
  const unsigned Bx = (unsigned)(p.B / p.xsplit);
  const unsigned per = Bx * (unsigned)p.nmax * G;            // lanes of this class
  const unsigned stride = (gridDim.x >> 3) * blockDim.x;
  const unsigned lane = threadIdx.x & 63;
  const int e = (int)(threadIdx.x & 3);
  const int base = (int)lane & ~(G - 1);
  const int i = e >> 1, j = e & 1;
  auto bc = [&](c128 v, int src) -> c128 {
    switch (src) {
      case 0: return dpp_qc<0x00>(v);
      case 1: return dpp_qc<0x55>(v);
      case 2: return dpp_qc<0xAA>(v);
      default: return dpp_qc<0xFF>(v);
    }
  };
  auto bci = [&](int v, int src) -> int {
    switch (src) {
      case 0: return dpp_qi<0x00>(v);
      case 1: return dpp_qi<0x55>(v);
      case 2: return dpp_qi<0xAA>(v);
      default: return dpp_qi<0xFF>(v);
    }
  };
  auto colv = [&](c128 v, int l) -> c128 { return l == 0 ? dpp_qc<0x44>(v) : dpp_qc<0xEE>(v); };
  auto rowv = [&](c128 v, int l) -> c128 { return l == 0 ? dpp_qc<0xA0>(v) : dpp_qc<0xF5>(v); };
  // the part of a group's inputs that addresses nothing else: its neighbour indices and own element
  struct Head {
    int lm[NI], lp[NI];
    c128 own;
    int n;
    unsigned hb, off;   // off: byte offset of this lane's element of the ADO row (BUF_OOB for a dead lane)
    bool live;
  };
  // every gather is a buffer load at a 32-bit byte offset (the host keeps every table below 2^31 bytes and the
  // factors of the __umul24 products below 2^24); a dead load takes BUF_OOB and returns zeros, the value the plain
  // form selects (no 64-bit address arithmetic, no branch around the loads)
  const unsigned nx = (unsigned)p.nmax;
  const __amdgpu_buffer_rsrc_t rX = buf_rsrc(p.xin, (int)(nx * (unsigned)p.B * 64u));
  const __amdgpu_buffer_rsrc_t rCo = buf_rsrc(p.coef, (int)(nx * (unsigned)K * 48u));
  const __amdgpu_buffer_rsrc_t rDa = buf_rsrc(p.damp, (int)(nx * 16u));
  const __amdgpu_buffer_rsrc_t rMi = buf_rsrc(p.minus, (int)(nx * (unsigned)K * 4u));
  const __amdgpu_buffer_rsrc_t rPl = buf_rsrc(p.plus, (int)(nx * (unsigned)K * 4u));
  const unsigned rsb = (unsigned)p.B * 64u;                 // ADO row stride in bytes
  const int xbytes = (int)(nx * (unsigned)p.B * 64u);
  const __amdgpu_buffer_rsrc_t rR = buf_rsrc(p.rho, p.rho ? xbytes : 0), rXo = buf_rsrc(p.xout, xbytes);
  const __amdgpu_buffer_rsrc_t rRo = buf_rsrc(p.rho_out, xbytes);
  // lane group lgrp = u / G of the class is (ADO hi, hierarchy lo) with lgrp = hi Bx + lo; a wave's next group is
  // stride / G further on, so (hi, lo) advance by a constant carry step instead of a division per group
  auto head = [&](unsigned uu, unsigned hi, unsigned lo, Head& h) {
    h.live = uu < per;
    h.n = h.live ? (int)hi : 0;
    h.hb = cls * Bx + (h.live ? lo : 0);
    const unsigned nk = __umul24((unsigned)h.n, (unsigned)K);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int k = e + G * q;
      const bool ok = h.live && k < K;
      const int vm = ld4_buf(rMi, ok ? (nk + (unsigned)k) * 4u : BUF_OOB);
      const int vp = ld4_buf(rPl, ok ? (nk + (unsigned)k) * 4u : BUF_OOB);
      h.lm[q] = ok ? vm : -1;
      h.lp[q] = ok ? vp : -1;
    }
    h.off = h.live ? __umul24((unsigned)h.n, rsb) + h.hb * 64u + (unsigned)e * 16u : BUF_OOB;
    h.own = ld16_buf(rX, h.off);
  };
  unsigned u = (blockIdx.x >> 3) * blockDim.x + threadIdx.x;
  const unsigned sg = stride / G, sg_hi = sg / Bx, sg_lo = sg - sg_hi * Bx;
  unsigned ghi = (u / G) / Bx, glo = (u / G) - ghi * Bx;
  Head cur;
  head(u, ghi, glo, cur);
  // the modes of the K directions, once (scalar loads): the per-group mode tests are then uniform branches that wait
  // on no memory
  int modek[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) modek[k] = k < K ? ld_uniform(p.mode + k) : 0;
  while (__builtin_amdgcn_readfirstlane(u - lane) < per) {   // wave-uniform trip count (DPP needs whole quads)
    // this group's prefactors, damping and neighbour rows
    c128 lc[NC];
    const unsigned n3k = __umul24((unsigned)cur.n, 3u * (unsigned)K);
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = e + G * q;
      lc[q] = ld16_buf(rCo, (cur.live && c < 3 * K) ? (n3k + (unsigned)c) * 16u : BUF_OOB);
    }
    const c128 dmp = ld16_buf(rDa, cur.live ? (unsigned)cur.n * 16u : BUF_OOB);
    // r0: the own element at stage 0, else rho's (zero on a dead lane: its offset is out of range)
    const c128 r0 = p.stage == 0 ? cur.own : p.ntst ? ld16_buf_nt(rR, cur.off) : ld16_buf(rR, cur.off);
    c128 ym[KMAX], yp[KMAX];
    const unsigned xb = cur.hb * 64u + (unsigned)e * 16u;   // this lane's element within a row
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int im = bci(cur.lm[k / G], k % G), ip = bci(cur.lp[k / G], k % G);
      ym[k] = ld16_buf(rX, (k < K && im >= 0) ? __umul24((unsigned)im, rsb) + xb : BUF_OOB);
      yp[k] = ld16_buf(rX, (k < K && ip >= 0) ? __umul24((unsigned)ip, rsb) + xb : BUF_OOB);
    }
    // the next group's head, in flight with the rows above
    const unsigned un = u + stride;
    unsigned nlo = glo + sg_lo, nhi = ghi + sg_hi;
    if (nlo >= Bx) {
      nlo -= Bx;
      ++nhi;
    }
    Head nxt;
    head(un, nhi, nlo, nxt);
    // stencil: deom_stage_grp_body's ns = 2 arithmetic, operation for operation
    c128 d = cmul(dmp, cur.own);
    c128 comm = cmk(0, 0);
#pragma unroll
    for (int l = 0; l < 2; ++l)
      comm = cadd(comm, csub(cmul(sH[i * 2 + l], colv(cur.own, l)), cmul(rowv(cur.own, l), sH[l * 2 + j])));
    d = cadd(d, cmulmi(comm));
    c128 SL = cmk(0, 0), SR = cmk(0, 0);
    auto flush = [&](int m) {
      const c128* Qm = sQ + m * 4;
      c128 t = cmk(0, 0);
#pragma unroll
      for (int l = 0; l < 2; ++l) t = cadd(t, cadd(cmul(Qm[i * 2 + l], colv(SL, l)), cmul(rowv(SR, l), Qm[l * 2 + j])));
      d = cadd(d, t);
    };
    int mcur = modek[0];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k >= K) break;
      const int m = modek[k];
      if (m != mcur) {
        flush(mcur);
        SL = SR = cmk(0, 0);
        mcur = m;
      }
      const c128 cL = bc(lc[(3 * k) / G], (3 * k) % G);
      const c128 cR = bc(lc[(3 * k + 1) / G], (3 * k + 1) % G);
      const c128 cP = bc(lc[(3 * k + 2) / G], (3 * k + 2) % G);
      const c128 py = cmul(cP, yp[k]);
      SL = cadd(SL, cadd(cmul(cL, ym[k]), py));
      SR = cadd(SR, csub(cmul(cR, ym[k]), py));
    }
    flush(mcur);
    {   // a dead lane's store goes to an out-of-range offset (dropped)
      c128 a0 = cmk(0, 0);
      const c128 v = deom_rk4_next(p.stage, true, p.dt, r0, a0, d);
      if (p.stage < 3) {
        st16_buf(rXo, cur.off, v);
      } else {
        st16_buf(rRo, cur.off, v);
        if (p.snap && cur.live && cur.n == 0) p.snap[((size_t)cur.hb * (p.nsteps + 1) + p.step + 1) * 4 + e] = v;
      }
    }
    cur = nxt;
    u = un;
    ghi = nhi;
    glo = nlo;
  }
}

// MFMA tile kernel for 9 <= ns <= 16 (zero-padded to 16 in registers), NM <= 2 bath modes, K <= 21: one wave per
// ADO.  The stencil regrouped by mode m:
//   d rho_n = damp_n x - iH x + x iH + sum_m (Q_m SL_m + SR_m Q_m),
//   SL_m = sum_{k: mode k = m} (cL_k x_{n-e_k} + cP_k x_{n+e_k}),  SR_m = sum_k (cR_k x_{n-e_k} - cP_k x_{n+e_k}),
// i.e. two complex 16 x 16(1+NM) x 16 GEMMs per ADO on v_mfma_f64_16x16x4_f64:
//   D  = [-iH | Q_1 .. Q_NM] [x; SL_1 ..]   (B operand = the D-register layout of x and SL: no data movement)
//   D += [x | SR_1 ..] [iH; Q_1 ..]          (A operand = the transposed layout: one 16 x 17 LDS transpose per block)
// Every matrix is loaded once in the MFMA D layout (lane l: rows (l>>4) + 4r, column l&15; 4 x 256-B row pieces
// per load instruction); neighbour loads are branch-free (absent neighbours read the ADO's own row with a zero
// coefficient) so the compiler can issue them ahead.  The RK4 epilogue is the group kernel's.
template <int NM>
__global__ __launch_bounds__(256) void deom_stage_mfma16_kernel(DeomParams p) {
  extern __shared__ c128 deom_lds[];
  c128* sH = deom_lds;                            // [16][16] H(t), zero padded
  c128* sQ = deom_lds + 256;                      // [NM][16][16] Q_m(t)
  c128* sT = deom_lds + 256 * (1 + NM) + (threadIdx.x >> 6) * (16 * 17);   // this wave's transpose tile
  const int ns = p.ns, ns2 = ns * ns, K = p.K;
  for (int e = threadIdx.x; e < 256 * (1 + NM); e += 256) {
    const int mtx = e >> 8, i = (e >> 4) & 15, j = e & 15;
    c128 v = cmk(0, 0);
    if (i < ns && j < ns) {
      const int q = i * ns + j;
      if (mtx == 0) v = p.Hdip ? cadd(p.H[q], cmul(p.Hdip[q], p.fs)) : p.H[q];
      else v = p.Qdip ? cadd(p.Q[(mtx - 1) * ns2 + q], cmul(p.Qdip[(mtx - 1) * ns2 + q], p.fc)) : p.Q[(mtx - 1) * ns2 + q];
    }
    deom_lds[e] = v;
  }
  const long total = (long)p.B * p.nmax;
  const long g0 = blockIdx.x * 4L + (threadIdx.x >> 6);
  const bool valid = g0 < total;                  // out-of-range waves compute a copy and store nothing
  const long grp = valid ? g0 : total - 1;
  const int n = (int)(grp % p.nmax);
  const long hb = grp / p.nmax;
  const c128* X = p.xin + hb * p.nmax * ns2;
  const int lane = threadIdx.x & 63, col = lane & 15, rq = lane >> 4;
  const bool colv = col < ns;
  auto ld = [&](const c128* M, int r) -> c128 {
    const int i = rq + 4 * r;
    return (colv && i < ns) ? M[i * ns + col] : cmk(0, 0);
  };
  int myidx = -1;
  c128 mycf = cmk(0, 0);
  if (lane < 2 * K) myidx = lane < K ? p.minus[(size_t)n * K + lane] : p.plus[(size_t)n * K + lane - K];
  if (lane < 3 * K) mycf = p.coef[(size_t)n * K * 3 + lane];
  const size_t own = (size_t)grp * ns2;
  c128 x[4], r0[4], a0[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    x[r] = ld(X + (size_t)n * ns2, r);
    r0[r] = p.rho ? ld(p.rho + own, r) : cmk(0, 0);
    a0[r] = (p.stage > 0 && !p.horner) ? ld(p.acc + own, r) : cmk(0, 0);
  }
  const c128 dmp = p.damp[n];
  c128 SL[NM][4], SR[NM][4];
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) SL[m][r] = SR[m][r] = cmk(0, 0);
  auto shc = [&](c128 v, int src) { return cmk(__shfl(v.re, src, 64), __shfl(v.im, src, 64)); };
#pragma unroll 2
  for (int k = 0; k < K; ++k) {
    const int m = NM == 1 ? 0 : p.mode[k];
    const int im = __shfl(myidx, k, 64), ip = __shfl(myidx, K + k, 64);
    const c128 cL = im >= 0 ? shc(mycf, 3 * k) : cmk(0, 0);
    const c128 cR = im >= 0 ? shc(mycf, 3 * k + 1) : cmk(0, 0);
    const c128 cP = ip >= 0 ? shc(mycf, 3 * k + 2) : cmk(0, 0);
    const c128* ym = X + (size_t)(im >= 0 ? im : n) * ns2;
    const c128* yp = X + (size_t)(ip >= 0 ? ip : n) * ns2;
    c128 vm[4], vp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      vm[r] = ld(ym, r);
      vp[r] = ld(yp, r);
    }
#pragma unroll
    for (int mm = 0; mm < NM; ++mm) {
      if (mm != m) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        SL[mm][r] = cadd(SL[mm][r], cadd(cmul(cL, vm[r]), cmul(cP, vp[r])));
        SR[mm][r] = cadd(SR[mm][r], csub(cmul(cR, vm[r]), cmul(cP, vp[r])));
      }
    }
  }
  __syncthreads();  // H(t) / Q(t) in LDS
  d4 Dre = d4{0.0, 0.0, 0.0, 0.0}, Dim = d4{0.0, 0.0, 0.0, 0.0};
  auto cmfma = [&](c128 a, c128 b) {  // D += a b (complex, one 16x16x4 k-step)
    Dre = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.re, Dre, 0, 0, 0);
    Dim = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.im, Dim, 0, 0, 0);
    Dre = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.im, b.im, Dre, 0, 0, 0);
    Dim = __builtin_amdgcn_mfma_f64_16x16x4f64(a.im, b.re, Dim, 0, 0, 0);
  };
  // GEMM 1: A = [-iH | Q_m] (lane: row l&15, column 4q + (l>>4)), B = [x; SL_m] in D layout (register q)
#pragma unroll
  for (int q = 0; q < 4; ++q) cmfma(cmulmi(sH[(lane & 15) * 16 + 4 * q + rq]), x[q]);
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) cmfma(sQ[m * 256 + (lane & 15) * 16 + 4 * q + rq], SL[m][q]);
  // GEMM 2: A = [x | SR_m] transposed through LDS, B = [iH; Q_m] (lane: row 4q + (l>>4), column l&15)
  auto gemm2_block = [&](const c128* Y, const c128* Bm, bool iH) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sT[(rq + 4 * r) * 17 + col] = Y[r];
    __syncthreads();
    c128 a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = sT[(lane & 15) * 17 + 4 * q + rq];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const c128 b = Bm[(4 * q + rq) * 16 + col];
      cmfma(a[q], iH ? cmuli(b) : b);
    }
  };
  gemm2_block(x, sH, true);
#pragma unroll
  for (int m = 0; m < NM; ++m) gemm2_block(SR[m], sQ + m * 256, false);

  const double dt = p.dt;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = rq + 4 * r;
    if (!(valid && colv && i < ns)) continue;
    const c128 d = cadd(cmk(Dre[r], Dim[r]), cmul(dmp, x[r]));
    const size_t idx = own + (size_t)i * ns + col;
    c128 a = a0[r];
    const c128 v = deom_rk4_next(p.stage, p.horner, dt, r0[r], a, d);
    if (p.stage < 3) {
      if (!p.horner) p.acc[idx] = a;
      p.xout[idx] = v;
    } else {
      p.rho_out[idx] = v;
      if (p.snap && n == 0) p.snap[(hb * (p.nsteps + 1) + p.step + 1) * ns2 + (size_t)i * ns + col] = v;
    }
  }
}

__global__ void deom_snap0_kernel(const c128* rho, c128* snap, int B, int nmax, int ns, int nsteps, int bminor) {
  const int ns2 = ns * ns;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < B * ns2; e += gridDim.x * blockDim.x) {
    const int b = e / ns2, ij = e % ns2;
    snap[(size_t)b * (nsteps + 1) * ns2 + ij] = rho[(size_t)b * (bminor ? 1 : nmax) * ns2 + ij];
  }
}

// Per-call setup of the banded launch in one kernel (instead of three memsets and a copy): both hand-off buffers to
// parity 1 in every double (bytes 0x01), the status words to 0, row 0 of the snapshots from the initial ADO 0.
__global__ void deom_band_prep_kernel(unsigned long long* buf, long nwords, int* stat, int* stat2, const c128* ados,
                                      c128* snap, int ns2, c128* saved, long tot) {
  const long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x, st = (long)gridDim.x * blockDim.x;
  for (long i = i0; i < nwords; i += st) buf[i] = 0x0101010101010101ull;
  if (saved)   // the initial ADOs for the stream-ordered fallback
    for (long i = i0; i < tot; i += st) saved[i] = ados[i];
  if (i0 == 0) {
    *stat = 0;
    if (stat2) *stat2 = 0;
  }
  if (snap && i0 < ns2) snap[i0] = ados[i0];
}

// obs[b][s][m] = Tr(E_m rho_0(s)) = sum_ij E_m[j][i] rho[i][j]   (deom.py:1100,1113)
__global__ void deom_trace_kernel(const c128* snap, const c128* E, int ne, int B, int ns, int nsnap, c128* obs) {
  const int ns2 = ns * ns;
  const int tot = B * nsnap * ne;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
    const int m = e % ne, bs = e / ne;
    const c128* r = snap + (size_t)bs * ns2;
    const c128* Em = E + (size_t)m * ns2;
    c128 s = cmk(0, 0);
    for (int i = 0; i < ns; ++i)
      for (int j = 0; j < ns; ++j) s = cadd(s, cmul(Em[j * ns + i], r[i * ns + j]));
    obs[e] = s;
  }
}

// oqs._heom (pyqed/oqs.py:1808-1875): single-exponential chain, explicit in-place sweep per
// step (ADO n uses the already-updated n-1, the old n and n+1; ADO nado-1 is never updated).
// One workgroup per hierarchy, threads loop over the ns^2 matrix elements (any ns); the new ADO n is
// staged in `tmp` (ns^2 per hierarchy) and copied in behind a barrier.
__global__ __launch_bounds__(256) void heom_chain_sweep_kernel(c128* ados, int nado, int ns, const c128* H,
                                                               const c128* Q, double gamma, c128 D0, double dt,
                                                               int nsteps, c128* snap, c128* tmp_all) {
  const int ns2 = ns * ns;
  c128* A = ados + (size_t)blockIdx.x * nado * ns2;
  c128* tmp = tmp_all + (size_t)blockIdx.x * ns2;
  auto comm = [&](const c128* X, const c128* Y, int ii, int jj) {  // (X Y - Y X)[ii][jj]
    c128 s = cmk(0, 0);
    for (int l = 0; l < ns; ++l) s = cadd(s, csub(cmul(X[ii * ns + l], Y[l * ns + jj]), cmul(Y[ii * ns + l], X[l * ns + jj])));
    return s;
  };
  auto acomm = [&](const c128* X, const c128* Y, int ii, int jj) {
    c128 s = cmk(0, 0);
    for (int l = 0; l < ns; ++l) s = cadd(s, cadd(cmul(X[ii * ns + l], Y[l * ns + jj]), cmul(Y[ii * ns + l], X[l * ns + jj])));
    return s;
  };
  if (snap)
    for (int t = threadIdx.x; t < ns2; t += blockDim.x) snap[(size_t)blockIdx.x * (nsteps + 1) * ns2 + t] = A[t];
  for (int s = 0; s < nsteps; ++s) {
    for (int n = 0; n < nado - 1; ++n) {
      for (int t = threadIdx.x; t < ns2; t += blockDim.x) {
        const int i = t / ns, j = t % ns;
        const c128* xn = A + (size_t)n * ns2;
        const c128* xp = A + (size_t)(n + 1) * ns2;
        const c128 x = xn[t];
        c128 v;
        if (n == 0) {
          v = csub(csub(x, cscale(cmuli(comm(H, xn, i, j)), dt)), cscale(comm(Q, xp, i, j), dt));
        } else {
          const c128* xm = A + (size_t)(n - 1) * ns2;
          const c128 coh = cscale(cmulmi(comm(H, xn, i, j)), dt);
          c128 inner = csub(cscale(comm(Q, xp, i, j), -1.0), cscale(x, n * gamma));
          const c128 mix = cadd(cscale(comm(Q, xm, i, j), D0.re), cmuli(cscale(acomm(Q, xm, i, j), D0.im)));
          inner = cadd(inner, cscale(mix, (double)n));
          v = cadd(x, cadd(coh, cscale(inner, dt)));
        }
        tmp[t] = v;
      }
      __syncthreads();
      for (int t = threadIdx.x; t < ns2; t += blockDim.x) A[(size_t)n * ns2 + t] = tmp[t];
      __syncthreads();
    }
    if (snap)
      for (int t = threadIdx.x; t < ns2; t += blockDim.x)
        snap[((size_t)blockIdx.x * (nsteps + 1) + s + 1) * ns2 + t] = A[t];
  }
}

// ---------------------------------------------------------------- any ns, any number of modes
// Tiled stage kernel for hierarchies the register / MFMA-16 kernels do not cover (ns > 16, more than
// DEOM_MAX_NMOD coupling operators, or K beyond their tables).  Grouping the stencil by mode m,
//   d_n = damp_n x_n + [-i H(t) | Q_1 .. Q_M] [x_n ; Y_1 .. Y_M] + [x_n | Z_1 .. Z_M] [i H(t) ; Q_1 .. Q_M],
//   Y_m = sum_{k: mode k = m} cL_nk x_{n-e_k} + cP_nk x_{n+e_k},   Z_m = sum_{k: mode k = m} cR_nk x_{n-e_k} - cP_nk x_{n+e_k},
// i.e. one complex GEMM of inner dimension 2 (1 + M) ns per ADO.  One workgroup per 16 x 16 output tile of one
// ADO (256 threads, one element each); the A / B operand tiles (16 x 16) are staged in LDS chunk by chunk, the
// neighbour combinations Y_m / Z_m formed while loading (no scratch), H(t) = H + f_s Hdip, Q(t) = Q + f_c Qdip
// likewise.  Same RK4 epilogue as deom_stage_kernel.  Flat-loop form (tools/cpu_emu runs it on the host).
constexpr int DEOM_TT = 16;

__global__ __launch_bounds__(256) void deom_stage_tile_kernel(DeomParams p) {
  __shared__ c128 sA[DEOM_TT][DEOM_TT + 1];
  __shared__ c128 sB[DEOM_TT][DEOM_TT + 1];
  __shared__ c128 sacc[DEOM_TT * DEOM_TT];
  const int ns = p.ns, ns2 = ns * ns, K = p.K;
  const int nt = (ns + DEOM_TT - 1) / DEOM_TT;
  const long tile = blockIdx.x;
  const int tj = (int)(tile % nt), ti = (int)((tile / nt) % nt);
  const long bn = tile / ((long)nt * nt);
  const int n = (int)(bn % p.nmax);
  const size_t bbase = (size_t)(bn - n) * ns2;
  const c128* X = p.xin + bbase;
  const c128* xn = X + (size_t)n * ns2;
  const int* mi = p.minus + (size_t)n * K;
  const int* pl = p.plus + (size_t)n * K;
  const c128* cf = p.coef + (size_t)n * K * 3;
  const int i0 = ti * DEOM_TT, j0 = tj * DEOM_TT;
  auto hq = [&](int seg, int r, int c) {   // segment 0: H(t), segment m + 1: Q_m(t)
    if (seg == 0) return p.Hdip ? cadd(p.H[r * ns + c], cmul(p.Hdip[r * ns + c], p.fs)) : p.H[r * ns + c];
    const size_t o = (size_t)(seg - 1) * ns2 + r * ns + c;
    return p.Qdip ? cadd(p.Q[o], cmul(p.Qdip[o], p.fc)) : p.Q[o];
  };
  auto mix = [&](int m, int r, int c, bool right) {   // Y_m (left) / Z_m (right) element (r, c)
    c128 v = cmk(0.0, 0.0);
    for (int k = 0; k < K; ++k) {
      if (p.mode[k] != m) continue;
      const int a = mi[k], b = pl[k];
      if (a >= 0) v = cadd(v, cmul(cf[3 * k + (right ? 1 : 0)], X[(size_t)a * ns2 + r * ns + c]));
      if (b >= 0) {
        const c128 t = cmul(cf[3 * k + 2], X[(size_t)b * ns2 + r * ns + c]);
        v = right ? csub(v, t) : cadd(v, t);
      }
    }
    return v;
  };
  for (int f = threadIdx.x; f < DEOM_TT * DEOM_TT; f += blockDim.x) sacc[f] = cmk(0.0, 0.0);
  for (int side = 0; side < 2; ++side) {
    for (int seg = 0; seg <= p.nmod; ++seg) {
      for (int l0 = 0; l0 < ns; l0 += DEOM_TT) {
        __syncthreads();
        for (int f = threadIdx.x; f < DEOM_TT * DEOM_TT; f += blockDim.x) {
          const int r = f / DEOM_TT, c = f % DEOM_TT;
          const int ia = i0 + r, la = l0 + c;     // A[ia][la]
          const int lb = l0 + r, jb = j0 + c;     // B[lb][jb]
          c128 a = cmk(0.0, 0.0), b = cmk(0.0, 0.0);
          if (side == 0) {           // [-i H | Q_m] x [x_n ; Y_m]
            if (ia < ns && la < ns) a = seg == 0 ? cmulmi(hq(0, ia, la)) : hq(seg, ia, la);
            if (lb < ns && jb < ns) b = seg == 0 ? xn[lb * ns + jb] : mix(seg - 1, lb, jb, false);
          } else {                   // [x_n | Z_m] x [i H ; Q_m]
            if (ia < ns && la < ns) a = seg == 0 ? xn[ia * ns + la] : mix(seg - 1, ia, la, true);
            if (lb < ns && jb < ns) b = seg == 0 ? cmuli(hq(0, lb, jb)) : hq(seg, lb, jb);
          }
          sA[r][c] = a;
          sB[r][c] = b;
        }
        __syncthreads();
        for (int f = threadIdx.x; f < DEOM_TT * DEOM_TT; f += blockDim.x) {
          const int r = f / DEOM_TT, c = f % DEOM_TT;
          c128 s = sacc[f];
          for (int kk = 0; kk < DEOM_TT; ++kk) s = cadd(s, cmul(sA[r][kk], sB[kk][c]));
          sacc[f] = s;
        }
      }
    }
  }
  __syncthreads();
  const double dt = p.dt;
  for (int f = threadIdx.x; f < DEOM_TT * DEOM_TT; f += blockDim.x) {
    const int i = i0 + f / DEOM_TT, j = j0 + f % DEOM_TT;
    if (i >= ns || j >= ns) continue;
    const size_t e = bbase + (size_t)n * ns2 + (size_t)i * ns + j;
    const c128 d = cadd(sacc[f], cmul(p.damp[n], xn[i * ns + j]));
    const c128 r0 = p.rho ? p.rho[e] : cmk(0, 0);   // rho == nullptr: qd_deom_apply
    c128 a = (p.stage > 0 && !p.horner) ? p.acc[e] : cmk(0, 0);
    const c128 v = deom_rk4_next(p.stage, p.horner, dt, r0, a, d);
    if (p.stage < 3) {
      if (!p.horner) p.acc[e] = a;
      p.xout[e] = v;
    } else {
      p.rho_out[e] = v;
      if (p.snap && n == 0) {
        const size_t b = bn / p.nmax;
        p.snap[(b * (p.nsteps + 1) + p.step + 1) * ns2 + i * ns + j] = v;
      }
    }
  }
}

// MFMA form of the tiled kernel (same regrouping, same epilogue) for ns >= 17: one wave per 16 x 16 output tile,
// the four waves of a workgroup on a 2 x 2 block of tiles of one ADO (their A / B strips meet in the CU's L1).  Each
// 16-wide chunk of the inner dimension is 4 v_mfma_f64_16x16x4_f64 k-steps x 4 real products; lane l holds
// A[i0 + (l & 15)][l0 + 4q + (l >> 4)] and B[l0 + 4q + (l >> 4)][j0 + (l & 15)] (the layouts of
// deom_stage_mfma16_kernel), D rows (l >> 4) + 4r, column l & 15.  Y_m / Z_m elements are formed from the
// neighbours while loading (wave-uniform k loop, scalar table loads).
__global__ __launch_bounds__(256) void deom_stage_tmfma_kernel(DeomParams p) {
  const int ns = p.ns, ns2 = ns * ns, K = p.K;
  const int nt = (ns + 15) / 16, nbk = (nt + 1) / 2;
  const long blk = blockIdx.x;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bj = (int)(blk % nbk), bi = (int)((blk / nbk) % nbk);
  const long bn = __builtin_amdgcn_readfirstlane((int)(blk / ((long)nbk * nbk)));
  const int ti = 2 * bi + (wv >> 1), tj = 2 * bj + (wv & 1);
  if (ti >= nt || tj >= nt) return;          // wave-uniform; no workgroup barrier below
  const int n = (int)(bn % p.nmax);
  const size_t bbase = (size_t)(bn - n) * ns2;
  const c128* X = p.xin + bbase;
  const c128* xn = X + (size_t)n * ns2;
  const int* mi = p.minus + (size_t)n * K;
  const int* pl = p.plus + (size_t)n * K;
  const c128* cf = p.coef + (size_t)n * K * 3;
  const int i0 = ti * 16, j0 = tj * 16;
  const int lr = lane & 15, rq = lane >> 4;
  auto hq = [&](int seg, int r, int c) -> c128 {
    if (r >= ns || c >= ns) return cmk(0.0, 0.0);
    if (seg == 0) return p.Hdip ? cadd(p.H[r * ns + c], cmul(p.Hdip[r * ns + c], p.fs)) : p.H[r * ns + c];
    const size_t o = (size_t)(seg - 1) * ns2 + r * ns + c;
    return p.Qdip ? cadd(p.Q[o], cmul(p.Qdip[o], p.fc)) : p.Q[o];
  };
  auto xat = [&](int r, int c) -> c128 { return (r < ns && c < ns) ? xn[r * ns + c] : cmk(0.0, 0.0); };
  auto mix = [&](int m, int r, int c, bool right) -> c128 {
    c128 v = cmk(0.0, 0.0);
    if (r >= ns || c >= ns) return v;
    for (int k = 0; k < K; ++k) {
      if (p.mode[k] != m) continue;
      const int a = mi[k], b = pl[k];
      if (a >= 0) v = cadd(v, cmul(cf[3 * k + (right ? 1 : 0)], X[(size_t)a * ns2 + r * ns + c]));
      if (b >= 0) {
        const c128 t = cmul(cf[3 * k + 2], X[(size_t)b * ns2 + r * ns + c]);
        v = right ? csub(v, t) : cadd(v, t);
      }
    }
    return v;
  };
  d4 Dre = d4{0.0, 0.0, 0.0, 0.0}, Dim = d4{0.0, 0.0, 0.0, 0.0};
  auto cmfma = [&](c128 a, c128 b) {
    Dre = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.re, Dre, 0, 0, 0);
    Dim = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.im, Dim, 0, 0, 0);
    Dre = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.im, b.im, Dre, 0, 0, 0);
    Dim = __builtin_amdgcn_mfma_f64_16x16x4f64(a.im, b.re, Dim, 0, 0, 0);
  };
  for (int seg = 0; seg <= p.nmod; ++seg) {
    for (int l0 = 0; l0 < ns; l0 += 16) {
      c128 a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // left: [-iH | Q_m] x [x_n ; Y_m]
        const int l = l0 + 4 * q + rq;
        a[q] = seg == 0 ? cmulmi(hq(0, i0 + lr, l)) : hq(seg, i0 + lr, l);
        b[q] = seg == 0 ? xat(l, j0 + lr) : mix(seg - 1, l, j0 + lr, false);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) cmfma(a[q], b[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // right: [x_n | Z_m] x [iH ; Q_m]
        const int l = l0 + 4 * q + rq;
        a[q] = seg == 0 ? xat(i0 + lr, l) : mix(seg - 1, i0 + lr, l, true);
        b[q] = seg == 0 ? cmuli(hq(0, l, j0 + lr)) : hq(seg, l, j0 + lr);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) cmfma(a[q], b[q]);
    }
  }
  const double dt = p.dt;
  const c128 dmp = p.damp[n];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + rq + 4 * r, j = j0 + lr;
    if (i >= ns || j >= ns) continue;
    const size_t e = bbase + (size_t)n * ns2 + (size_t)i * ns + j;
    const c128 d = cadd(cmk(Dre[r], Dim[r]), cmul(dmp, xn[i * ns + j]));
    const c128 r0 = p.rho ? p.rho[e] : cmk(0, 0);   // rho == nullptr: qd_deom_apply
    c128 a = (p.stage > 0 && !p.horner) ? p.acc[e] : cmk(0, 0);
    const c128 v = deom_rk4_next(p.stage, p.horner, dt, r0, a, d);
    if (p.stage < 3) {
      if (!p.horner) p.acc[e] = a;
      p.xout[e] = v;
    } else {
      p.rho_out[e] = v;
      if (p.snap && n == 0) {
        const size_t b = bn / p.nmax;
        p.snap[(b * (p.nsteps + 1) + p.step + 1) * ns2 + i * ns + j] = v;
      }
    }
  }
}

}  // namespace
}  // namespace qd

using namespace qd;

namespace {
// Launch one RK4 stage of the hierarchy described by p (kernel chosen from ns, K, nmod, layout).
int deom_launch_stage(const DeomParams& p, hipStream_t st) {
  const int ns = p.ns, K = p.K, nmod = p.nmod, B = p.B, nmax = p.nmax, bminor = p.bminor;
  const size_t ns2 = (size_t)ns * ns;
  const size_t tot = (size_t)B * nmax * ns2;
  // group kernel when ns^2 <= 64 lanes and K <= 8; MFMA tile kernel for 9 <= ns <= 16 (nmod <= 2, K <= 21); the
  // tiled kernels for what the element kernel's LDS tables (ns <= 16, nmod <= 8) do not hold; else the element kernel
  int G = 1;
  while (G < (int)ns2) G *= 2;
  const bool grp = G <= 64 && K <= 8;
  const bool mfma = !grp && !bminor && ns >= 9 && ns <= 16 && nmod <= 2 && K <= 21;
  QD_CHECK_ARG(!bminor || grp, "qd_deom_rk4_ado_major: needs ns^2 <= 64 and K <= 8 (group kernel)");
  QD_CHECK_ARG(!grp || (size_t)B * nmax * G < (1u << 31), "qd_deom_rk4: B nmax = %zu ADO rows exceed the 32-bit lane range", (size_t)B * nmax);
  const size_t nthreads = grp ? (size_t)B * nmax * G : tot;
  // A small hierarchy (one at L = 12, K = 5: 24.8k lanes) as 256-thread blocks would occupy ~100 of the
  // 256 CUs, each CU then issuing the loads of 4 waves; 64-thread blocks spread the same lanes over every CU.
  int tpb = (nthreads + DEOM_TPB - 1) / DEOM_TPB < 1024 ? 64 : DEOM_TPB;
  if (!grp) tpb = DEOM_TPB;
  int grid = (int)((nthreads + tpb - 1) / tpb);
  // XCD classes for the group kernel (p.xsplit, see the kernel): batches of 8k hierarchies are dealt over the
  // 8 block classes
  DeomParams q = p;
  q.xsplit = 0;
  if (grp && B >= 8 && B % 8 == 0) {
    q.xsplit = 8;
    const size_t per = (size_t)(B / 8) * nmax * G;   // lanes per class
    grid = 8 * (int)((per + tpb - 1) / tpb);
  }
  // non-temporal rho / acc from 64 MB of state per buffer (four buffers of 25 MB at 64 hierarchies of the bench
  // hierarchy stay in the 256 MB Infinity Cache: 32.7 vs 34.2 us per stage plain / non-temporal; at 256, 101 MB
  // each: 127 vs 116 us, profiles/r02/deom/nontemporal_state_ab.txt)
  q.ntst = tot * sizeof(c128) >= ((size_t)64 << 20);
  const size_t lds = (size_t)(1 + nmod) * ns2 * sizeof(c128);   // H(t), Q(t) of the group kernel
  // the software-pipelined persistent form (undriven ns = 2 ADO-major batches of >= 64 hierarchies in 8 XCD classes,
  // no hierarchy chunks).  Its buffer loads take 32-bit byte offsets: every table below 2^31 - 2^20 bytes, __umul24
  // factors below 2^24.
  const bool small_tables = (size_t)nmax * B * 64 < ((size_t)1 << 31) - ((size_t)1 << 20) && nmax < (1 << 24) &&
                            (size_t)B * 64 < ((size_t)1 << 24);
  const bool pipe_ok = grp && G == 4 && q.horner && bminor && q.xsplit == 8 && B >= 64 && K <= 6 &&
                       tpb == DEOM_TPB && small_tables;
  // hierarchy chunks of 16 in classes of more (ADO-major) for the stage kernels: 256 hierarchies = 8 classes of 32,
  // see the kernel; not for the pipelined form (256 hierarchies: 97.0 us per stage unchunked vs 102.7-103.3 for the
  // chunked stage kernel, profiles/r04/deom/deom_bchunk_pipe_ab.txt)
  q.bchunk = 0;
  if (grp && bminor && q.xsplit > 0) {
    const int Bx = B / q.xsplit;
    q.bchunk = (!pipe_ok && Bx > 16 && Bx % 16 == 0) ? 16 : 0;
  }
  // wave-uniform ADO (scalar tables): ADO-major, classes (chunks) of a multiple of 64 / G hierarchies, 64-multiple
  // blocks
  const int wb = q.bchunk > 0 ? q.bchunk : (q.xsplit > 0 ? B / q.xsplit : 0);
  const bool uni = grp && G == 4 && bminor && q.xsplit > 0 && wb % (64 / G) == 0 && tpb % 64 == 0;
  const bool tiled = !bminor && !grp && !mfma && (ns > DEOM_MAX_NS || nmod > DEOM_MAX_NMOD);
  const bool first = p.step == 0 && p.stage == 0;   // dispatch notes once per run (qd_take_path)
  auto note = [&](const char* name) {
    if (first) note_path(name);
  };
  auto launch_stage = [&]() {
    if (tiled) {
      q.xsplit = 0;
      if (ns >= 17) {   // MFMA tiles
        note("deom_tmfma");
        const int nt = (ns + 15) / 16, nbk = (nt + 1) / 2;
        hipLaunchKernelGGL(deom_stage_tmfma_kernel, dim3((unsigned)((long)B * nmax * nbk * nbk)), dim3(256), 0, st, q);
        return;
      }
      note("deom_tile");
      const int nt = (ns + DEOM_TT - 1) / DEOM_TT;
      hipLaunchKernelGGL(deom_stage_tile_kernel, dim3((unsigned)((long)B * nmax * nt * nt)), dim3(256), 0, st, q);
      return;
    }
    if (mfma) {
      note("deom_mfma16");
      const int wg = (int)(((long)B * nmax + 3) / 4);
      const size_t lds_m = (size_t)(256 * (1 + nmod) + 4 * 16 * 17) * sizeof(c128);
      if (nmod == 1) hipLaunchKernelGGL(deom_stage_mfma16_kernel<1>, dim3(wg), dim3(256), lds_m, st, q);
      else hipLaunchKernelGGL(deom_stage_mfma16_kernel<2>, dim3(wg), dim3(256), lds_m, st, q);
      return;
    }
    if (!grp) {
      note("deom_element");
      hipLaunchKernelGGL(deom_stage_kernel, dim3(grid), dim3(tpb), 0, st, q);
      return;
    }
    // the software-pipelined persistent form (pipe_ok above)
    if (pipe_ok && q.bchunk == 0) {
      auto go = [&](const void* fn, auto kern) {
        // workgroups per class: what one XCD's CUs hold at once (every wave persistent, no tail generation)
        static thread_local const void* last_fn = nullptr;   // one lookup per kernel / LDS size / device
        static thread_local size_t last_lds = 0;
        static thread_local int last_dev = -1, last_bpc = 1;
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (fn != last_fn || lds != last_lds || dev != last_dev) {
          int per_cu = 0, cus = 0;
          (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
          (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, DEOM_TPB, lds);
          last_fn = fn;
          last_lds = lds;
          last_dev = dev;
          last_bpc = std::max(1, per_cu) * std::max(1, cus / 8);
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)(8 * last_bpc)), dim3(DEOM_TPB), lds, st, q);
      };
      if (K == 5) {
        note("deom_pipe_k5");
        go((const void*)deom_stage_pipe_kernel<5>, deom_stage_pipe_kernel<5>);
      } else if (K <= 4) {
        note("deom_pipe_k4");
        go((const void*)deom_stage_pipe_kernel<4>, deom_stage_pipe_kernel<4>);
      } else {
        note("deom_pipe_k6");
        go((const void*)deom_stage_pipe_kernel<6>, deom_stage_pipe_kernel<6>);
      }
      return;
    }
    auto launch_g4 = [&](auto hmc) {
      constexpr int HM = decltype(hmc)::value;
      note(uni ? "deom_grp4_uniform" : (K == 5 && HM && B >= 64) ? "deom_grp4_w5" : "deom_grp4");
      if (uni) {
        if (K <= 4) hipLaunchKernelGGL((deom_stage_grp_kernel<4, 4, true, true, HM>), dim3(grid), dim3(tpb), lds, st, q);
        else if (K == 5) hipLaunchKernelGGL((deom_stage_grp_kernel<4, 5, true, true, HM>), dim3(grid), dim3(tpb), lds, st, q);
        else if (K <= 6) hipLaunchKernelGGL((deom_stage_grp_kernel<4, 6, true, true, HM>), dim3(grid), dim3(tpb), lds, st, q);
        else hipLaunchKernelGGL((deom_stage_grp_kernel<4, 8, true, true, HM>), dim3(grid), dim3(tpb), lds, st, q);
      } else {
        if (K <= 4) hipLaunchKernelGGL((deom_stage_grp_kernel<4, 4, true, false, HM>), dim3(grid), dim3(tpb), lds, st, q);
        else if (K == 5 && HM && B >= 64)
          hipLaunchKernelGGL((deom_stage_grp_w5_kernel<4, 5, true, false, 1>), dim3(grid), dim3(tpb), lds, st, q);
        else if (K == 5) hipLaunchKernelGGL((deom_stage_grp_kernel<4, 5, true, false, HM>), dim3(grid), dim3(tpb), lds, st, q);
        else if (K <= 6) hipLaunchKernelGGL((deom_stage_grp_kernel<4, 6, true, false, HM>), dim3(grid), dim3(tpb), lds, st, q);
        else hipLaunchKernelGGL((deom_stage_grp_kernel<4, 8, true, false, HM>), dim3(grid), dim3(tpb), lds, st, q);
      }
    };
    if (G != 4) note("deom_grp");
    switch (G) {
      case 1: hipLaunchKernelGGL((deom_stage_grp_kernel<1, 8, false>), dim3(grid), dim3(tpb), lds, st, q); break;
      case 4:  // ns = 2; registers sized to K (ym/yp/indices scale with KMAX); K = 5 (the bench bath, Pade npsd = 4):
               // 104 instead of 116 VGPRs, same speed (profiles/r02/deom/kmax5_ab.txt); undriven runs take the
               // compile-time Horner instantiations (HM = 1)
        if (q.horner) launch_g4(std::integral_constant<int, 1>{});
        else launch_g4(std::integral_constant<int, 0>{});
        break;
      case 16: hipLaunchKernelGGL((deom_stage_grp_kernel<16, 8, false>), dim3(grid), dim3(tpb), lds, st, q); break;
      case 32: hipLaunchKernelGGL((deom_stage_grp_kernel<32, 8, false>), dim3(grid), dim3(tpb), lds, st, q); break;
      default: hipLaunchKernelGGL((deom_stage_grp_kernel<64, 8, false>), dim3(grid), dim3(tpb), lds, st, q); break;
    }
  };
  launch_stage();
  QD_HIP(hipGetLastError());
  return QD_OK;
}

int deom_run(qd_c128* ados, int B, int nmax, int K, int ns, const int32_t* minus, const int32_t* plus,
             const qd_c128* coef, const qd_c128* damp, const int32_t* mode, int nmod, const qd_c128* H,
             const qd_c128* Hdip, const qd_c128* Q, const qd_c128* Qdip, const qd_c128* fsys, const qd_c128* fcoup,
             double dt, int nsteps, qd_c128* rho_sys, const qd_c128* E, int ne, qd_c128* trace, void* stream,
             int bminor) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(ados && minus && plus && coef && damp && mode && H && Q, "qd_deom_rk4: null pointer");
  QD_CHECK_ARG(B >= 1 && nmax >= 1 && K >= 1 && nsteps >= 0, "qd_deom_rk4: bad sizes B=%d nmax=%d K=%d", B, nmax, K);
  QD_CHECK_ARG(ns >= 1 && nmod >= 1, "qd_deom_rk4: ns=%d nmod=%d", ns, nmod);
  QD_CHECK_ARG(!Hdip || fsys, "qd_deom_rk4: Hdip given without fsys");
  QD_CHECK_ARG(!Qdip || fcoup, "qd_deom_rk4: Qdip given without fcoup");
  QD_CHECK_ARG(!trace || (E && ne >= 1), "qd_deom_rk4: trace requested without observables");
  hipStream_t st = (hipStream_t)stream;
  const size_t ns2 = (size_t)ns * ns;
  const size_t tot = (size_t)B * nmax * ns2;
  const bool need_snap = rho_sys || trace;
  const size_t snap_elems = need_snap && !rho_sys ? (size_t)B * (nsteps + 1) * ns2 : 0;
  void* w = nullptr;
  int rc = workspace(WS_DEOM, (3 * tot + snap_elems) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* acc = (c128*)w;
  c128* xs[2] = {acc + tot, acc + 2 * tot};
  c128* snap = rho_sys ? (c128*)rho_sys : (need_snap ? acc + 3 * tot : nullptr);
  // fsys/fcoup are host arrays [nsteps][3] (values at t, t+dt/2, t+dt): kernel args per stage
  const qd_c128* fs_h = fsys;
  const qd_c128* fc_h = fcoup;
  if (snap) {
    hipLaunchKernelGGL(deom_snap0_kernel, dim3(std::max(1, std::min(1024, (int)((B * ns2 + 255) / 256)))), dim3(256),
                       0, st, (const c128*)ados, snap, B, nmax, ns, nsteps, bminor);
    QD_HIP(hipGetLastError());
  }
  DeomParams p;
  p.rho = (const c128*)ados;
  p.rho_out = (c128*)ados;
  p.acc = acc;
  p.minus = minus;
  p.plus = plus;
  p.coef = (const c128*)coef;
  p.damp = (const c128*)damp;
  p.mode = mode;
  p.H = (const c128*)H;
  p.Hdip = (const c128*)Hdip;
  p.Q = (const c128*)Q;
  p.Qdip = (const c128*)Qdip;
  p.snap = snap;
  p.B = B;
  p.nmax = nmax;
  p.K = K;
  p.ns = ns;
  p.nmod = nmod;
  p.nsteps = nsteps;
  p.dt = dt;
  p.bminor = bminor;
  // Horner-form RK4 unless the run is driven
  p.horner = !Hdip && !Qdip;
  static const int stage_time[4] = {0, 1, 1, 2};
  for (int s = 0; s < nsteps; ++s) {
    p.step = s;
    for (int stage = 0; stage < 4; ++stage) {
      p.stage = stage;
      p.xin = stage == 0 ? (const c128*)ados : xs[(stage - 1) & 1];
      p.xout = xs[stage & 1];
      const int ti = s * 3 + stage_time[stage];
      p.fs = fs_h ? cmk(fs_h[ti].re, fs_h[ti].im) : cmk(0, 0);
      p.fc = fc_h ? cmk(fc_h[ti].re, fc_h[ti].im) : cmk(0, 0);
      if (int rc2 = deom_launch_stage(p, st)) return rc2;
    }
  }
  if (trace) {
    const int n = B * (nsteps + 1) * ne;
    hipLaunchKernelGGL(deom_trace_kernel, dim3(std::max(1, std::min(1024, (n + 255) / 256))), dim3(256), 0, st,
                       (const c128*)snap, (const c128*)E, ne, B, ns, nsteps + 1, (c128*)trace);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}

}  // namespace

extern "C" int qd_deom_rk4(qd_c128* ados, int B, int nmax, int K, int ns, const int32_t* minus, const int32_t* plus,
                           const qd_c128* coef, const qd_c128* damp, const int32_t* mode, int nmod, const qd_c128* H,
                           const qd_c128* Hdip, const qd_c128* Q, const qd_c128* Qdip, const qd_c128* fsys,
                           const qd_c128* fcoup, double dt, int nsteps, qd_c128* rho_sys, const qd_c128* E, int ne,
                           qd_c128* trace, void* stream) {
  return deom_run(ados, B, nmax, K, ns, minus, plus, coef, damp, mode, nmod, H, Hdip, Q, Qdip, fsys, fcoup, dt, nsteps,
                  rho_sys, E, ne, trace, stream, 0);
}

extern "C" int qd_deom_rk4_ado_major(qd_c128* ados, int B, int nmax, int K, int ns, const int32_t* minus,
                                     const int32_t* plus, const qd_c128* coef, const qd_c128* damp,
                                     const int32_t* mode, int nmod, const qd_c128* H, const qd_c128* Hdip,
                                     const qd_c128* Q, const qd_c128* Qdip, const qd_c128* fsys,
                                     const qd_c128* fcoup, double dt, int nsteps, qd_c128* rho_sys, const qd_c128* E,
                                     int ne, qd_c128* trace, void* stream) {
  return deom_run(ados, B, nmax, K, ns, minus, plus, coef, damp, mode, nmod, H, Hdip, Q, Qdip, fsys, fcoup, dt, nsteps,
                  rho_sys, E, ne, trace, stream, 1);
}

// One RK4 stage over a band of ADOs (tier-banded sharding of one hierarchy): rows [0, n_own) of
// rho / xin / xout are this band's ADOs, rows [n_own, n_loc) of xin the halo copies of the neighbours other bands
// own; minus / plus [n_own][K] hold LOCAL row indices (-1 = absent).  Stage s reads xin (s = 0: rho), writes the
// owned rows of xout (s < 3) and acc, and at s = 3 the owned rows of rho; snap (band owning ADO 0 only) receives
// rho_0 after the step.  Same kernels and arithmetic as qd_deom_rk4: acc = null selects the Horner-form stages
// (what qd_deom_rk4 runs without a pulse; then stage s writes rho + dt / (4 - s) L x), a non-null acc the classic
// RK4 bookkeeping (required for driven stages).
extern "C" int qd_deom_stage(qd_c128* rho, const qd_c128* xin, qd_c128* xout, qd_c128* acc, int n_own, int K, int ns,
                             const int32_t* minus, const int32_t* plus, const qd_c128* coef, const qd_c128* damp,
                             const int32_t* mode, int nmod, const qd_c128* H, const qd_c128* Hdip, const qd_c128* Q,
                             const qd_c128* Qdip, double fs_re, double fs_im, double fc_re, double fc_im, int stage,
                             double dt, qd_c128* snap, int step, int nsteps, void* stream) {
  QD_CHECK_ARG(rho && xin && minus && plus && coef && damp && mode && H && Q, "qd_deom_stage: null pointer");
  QD_CHECK_ARG(acc || (!Hdip && !Qdip), "qd_deom_stage: a driven stage needs the RK4 accumulator acc");
  QD_CHECK_ARG(stage >= 0 && stage <= 3 && (stage == 3 || xout), "qd_deom_stage: bad stage %d / null xout", stage);
  QD_CHECK_ARG(n_own >= 1 && K >= 1, "qd_deom_stage: bad sizes n_own=%d K=%d", n_own, K);
  QD_CHECK_ARG(ns >= 1 && nmod >= 1, "qd_deom_stage: ns=%d nmod=%d", ns, nmod);
  QD_CHECK_ARG(!snap || (step >= 0 && step < nsteps), "qd_deom_stage: snapshot step %d outside [0, %d)", step, nsteps);
  DeomParams p;
  p.rho = (const c128*)rho;
  p.rho_out = (c128*)rho;
  p.xin = (const c128*)xin;
  p.xout = (c128*)xout;
  p.acc = (c128*)acc;
  p.minus = minus;
  p.plus = plus;
  p.coef = (const c128*)coef;
  p.damp = (const c128*)damp;
  p.mode = mode;
  p.H = (const c128*)H;
  p.Hdip = (const c128*)Hdip;
  p.Q = (const c128*)Q;
  p.Qdip = (const c128*)Qdip;
  p.fs = cmk(fs_re, fs_im);
  p.fc = cmk(fc_re, fc_im);
  p.snap = (c128*)snap;
  p.B = 1;
  p.nmax = n_own;
  p.K = K;
  p.ns = ns;
  p.nmod = nmod;
  p.stage = stage;
  p.step = step;
  p.nsteps = nsteps;
  p.dt = dt;
  p.bminor = 0;
  p.horner = acc == nullptr;   // no accumulator: Horner-form stages (constant generator over the step)
  return deom_launch_stage(p, (hipStream_t)stream);
}

// y = alpha P x for B ADO vectors (the generator of generate_dot_element, heom/deom.py:641-664, as an operator; the
// Krylov form of DEOMSolver.correlation_4op_3t applies it and its transpose, pyqed_amd/deom_krylov.py).  One stage
// launch of the stage kernels: Horner stage 2 (s_3 = rho + dt / 2 L s_2) with rho = 0 (a null rho: nothing is read
// for it) and dt = 2 alpha, so the coefficient is alpha exactly and the kernel reads its input only from xin.
extern "C" int qd_deom_apply(const qd_c128* x, qd_c128* y, const qd_c128* x0, int B, int nmax, int K, int ns,
                             const int32_t* minus,
                             const int32_t* plus, const qd_c128* coef, const qd_c128* damp, const int32_t* mode,
                             int nmod, const qd_c128* H, const qd_c128* Q, double alpha, int ado_major, void* stream) {
  QD_CHECK_ARG(x && y && minus && plus && coef && damp && mode && H && Q, "qd_deom_apply: null pointer");
  QD_CHECK_ARG(x != y && x0 != y, "qd_deom_apply: y must alias neither x nor x0");
  QD_CHECK_ARG(B >= 1 && nmax >= 1 && K >= 1 && ns >= 1 && nmod >= 1, "qd_deom_apply: bad sizes B=%d nmax=%d K=%d ns=%d",
               B, nmax, K, ns);
  hipStream_t st = (hipStream_t)stream;
  // the Horner stage-2 form y = rho + (dt / 2) L x with rho = x0 and dt = 2 alpha; rho == nullptr (x0 NULL): the stage
  // kernels take rho = 0 without a zeroed buffer to read; stage 2 never writes rho_out
  DeomParams p{};
  p.rho = (const c128*)x0;
  p.rho_out = nullptr;
  p.xin = (const c128*)x;
  p.xout = (c128*)y;
  p.acc = nullptr;
  p.minus = minus;
  p.plus = plus;
  p.coef = (const c128*)coef;
  p.damp = (const c128*)damp;
  p.mode = mode;
  p.H = (const c128*)H;
  p.Hdip = nullptr;
  p.Q = (const c128*)Q;
  p.Qdip = nullptr;
  p.fs = cmk(0.0, 0.0);
  p.fc = cmk(0.0, 0.0);
  p.snap = nullptr;
  p.B = B;
  p.nmax = nmax;
  p.K = K;
  p.ns = ns;
  p.nmod = nmod;
  p.stage = 2;
  p.step = 1;   // not a run's first stage: no dispatch notes from the launcher
  p.nsteps = 2;
  p.dt = 2.0 * alpha;
  p.bminor = ado_major ? 1 : 0;
  p.horner = 1;
  note_path("deom_apply");
  return deom_launch_stage(p, st);
}

namespace {
// Bounds-checked (the round-3 kernel trusted idx): a row index outside [0, nsrc) reads
// nothing, writes NaN and raises *bad, which the host entry point reports.
__global__ void gather_rows_kernel(const c128* src, int nsrc, const int32_t* idx, int n, int row, c128* dst,
                                   int* bad) {
  const size_t tot = (size_t)n * row;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int r = idx[e / row];
    if (r >= 0 && r < nsrc) {
      dst[e] = src[(size_t)r * row + e % row];
    } else {
      dst[e] = cmk(__builtin_nan(""), __builtin_nan(""));
      if (bad) *bad = 1;   // vector store (global_store): benign race, every writer stores 1
    }
  }
}
}  // namespace

// dst[i][:] = src[idx[i]][:] for i < n, rows of `row_elems` complex (packs a band's halo rows for the exchange);
// src holds nsrc rows.  check != 0: synchronise and return QD_EINVAL if an index was out of range.
extern "C" int qd_gather_rows(const qd_c128* src, int nsrc, const int32_t* idx, int n, int row_elems, qd_c128* dst,
                              int check, void* stream) {
  QD_CHECK_ARG(n >= 0 && row_elems >= 1 && nsrc >= 0, "qd_gather_rows: bad sizes n=%d row=%d nsrc=%d", n, row_elems,
               nsrc);
  if (n == 0) return QD_OK;
  QD_CHECK_ARG(src && idx && dst, "qd_gather_rows: null pointer");
  WsScope wss_((hipStream_t)stream);
  void* w = nullptr;   // the bad-index flag, only when the caller asks for the check
  if (check) {
    int rc = workspace(WS_MISC, sizeof(int), &w, (hipStream_t)stream);
    if (rc) return rc;
    QD_TRY(fill_bytes(w, 0, sizeof(int), (hipStream_t)stream));
  }
  const size_t tot = (size_t)n * row_elems;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((int)std::min<size_t>((tot + 255) / 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, (const c128*)src, nsrc, idx, n, row_elems, (c128*)dst, (int*)w);
  QD_HIP(hipGetLastError());
  if (check) {
    int h = 0;
    QD_HIP(hipMemcpyAsync(&h, w, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    QD_HIP(hipStreamSynchronize((hipStream_t)stream));
    QD_CHECK_ARG(h == 0, "qd_gather_rows: a row index outside [0, %d)", nsrc);
  }
  return QD_OK;
}

// obs[s][m] = Tr(E_m rho_0(s)) for s < nsnap (DEOMSolver.run's Tr(p1 rho_0), heom/deom.py:1100,1113)
extern "C" int qd_deom_trace(const qd_c128* snap, const qd_c128* E, int ne, int nsnap, int ns, qd_c128* obs,
                             void* stream) {
  QD_CHECK_ARG(snap && E && obs && ne >= 1 && nsnap >= 1 && ns >= 1, "qd_deom_trace: bad arguments");
  const int n = nsnap * ne;
  hipLaunchKernelGGL(deom_trace_kernel, dim3(std::max(1, std::min(1024, (n + 255) / 256))), dim3(256), 0,
                     (hipStream_t)stream, (const c128*)snap, (const c128*)E, ne, 1, ns, nsnap, (c128*)obs);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_heom_chain_euler(qd_c128* ados, int B, int nado, int ns, const qd_c128* H, const qd_c128* Q,
                                   double gamma, double D0_re, double D0_im, double dt, int nsteps, qd_c128* rho_sys,
                                   const qd_c128* E, int ne, qd_c128* obs, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(ados && H && Q, "qd_heom_chain_euler: null pointer");
  QD_CHECK_ARG(B >= 1 && nado >= 2 && nsteps >= 0, "qd_heom_chain_euler: bad sizes B=%d nado=%d", B, nado);
  QD_CHECK_ARG(ns >= 1, "qd_heom_chain_euler: ns=%d", ns);
  QD_CHECK_ARG(!obs || (E && ne >= 1), "qd_heom_chain_euler: obs requested without observables");
  hipStream_t st = (hipStream_t)stream;
  const size_t ns2 = (size_t)ns * ns;
  c128* snap = (c128*)rho_sys;
  const size_t snap_elems = (!snap && obs) ? (size_t)B * (nsteps + 1) * ns2 : 0;
  void* w = nullptr;
  int rc = workspace(WS_DEOM, (snap_elems + (size_t)B * ns2) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* tmp = (c128*)w;
  if (snap_elems) snap = tmp + (size_t)B * ns2;
  hipLaunchKernelGGL(heom_chain_sweep_kernel, dim3(B), dim3(256), 0, st, (c128*)ados, nado, ns, (const c128*)H,
                     (const c128*)Q, gamma, cmk(D0_re, D0_im), dt, nsteps, snap, tmp);
  QD_HIP(hipGetLastError());
  if (obs) {
    const int n = B * (nsteps + 1) * ne;
    hipLaunchKernelGGL(deom_trace_kernel, dim3(std::max(1, std::min(1024, (n + 255) / 256))), dim3(256), 0, st,
                       (const c128*)snap, (const c128*)E, ne, B, ns, nsteps + 1, (c128*)obs);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}

namespace {

// ---------------------------------------------------------------------------------------------------------------
// One hierarchy as ONE persistent launch over a handful of tier bands (qd_deom_rk4_banded).
//
// The unbanded path runs one launch per RK4 stage: at the bench hierarchy (6188 ADOs, 396 KB of state) a stage is
// two dependent memory round trips plus the ~1.5 us kernel boundary, 4.8 us in all.  Here workgroup w owns the
// contiguous ADO band [band_lo[w], band_lo[w+1]) of the partition deom_shard.make_plans builds (the keys are tier
// ordered, so a band's outside neighbours sit in tiers l -/+ 1 of it).  Its LDS holds the stage input of its owned
// rows followed by its halo rows (local rows: lminus / lplus), its registers hold rho and the RK4 accumulator of
// its owned elements for the whole run.  Per stage a workgroup
//   1. loads its halo rows of the previous stage's output with sc1 (L1-bypassing) 16-B loads into LDS, re-loading
//      every element whose doubles do not yet carry that stage's parity in their lowest mantissa bit (the data is
//      the flag, cdna_hip_programming.md Guideline 16 R2; s_sleep between sweeps, bounded spin);
//   2. evaluates the stencil of the group kernel (same arithmetic, same operand order) from LDS and runs the RK4
//      epilogue in registers;
//   3. writes the next stage input to its LDS rows (exact) and, write-through (sc1 stores) with its parity in every
//      double's lowest bit, to buf[g & 1]; no drain, no barrier, no epoch word.
// A halo value is thus off by at most one unit in its last place; it reaches the result only through dt x stencil
// (never a band's own state, which stays exact in registers and LDS; the last stage stores untagged): within 1e-13 of
// the stage launches, bit-identical with one band.  Against the epoch-word form (drain, barrier, flag; one wave
// polls, barrier, loads) 100-104k -> 115k steps/s at 6188 ADOs, 73.6k -> 85.2k at 18,564
// (profiles/r05/deom/band_r2_handoff_ab.txt).  Reuse of buf[g & 1] is safe: a band overwrites its rows at stage g
// after it loaded stage g - 1's rows of every source, which each stored only after loading its halo of stage g - 2
// (its halo loads complete before its stencil's barrier), and the neighbour relation is symmetric (sources ==
// consumers).  Both buffers are preset to parity 1 (stages 0 and 1, their first writers, carry 0).
// Stage 0 of step 0 reads the caller's ados (written before the launch); the last stage 3 writes the final rho
// straight into ados.  A spin that exceeds its bound (bands not co-resident)
// sets *status = 1 and every band leaves its loop (results then invalid; the host reports it).
constexpr unsigned BAND_SPIN_LIMIT = 1u << 21;  // sweeps (one round trip each): ~1 s

struct BandParams {
  const c128* ados;      // [nmax][ns2] rho at t = 0 (read at stage 0 of step 0 only)
  c128* buf;             // [2][nmax][ns2] stage outputs (hand-off buffers)
  int* status;           // [1] 0 = ok, 1 = a hand-off timed out
  const int* band_lo;    // [nbands + 1]
  const int* halo_off;   // [nbands + 1]
  const int* halo_idx;   // global ADO rows of each band's halo
  const int* src_off;    // [nbands + 1]
  const int* src;        // bands owning each band's halo rows
  const int* lminus;     // [nmax][K] local rows (owned first, then halo), -1 absent
  const int* lplus;
  const c128* coef;      // [nmax][K][3] cL, cR, cP
  const c128* damp;      // [nmax]
  const int* mode;       // [K]
  const c128* H;
  const c128* Hdip;      // or null
  const c128* Q;
  const c128* Qdip;      // or null
  const c128* fsv;       // [nsteps][3] pulse values (t, t + dt/2, t + dt) or null
  const c128* fcv;
  c128* snap;            // [nsteps + 1][ns2] rho_0 after each step, or null
  unsigned long long* tim;   // QD_PHASE_TIMING builds: [nbands][4] wall-clock ticks per phase
  int nmax, K, ns, nmod, nsteps, max_loc;
  double dt;
};

constexpr int BAND_HM = 8;   // halo elements per thread held as precomputed offsets (one batched load per stage)
#ifndef DEOM_BAND_EARLY
#define DEOM_BAND_EARLY 1   // undriven runs: the next stage's damping + coherent part computed before the poll (A/B: 0)
#endif
__device__ __forceinline__ c128 ld_sc1(const c128* q) {
  return cmk(__hip_atomic_load(&q->re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_load(&q->im, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(c128* q, c128 v) {
  __hip_atomic_store(&q->re, v.re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&q->im, v.im, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// R2 hand-off granules (cdna_hip_programming.md Guideline 16: the data is the flag): the parity of the producing
// stage in the lowest mantissa bit of both halves of a handed-off element (at most one unit in the last place; it
// reaches the result only through dt times the stencil of a neighbour, never a band's own state)
__device__ __forceinline__ c128 band_tag(c128 v, unsigned t) {
  const unsigned long long x = __builtin_bit_cast(unsigned long long, v.re);
  const unsigned long long y = __builtin_bit_cast(unsigned long long, v.im);
  return cmk(__builtin_bit_cast(double, (x & ~1ull) | t), __builtin_bit_cast(double, (y & ~1ull) | t));
}
__device__ __forceinline__ bool band_has(c128 v, unsigned t) {
  const unsigned x = (unsigned)__builtin_bit_cast(unsigned long long, v.re);
  const unsigned y = (unsigned)__builtin_bit_cast(unsigned long long, v.im);
  return (((x ^ t) | (y ^ t)) & 1u) == 0;
}
// every 256 sweeps: has another band reported a timeout?
__device__ __forceinline__ bool band_abort_seen(const int* status, unsigned spins) {
  return (spins & 255) == 0 && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// FAST (ns = 2, K == KMAX, one bath mode): the mode loop, the K bound and H / Q fold to constants and registers.
template <int G, int KMAX, bool NS2, int TPB, bool FAST>
__global__ __launch_bounds__(TPB) void deom_band_kernel(BandParams p) {
  static_assert(!FAST || NS2, "FAST is the ns = 2 specialisation");
  extern __shared__ c128 deom_lds[];
  __shared__ int sAbort[2];   // a band's timed-out sweep in stage g sets sAbort[g & 1]
  const int ns = NS2 ? 2 : p.ns, ns2 = ns * ns, K = FAST ? KMAX : p.K;
  c128* sH = deom_lds;
  c128* sQ = deom_lds + ns2;
  c128* sX = deom_lds + (size_t)(1 + p.nmod) * ns2;   // [n_own + n_halo][ns2], then one zero row (absent neighbours)
  const int w = blockIdx.x;
  const int lo = p.band_lo[w], no = p.band_lo[w + 1] - lo;
  const int hoff = p.halo_off[w], nh = p.halo_off[w + 1] - hoff;
  const int soff = p.src_off[w], nsrc = p.src_off[w + 1] - soff;
  const int tid = threadIdx.x;
  const int a = tid / G, e = tid % G;
  const bool live = a < no;                  // uniform within a group
  const bool valid = live && e < ns2;
  const int ee = e < ns2 ? e : 0;            // padding lanes shadow element 0
  const int al = live ? a : 0;
  const int n = lo + al;
  const int base = (tid & 63) & ~(G - 1);
  auto shfl = [&](c128 v, int s) { return cmk(__shfl(v.re, base + s, 64), __shfl(v.im, base + s, 64)); };
  auto bc = [&](c128 v, int s) -> c128 {
    if constexpr (G == 4) {
      switch (s) {
        case 0: return dpp_qc<0x00>(v);
        case 1: return dpp_qc<0x55>(v);
        case 2: return dpp_qc<0xAA>(v);
        default: return dpp_qc<0xFF>(v);
      }
    } else {
      return shfl(v, s);
    }
  };
  auto bci = [&](int v, int s) -> int {
    if constexpr (G == 4) {
      switch (s) {
        case 0: return dpp_qi<0x00>(v);
        case 1: return dpp_qi<0x55>(v);
        case 2: return dpp_qi<0xAA>(v);
        default: return dpp_qi<0xFF>(v);
      }
    } else {
      return __shfl(v, base + s, 64);
    }
  };

  // tables of the owned ADO, once per launch: local neighbour rows broadcast into every lane of the group, the
  // 3K prefactors kept split over the group's lanes (broadcast per stage, as the group kernel)
  constexpr int NI = (KMAX + G - 1) / G;
  constexpr int NC = (3 * KMAX + G - 1) / G;
  int lm[NI], lp[NI];
  c128 lc[NC];
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    const int k = e + G * q;
    lm[q] = (live && k < K) ? p.lminus[(size_t)n * K + k] : -1;
    lp[q] = (live && k < K) ? p.lplus[(size_t)n * K + k] : -1;
  }
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = e + G * q;
    lc[q] = (live && c < 3 * K) ? p.coef[(size_t)n * K * 3 + c] : cmk(0, 0);
  }
  const c128 dmp = live ? p.damp[n] : cmk(0, 0);
  int im[KMAX], ip[KMAX], md[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    im[k] = bci(lm[k / G], k % G);
    ip[k] = bci(lp[k / G], k % G);
    md[k] = FAST ? 0 : (k < K ? __builtin_amdgcn_readfirstlane(p.mode[k]) : -1);
  }
  // up to 512 threads (<= 2 waves per SIMD, 256 VGPRs) the prefactors are broadcast once into every lane of the
  // group instead of once per stage
  constexpr bool FULLC = TPB <= 512;
  c128 cf[FULLC ? 3 * KMAX : 1];
  if constexpr (FULLC) {
#pragma unroll
    for (int c = 0; c < 3 * KMAX; ++c) cf[c] = bc(lc[c / G], c % G);
  }
  const bool pulsed = p.Hdip || p.Qdip;
  if (!pulsed) {
    for (int q = tid; q < ns2; q += blockDim.x) sH[q] = p.H[q];
    for (int q = tid; q < p.nmod * ns2; q += blockDim.x) sQ[q] = p.Q[q];
  }
  c128 r0 = valid ? p.ados[(size_t)n * ns2 + e] : cmk(0, 0);
  c128 acc = cmk(0, 0);
  if (valid) sX[(size_t)a * ns2 + e] = r0;
  if (tid < 2) sAbort[tid] = 0;
  // LDS element index of the own and neighbour elements this lane reads every stage; absent neighbours read the
  // zero row after the band's rows (the host sizes LDS for max_loc + 1 rows; halo writes never reach it)
  const int zrow = p.max_loc;
  for (int q = tid; q < ns2; q += blockDim.x) sX[(size_t)zrow * ns2 + q] = cmk(0, 0);
  const int oown = al * ns2 + ee;
  int om[KMAX], op[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    om[k] = ((k < K && im[k] >= 0) ? im[k] : zrow) * ns2 + ee;
    op[k] = ((k < K && ip[k] >= 0) ? ip[k] : zrow) * ns2 + ee;
  }

  const int i = ee / ns, j = ee % ns;
  auto colv = [&](c128 v, int l) -> c128 {
    if constexpr (NS2) return l == 0 ? dpp_qc<0x44>(v) : dpp_qc<0xEE>(v);
    else return shfl(v, l * ns + j);
  };
  auto rowv = [&](c128 v, int l) -> c128 {
    if constexpr (NS2) return l == 0 ? dpp_qc<0xA0>(v) : dpp_qc<0xF5>(v);
    else return shfl(v, i * ns + l);
  };
  auto for_l = [&](auto&& f) {
    if constexpr (NS2) {
      f(0);
      f(1);
    } else {
      for (int l = 0; l < ns; ++l) f(l);
    }
  };
  // H(t) / Q(t) entries this lane multiplies: H[i][l], H[l][j] (FAST: the two of each; read once for the run when
  // undriven, per stage when driven)
  c128 hil[2], hlj[2], qil[2], qlj[2];
  auto read_hq = [&]() {
    if constexpr (FAST) {
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        hil[l] = sH[i * 2 + l];
        hlj[l] = sH[l * 2 + j];
        qil[l] = sQ[i * 2 + l];
        qlj[l] = sQ[l * 2 + j];
      }
    }
  };
  // damping + coherent part of the stencil, damp_n x - i[H, x], from the lane group's own elements only
  auto dlocal = [&](c128 own) -> c128 {
    c128 d = cmul(dmp, own);
    c128 comm = cmk(0, 0);
    for_l([&](int l) {
      if constexpr (FAST)
        comm = cadd(comm, csub(cmul(hil[l], colv(own, l)), cmul(rowv(own, l), hlj[l])));
      else
        comm = cadd(comm, csub(cmul(sH[i * ns + l], colv(own, l)), cmul(rowv(own, l), sH[l * ns + j])));
    });
    return cadd(d, cmulmi(comm));
  };
  // Undriven runs (H fixed): that part of stage g + 1 depends on the lane group's own rows only, so it is evaluated
  // right after stage g is published, while the source bands publish theirs (the same operations in the same
  // order: bit-identical to the stage launches)
  const bool early = DEOM_BAND_EARLY && !pulsed;
  __syncthreads();   // sH / sQ and the band's rows written above
  if (!pulsed) read_hq();
  c128 dpre = early ? dlocal(sX[oown]) : cmk(0, 0);
  static constexpr int stage_time[4] = {0, 1, 1, 2};
  const double dt = p.dt;
  const size_t slab = (size_t)p.nmax * ns2;
  const int G4 = 4 * p.nsteps;
  // this thread's halo elements q = tid + i blockDim (i < BAND_HM): byte offsets in a stage buffer, fixed for the
  // launch, so a stage issues all its halo loads back to back (one round trip); -1 = none (then element 0 is
  // loaded and dropped: branch-free).  Elements beyond BAND_HM blockDim take the generic loop below.
  const int nhe = nh * ns2;
  int hsrc[BAND_HM];
#pragma unroll
  for (int h = 0; h < BAND_HM; ++h) {
    const int q = tid + h * (int)blockDim.x;
    hsrc[h] = q < nhe ? (p.halo_idx[hoff + q / ns2] * ns2 + q % ns2) * 16 : -1;
  }
  const int slab_bytes = __builtin_amdgcn_readfirstlane((int)(slab * sizeof(c128)));
#ifdef QD_PHASE_TIMING
  unsigned long long tph[4] = {0, 0, 0, 0};
#endif

  for (int g = 0; g < G4; ++g) {
    const int step = g >> 2, stage = g & 3;
    const c128* in = g == 0 ? p.ados : p.buf + (size_t)((g - 1) & 1) * slab;
    const __amdgpu_buffer_rsrc_t rin = sc1_rsrc(in, slab_bytes);
    // the last stage's rows go straight to the caller's ados (every read of ados, stage 0's, is long done: a band
    // at stage >= 2 has loaded its sources' stage-1 rows, made after their stage-0 reads)
    const __amdgpu_buffer_rsrc_t rout =
        sc1_rsrc(g + 1 < G4 ? p.buf + (size_t)(g & 1) * slab : (c128*)p.ados, slab_bytes);
#ifdef QD_PHASE_TIMING
    const unsigned long long t0 = wall_clock64();
#endif
    // H(t), Q(t) of this stage (driven runs; every read of the previous stage's values is behind the barrier that
    // closed its stencil)
    if (pulsed) {
      const int ti = step * 3 + stage_time[stage];
      const c128 fs = p.fsv ? p.fsv[ti] : cmk(0, 0), fc = p.fcv ? p.fcv[ti] : cmk(0, 0);
      for (int q = tid; q < ns2; q += blockDim.x) sH[q] = p.Hdip ? cadd(p.H[q], cmul(p.Hdip[q], fs)) : p.H[q];
      for (int q = tid; q < p.nmod * ns2; q += blockDim.x)
        sQ[q] = p.Qdip ? cadd(p.Q[q], cmul(p.Qdip[q], fc)) : p.Q[q];
    }
#ifdef QD_PHASE_TIMING
    const unsigned long long t1 = wall_clock64();
#endif
    // 1-2. halo rows of the stage input -> LDS: sc1 loads re-issued for the granules whose lowest bits do not yet
    // hold stage g - 1's parity (the data is the flag; stage 0 of step 0 reads the caller's ados)
    {
      const unsigned tg = (unsigned)((g - 1) >> 1) & 1u;
      bool good = true;
      c128 hv[BAND_HM];
      // the first pass ~256 clocks after the publish (sooner only adds traffic; 116k -> 119k steps/s at 6188 ADOs,
      // 8 or 16 units were no better, 32 slower: profiles/r05/deom/band_first_sweep.txt)
      if (g > 0) __builtin_amdgcn_s_sleep(4);
#pragma unroll
      for (int h = 0; h < BAND_HM; ++h) hv[h] = ld16_sc1(rin, hsrc[h] < 0 ? 0 : hsrc[h]);
      if (g > 0) {
        for (unsigned spins = 0;;) {
          bool okh[BAND_HM], ok = true;
#pragma unroll
          for (int h = 0; h < BAND_HM; ++h) {
            okh[h] = hsrc[h] < 0 || band_has(hv[h], tg);
            ok &= okh[h];
          }
          if (__all(ok)) break;
          if (++spins > BAND_SPIN_LIMIT || band_abort_seen(p.status, spins)) {
            good = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          asm volatile("" ::: "memory");   // the granules change under us: re-load, never reuse the value
#pragma unroll
          for (int h = 0; h < BAND_HM; ++h)
            if (!okh[h]) hv[h] = ld16_sc1(rin, hsrc[h]);
        }
      }
#pragma unroll
      for (int h = 0; h < BAND_HM; ++h)
        if (hsrc[h] >= 0) sX[(size_t)no * ns2 + tid + h * blockDim.x] = hv[h];
      for (int q = tid + BAND_HM * (int)blockDim.x; q < nhe && good; q += blockDim.x) {
        const int r = q / ns2, c = q - r * ns2, off = (p.halo_idx[hoff + r] * ns2 + c) * 16;
        c128 v = ld16_sc1(rin, off);
        for (unsigned spins = 0; g > 0 && !band_has(v, tg);) {
          if (++spins > BAND_SPIN_LIMIT || band_abort_seen(p.status, spins)) {
            good = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          asm volatile("" ::: "memory");
          v = ld16_sc1(rin, off);
        }
        sX[(size_t)(no + r) * ns2 + c] = v;
      }
      if (!good) {
        sAbort[g & 1] = 1;
        __hip_atomic_store(p.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    if (sAbort[g & 1]) break;   // uniform: written before this barrier, rewritten (slot g & 1) only after the next
#ifdef QD_PHASE_TIMING
    const unsigned long long t2 = wall_clock64();
#endif

    // 3. stencil (group-kernel arithmetic and order) from LDS
    const c128 own = sX[oown];
    c128 ym[KMAX], yp[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      ym[k] = sX[om[k]];
      yp[k] = sX[op[k]];
    }
    if (pulsed) read_hq();
    c128 d = early ? dpre : dlocal(own);
    c128 SL = cmk(0, 0), SR = cmk(0, 0);
    auto flush = [&](int m) {
      const c128* Qm = sQ + m * ns2;
      c128 t = cmk(0, 0);
      for_l([&](int l) {
        if constexpr (FAST)
          t = cadd(t, cadd(cmul(qil[l], colv(SL, l)), cmul(rowv(SR, l), qlj[l])));
        else
          t = cadd(t, cadd(cmul(Qm[i * ns + l], colv(SL, l)), cmul(rowv(SR, l), Qm[l * ns + j])));
      });
      d = cadd(d, t);
    };
    int mcur = md[0];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k >= K) break;
      const int m = md[k];
      if (m != mcur) {
        flush(mcur);
        SL = SR = cmk(0, 0);
        mcur = m;
      }
      c128 cL, cR, cP;
      if constexpr (FULLC) {
        cL = cf[3 * k];
        cR = cf[3 * k + 1];
        cP = cf[3 * k + 2];
      } else {
        cL = bc(lc[(3 * k) / G], (3 * k) % G);
        cR = bc(lc[(3 * k + 1) / G], (3 * k + 1) % G);
        cP = bc(lc[(3 * k + 2) / G], (3 * k + 2) % G);
      }
      const c128 py = cmul(cP, yp[k]);
      SL = cadd(SL, cadd(cmul(cL, ym[k]), py));
      SR = cadd(SR, csub(cmul(cR, ym[k]), py));
    }
    flush(mcur);
    // RK4 epilogue (deom_rk4_next, as the stage kernels: Horner form unless driven)
    const c128 xo = deom_rk4_next(stage, !pulsed, dt, r0, acc, d);
    if (stage == 3) r0 = xo;
    // 4. publish: the global row write-through with stage g's parity in every double's lowest bit (the last stage's
    // rows, read by no band, carry the exact final state the host copies out) -- ahead of the barrier, which only
    // guards the band's LDS rows -- then the LDS row
    if (valid) st16_sc1(rout, (n * ns2 + e) * 16, g + 1 < G4 ? band_tag(xo, (unsigned)(g >> 1) & 1u) : xo);
    __syncthreads();   // every read of sX done
#ifdef QD_PHASE_TIMING
    const unsigned long long t3 = wall_clock64();
#endif
    if (valid) {
      sX[(size_t)a * ns2 + e] = xo;
      if (stage == 3 && p.snap && n == 0) p.snap[(size_t)(step + 1) * ns2 + e] = r0;
    }
    if (early) dpre = dlocal(xo);   // next stage's own element is xo (a padding lane's is never read)
#ifdef QD_PHASE_TIMING
    const unsigned long long t4 = wall_clock64();
    tph[0] += t1 - t0;
    tph[1] += t2 - t1;
    tph[2] += t3 - t2;
    tph[3] += t4 - t3;
#endif
  }
#ifdef QD_PHASE_TIMING
  if (tid == 0 && p.tim)
    for (int h = 0; h < 4; ++h) p.tim[w * 4 + h] = tph[h];
#endif
}

// The bands spin on each other's epochs, so all of them must be resident at once.  The launch is cooperative
// (hipLaunchCooperativeKernel checks the grid against the occupancy of the kernel and refuses an oversize one with
// hipErrorCooperativeLaunchTooLarge instead of stranding bands; +15-19 us once per run, MI355X_MICROARCH.md row
// coop-launch).  Work queued on other streams can still delay a band's start; the bounded spin then sets *status and
// the caller re-runs on the stage launches (DEOMSolver.run).  QD_OPT_COOP_LAUNCH = 0: plain launch (profiling).
template <typename Kern>
hipError_t band_launch_one(Kern kern, BandParams p, int nbands, int tpb, size_t lds, hipStream_t st) {
  if (!option(QD_OPT_COOP_LAUNCH)) {
    hipLaunchKernelGGL(kern, dim3(nbands), dim3(tpb), lds, st, p);
    return hipGetLastError();
  }
  void* args[] = {(void*)&p};
  return hipLaunchCooperativeKernel((const void*)kern, dim3(nbands), dim3(tpb), args, (unsigned)lds, st);
}

template <int G, int KMAX, bool NS2, bool FAST = false>
hipError_t launch_band(const BandParams& p, int nbands, int tpb, size_t lds, hipStream_t st) {
  if (tpb <= 256) return band_launch_one(deom_band_kernel<G, KMAX, NS2, 256, FAST>, p, nbands, tpb, lds, st);
  if (tpb <= 512) return band_launch_one(deom_band_kernel<G, KMAX, NS2, 512, FAST>, p, nbands, tpb, lds, st);
  return band_launch_one(deom_band_kernel<G, KMAX, NS2, 1024, FAST>, p, nbands, tpb, lds, st);
}

}  // namespace

// One hierarchy (B = 1) as one persistent launch over `nbands` tier bands (see the kernel above).  The band
// tables come from deom_shard.make_plans: band_lo [nbands + 1], halo_off / halo_idx (global halo rows per band),
// src_off / src (bands owning them), lminus / lplus [nmax][K] local rows; max_own / max_loc the largest band's
// owned / owned + halo row counts.  ns^2 <= 16 (ns <= 4), K <= 8, max_own ns'^2 <= 1024 lanes (ns' = 2 or 4),
// every band's rows in LDS.  status (device int, or null): 1 after the run if a hand-off timed out (the caller
// re-runs); with null the call stays asynchronous and queues a stream-ordered fallback that re-runs the propagation
// on one workgroup when (and only when) a hand-off timed out (deom_banded_fallback_kernel).
extern "C" int qd_deom_rk4_banded(qd_c128* ados, int nmax, int K, int ns, const int32_t* lminus, const int32_t* lplus,
                                  const int32_t* band_lo, const int32_t* halo_off, const int32_t* halo_idx,
                                  const int32_t* src_off, const int32_t* src, int nbands, int max_own, int max_loc,
                                  const qd_c128* coef, const qd_c128* damp, const int32_t* mode, int nmod,
                                  const qd_c128* H, const qd_c128* Hdip, const qd_c128* Q, const qd_c128* Qdip,
                                  const qd_c128* fsys, const qd_c128* fcoup, double dt, int nsteps, qd_c128* rho_sys,
                                  const qd_c128* E, int ne, qd_c128* trace, int32_t* status, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(ados && lminus && lplus && band_lo && halo_off && src_off && coef && damp && mode && H && Q,
               "qd_deom_rk4_banded: null pointer");
  QD_CHECK_ARG(nmax >= 1 && K >= 1 && K <= 8 && nsteps >= 0 && nmod >= 1,
               "qd_deom_rk4_banded: bad sizes nmax=%d K=%d nmod=%d (K <= 8)", nmax, K, nmod);
  QD_CHECK_ARG(ns >= 2 && ns <= 4, "qd_deom_rk4_banded: ns=%d outside [2, 4]", ns);
  QD_CHECK_ARG(nbands >= 1 && max_own >= 1 && max_loc >= max_own,
               "qd_deom_rk4_banded: bad band sizes nbands=%d max_own=%d max_loc=%d", nbands, max_own, max_loc);
  {  // the bands wait on each other: every band's workgroup must be resident at once (one per CU suffices)
    int dev = 0, cus = 0;
    QD_HIP(hipGetDevice(&dev));
    QD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    QD_CHECK_ARG(nbands <= cus, "qd_deom_rk4_banded: %d bands exceed the %d CUs (bands must be co-resident)", nbands,
                 cus);
  }
  QD_CHECK_ARG(!Hdip || fsys, "qd_deom_rk4_banded: Hdip given without fsys");
  QD_CHECK_ARG(!Qdip || fcoup, "qd_deom_rk4_banded: Qdip given without fcoup");
  QD_CHECK_ARG(!trace || (E && ne >= 1), "qd_deom_rk4_banded: trace requested without observables");
  const int G = ns == 2 ? 4 : 16;
  const int tpb = (max_own * G + 63) / 64 * 64;
  QD_CHECK_ARG(tpb <= 1024, "qd_deom_rk4_banded: %d owned rows x %d lanes exceed one 1024-thread workgroup",
               max_own, G);
  const size_t ns2 = (size_t)ns * ns;
  const size_t lds = ((size_t)(1 + nmod) + (size_t)max_loc + 1) * ns2 * sizeof(c128);   // + the zero row
  QD_CHECK_ARG(lds <= 160 * 1024, "qd_deom_rk4_banded: %zu B of band rows exceed the 160 KB LDS (more bands)", lds);
  hipStream_t st = (hipStream_t)stream;
  const size_t tot = (size_t)nmax * ns2;
  QD_CHECK_ARG(tot * sizeof(c128) < ((size_t)1 << 31), "qd_deom_rk4_banded: %zu ADO elements exceed 32-bit offsets",
               tot);
  const bool need_snap = rho_sys || trace;
  const size_t snap_elems = need_snap && !rho_sys ? (size_t)(nsteps + 1) * ns2 : 0;
  const size_t nf = fsys ? (size_t)nsteps * 3 : 0, nc = fcoup ? (size_t)nsteps * 3 : 0;
  const size_t flag_bytes = 16;   // the status word, 16-B padded
  // without a caller status word the call stays asynchronous: the initial ADOs are saved (and, for driven runs, an
  // accumulator kept) for a stream-ordered fallback launch that re-runs the propagation only if a hand-off timed out
  const bool guard = !status && nsteps > 0;
  const size_t gtab_elems = ((size_t)2 * nmax * K * sizeof(int32_t) + sizeof(c128) - 1) / sizeof(c128);
  const size_t fb_elems = guard ? (Hdip || Qdip ? 2 : 1) * tot + gtab_elems : 0;
  void* w = nullptr;
  int rc = workspace(WS_DEOM, (2 * tot + snap_elems + nf + nc + fb_elems) * sizeof(c128) + flag_bytes, &w, st);
  if (rc) return rc;
  c128* buf = (c128*)w;
  c128* snap = rho_sys ? (c128*)rho_sys : (need_snap ? buf + 2 * tot : nullptr);
  c128* fsv = nf ? buf + 2 * tot + snap_elems : nullptr;
  c128* fcv = nc ? buf + 2 * tot + snap_elems + nf : nullptr;
  c128* saved = guard ? buf + 2 * tot + snap_elems + nf + nc : nullptr;
  c128* fb_acc = guard && (Hdip || Qdip) ? saved + tot : nullptr;
  int* gtab = guard ? (int*)(saved + (Hdip || Qdip ? 2 : 1) * tot) : nullptr;
  int* stat_ws = (int*)(buf + 2 * tot + snap_elems + nf + nc + fb_elems);
  int* stat = status ? (int*)status : stat_ws;
  if (fsv) QD_TRY(upload(fsv, fsys, nf * sizeof(c128), st));
  if (fcv) QD_TRY(upload(fcv, fcoup, nc * sizeof(c128), st));
  // both hand-off buffers preset to parity 1 in every double (stages 0 and 1, their first writers, carry parity 0),
  // the status words zeroed, snapshot row 0 written: one kernel
  {
    const long nwords = (long)(2 * tot * sizeof(c128) / 8);
    hipLaunchKernelGGL(deom_band_prep_kernel, dim3((int)std::min<long>((nwords + 255) / 256, 1024)), dim3(256), 0, st,
                       (unsigned long long*)buf, nwords, stat_ws, status ? (int*)status : nullptr,
                       (const c128*)ados, snap, (int)ns2, saved, (long)tot);
    QD_HIP(hipGetLastError());
  }
  if (nsteps > 0) {
    BandParams p;
    p.ados = (const c128*)ados;
    p.buf = buf;
    p.status = stat;
    p.band_lo = band_lo;
    p.halo_off = halo_off;
    p.halo_idx = halo_idx;
    p.src_off = src_off;
    p.src = src;
    p.lminus = lminus;
    p.lplus = lplus;
    p.coef = (const c128*)coef;
    p.damp = (const c128*)damp;
    p.mode = mode;
    p.H = (const c128*)H;
    p.Hdip = (const c128*)Hdip;
    p.Q = (const c128*)Q;
    p.Qdip = (const c128*)Qdip;
    p.fsv = fsv;
    p.fcv = fcv;
    p.snap = snap;
    p.tim = nullptr;
#ifdef QD_PHASE_TIMING
    void* tw = nullptr;
    if (int rc2 = workspace(WS_MISC, (size_t)nbands * 4 * sizeof(unsigned long long), &tw, st)) return rc2;
    p.tim = (unsigned long long*)tw;
#endif
    p.nmax = nmax;
    p.K = K;
    p.ns = ns;
    p.nmod = nmod;
    p.nsteps = nsteps;
    p.max_loc = max_loc;
    p.dt = dt;
    hipError_t le;
    if (G == 4) {
      const bool fast = nmod == 1;
      note_path(fast && (K == 5 || K == 6) ? "deom_banded_fast" : "deom_banded");
      if (fast && K == 5) le = launch_band<4, 5, true, true>(p, nbands, tpb, lds, st);        // the bench bath
      else if (fast && K == 6) le = launch_band<4, 6, true, true>(p, nbands, tpb, lds, st);   // its stretch (npsd 5)
      else if (K <= 5) le = launch_band<4, 5, true>(p, nbands, tpb, lds, st);
      else le = launch_band<4, 8, true>(p, nbands, tpb, lds, st);
    } else {
      note_path("deom_banded_g16");
      le = launch_band<16, 8, false>(p, nbands, tpb, lds, st);
    }
    if (le == hipErrorCooperativeLaunchTooLarge) {
      (void)hipGetLastError();
      set_error("qd_deom_rk4_banded: %d bands of %d threads / %zu B LDS cannot all be co-resident "
                "(hipErrorCooperativeLaunchTooLarge); use fewer bands or the stage launches", nbands, tpb, lds);
      return QD_EBUSY;
    }
    QD_HIP(le);
    if (option(QD_OPT_FAKE_TIMEOUT))   // tests: report a hand-off timeout after the run
      QD_TRY(fill_bytes(stat, 1, 1, st));
#ifdef QD_PHASE_TIMING
    {   // per-phase wall-clock (100 MHz ticks) summed over the stages: mean and max over bands, per stage, in us
      std::vector<unsigned long long> h((size_t)nbands * 4);
      QD_HIP(hipMemcpyAsync(h.data(), p.tim, h.size() * 8, hipMemcpyDeviceToHost, st));
      QD_HIP(hipStreamSynchronize(st));
      const char* nm[4] = {"wait", "halo", "compute", "publish"};
      for (int k = 0; k < 4; ++k) {
        double sm = 0, mx = 0;
        for (int b = 0; b < nbands; ++b) {
          sm += (double)h[(size_t)b * 4 + k];
          mx = std::max(mx, (double)h[(size_t)b * 4 + k]);
        }
        fprintf(stderr, "band phase %-8s mean %.3f us max %.3f us per stage\n", nm[k], sm / nbands / 100.0 / (4.0 * nsteps),
                mx / 100.0 / (4.0 * nsteps));
      }
    }
#endif
    // the last stage 3 wrote the final rho straight into ados (deom_band_kernel)
    if (guard) {   // stream-ordered fallback: a no-op unless the banded launch reported a hand-off timeout
      DeomParams f{};
      f.acc = fb_acc;
      f.coef = (const c128*)coef;
      f.damp = (const c128*)damp;
      f.mode = mode;
      f.H = (const c128*)H;
      f.Hdip = (const c128*)Hdip;
      f.Q = (const c128*)Q;
      f.Qdip = (const c128*)Qdip;
      f.snap = snap;
      f.B = 1;
      f.nmax = nmax;
      f.K = K;
      f.ns = ns;
      f.nmod = nmod;
      f.nsteps = nsteps;
      f.dt = dt;
      f.horner = !Hdip && !Qdip;
      note_path("deom_banded_guarded");
      hipLaunchKernelGGL(deom_banded_fallback_kernel, dim3(1), dim3(1024), 0, st, f, (const int*)stat,
                         (const c128*)saved, (c128*)ados, buf, buf + tot, (const c128*)fsv, (const c128*)fcv,
                         lminus, lplus, band_lo, halo_off, halo_idx, nbands, gtab, gtab + (size_t)nmax * K);
      QD_HIP(hipGetLastError());
    }
  }
  if (trace) {
    const int n = (nsteps + 1) * ne;
    hipLaunchKernelGGL(deom_trace_kernel, dim3(std::max(1, std::min(1024, (n + 255) / 256))), dim3(256), 0, st,
                       (const c128*)snap, (const c128*)E, ne, 1, ns, nsteps + 1, (c128*)trace);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}
