// tdse.hip — batched RK4 for the time-dependent Schroedinger equation dpsi/dt = -i H psi.
//
// Replaces the loop of pyqed/mol.py:1653-1666 (_quantum_dynamics, reached from
// SESolver.run mol.py:1392 and Mol.run mol.py:628) with tdse = -1j H psi
// (phys.py:1322) and phys.rk4 (phys.py:1051-1064).  Observables are
// <psi|E_m|psi> (phys.obs, phys.py:1266-1283) at t0 and after every
// `save_every` steps.
//
// Every stage is one launch: a wave per row of H (the row path), or, for batches at larger N, a split-K MFMA GEMM of
// the whole batch (the GEMM path).  Round 1's persistent one-workgroup-per-wavefunction kernel lost to the row path at
// every measured size (tools/tdse_bench.py) and was removed in round 5.
#include "qd_common.hpp"

#include <cstdlib>
#include <functional>

namespace qd {
namespace {

// Ht = H0 - sum_d f_d Hd_d, row-major (driven step block of the row-parallel path; f on the device)
__global__ void tdse_driven_h_kernel(const c128* H0, const c128* Hd, int nd, const c128* f, int N, c128* Ht) {
  const size_t NN = (size_t)N * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    c128 h = H0[e];
    for (int d = 0; d < nd; ++d) h = csub(h, cmul(f[d], Hd[d * NN + e]));
    Ht[e] = h;
  }
}

// ---- row path (any N): every stage is one launch: a wave per row r computes k_r = -i sum_j H[r][j] x_j (lanes over
// j, coalesced 1 KB row pieces, fixed-order wave reduction) and lane 0 runs the RK4 update of element r.  (A
// persistent workgroup per wavefunction leaves the chip idle and re-streams H through one CU every stage.)  Buffers per wavefunction: psi (in place), two stage
// inputs and the accumulator.  Observables: a wave per (row, E_m) forms conj(psi_r) (E_m psi)_r, then one
// block per (b, m) sums the rows in fixed order.
__device__ __forceinline__ c128 wave_row_dot(const c128* row, const c128* x, int N) {
  const int lane = threadIdx.x & 63;
  double sr = 0.0, si = 0.0;
  for (int j = lane; j < N; j += 64) {
    const c128 h = row[j], v = x[j];
    sr += h.re * v.re - h.im * v.im;
    si += h.re * v.im + h.im * v.re;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sr += __shfl_xor(sr, off, 64);
    si += __shfl_xor(si, off, 64);
  }
  return cmk(sr, si);
}

// grid (ceil(N / 4), ceil(B / NB)), 256 threads: wave w of block x handles row r = 4 x + w for the (up to
// NB) wavefunctions of group blockIdx.y.  NB = 1 is the launched form: reading each H row once for 8
// wavefunctions (NB = 8) measured 2x slower at N = 2048, B = 8 (8 dependent loads per lane per row piece,
// 1/8 of the waves in flight), since the H rows of one stage stay L2/MALL-resident across the B waves anyway.
template <int NB>
__global__ __launch_bounds__(256) void tdse_row_stage_kernel(const c128* H, c128* psi_g, c128* ws, int N, int B,
                                                             double dt, int stage) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;
  const int b0 = blockIdx.y * NB;
  const int nb = min(NB, B - b0);
  const int lane = threadIdx.x & 63;
  const c128* row = H + (size_t)r * N;
  double sr[NB], si[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) sr[q] = si[q] = 0.0;
  // stage inputs: stage 0 psi, stage 1 x0, stage 2 x1, stage 3 x0 (x0, x1, acc per wavefunction in ws)
  auto xin = [&](int b) -> const c128* {
    return stage == 0 ? psi_g + (size_t)b * N : ws + (size_t)b * 3 * N + ((stage & 1) ? 0 : N);
  };
  for (int j = lane; j < N; j += 64) {
    const c128 h = row[j];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      if (q < nb) {
        const c128 v = xin(b0 + q)[j];
        sr[q] += h.re * v.re - h.im * v.im;
        si[q] += h.re * v.im + h.im * v.re;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      sr[q] += __shfl_xor(sr[q], off, 64);
      si[q] += __shfl_xor(si[q], off, 64);
    }
  }
  if (lane != 0) return;
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (q >= nb) break;
    const size_t b = b0 + q;
    c128* psi = psi_g + b * N;
    c128* x0 = ws + b * 3 * N;
    c128* xout = stage == 3 ? psi : (stage & 1) ? x0 + N : x0;   // stage 0: x0, 1: x1, 2: x0, 3: psi
    const c128 k = cmulmi(cmk(sr[q], si[q]));
    xout[r] = cadd(psi[r], cscale(k, rk4_horner_coef(dt, stage)));   // Horner-form RK4
  }
}

// part[b][m][r] = conj(psi_r) (E_m psi)_r ; grid (ceil(N / 4), B * ne)
__global__ __launch_bounds__(256) void tdse_obs_rows_kernel(const c128* E, int ne, const c128* psi_g, int N,
                                                            c128* part) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;
  const int b = blockIdx.y / ne, m = blockIdx.y % ne;
  const c128* psi = psi_g + (size_t)b * N;
  const c128 y = wave_row_dot(E + ((size_t)m * N + r) * N, psi, N);
  if ((threadIdx.x & 63) == 0) part[((size_t)b * ne + m) * N + r] = cmul(cconj(psi[r]), y);
}

// obs[b][idx][m] = sum_r part[b][m][r] (per-thread strided partials, wave butterfly, 4-wave sum: fixed order)
__global__ __launch_bounds__(256) void tdse_obs_sum_kernel(const c128* part, int ne, int N, int nsave, int idx,
                                                           c128* obs) {
  __shared__ c128 red[4];
  const int b = blockIdx.x / ne, m = blockIdx.x % ne;
  const c128* p = part + ((size_t)b * ne + m) * N;
  double sr = 0.0, si = 0.0;
  for (int r = threadIdx.x; r < N; r += 256) {
    sr += p[r].re;
    si += p[r].im;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sr += __shfl_xor(sr, off, 64);
    si += __shfl_xor(si, off, 64);
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cmk(sr, si);
  __syncthreads();
  if (threadIdx.x == 0) obs[((size_t)b * (nsave + 1) + idx) * ne + m] = cadd(cadd(red[0], red[1]), cadd(red[2], red[3]));
}

__global__ void tdse_snap_kernel(const c128* psi, int B, int N, int nsave, int idx, c128* snap) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < (size_t)B * N; e += (size_t)gridDim.x * blockDim.x)
    snap[((e / N) * nsave + idx - 1) * N + e % N] = psi[e];
}

// ---- batches at larger N: one stage is the GEMM K^T = X^T (-iH)^T ([Bp][Np] x [Np][Np], the split-K MFMA
// engine of the 2DES grids), which reads H once per stage for the whole batch instead of once per
// wavefunction; the slab sum and the RK4 update are one elementwise kernel.  All state in padded [Bp][Np]
// buffers (padding stays zero: zero rows of X, zero columns of (-iH)^T).
__global__ void tdse_pad_h_kernel(const c128* H, int N, int Np, c128* mHTp) {
  const size_t tot = (size_t)Np * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(e / Np), r = (int)(e % Np);
    mHTp[e] = (j < N && r < N) ? cmulmi(H[(size_t)r * N + j]) : cmk(0, 0);   // (-iH)^T [j][r]
  }
}

// dir 0: pad psi [B][N] -> P [Bp][Np]; dir 1: unpad P -> psi
__global__ void tdse_pad_psi_kernel(c128* psi, int B, int N, int Bp, int Np, c128* P, int dir) {
  const size_t tot = (size_t)Bp * Np;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / Np), r = (int)(e % Np);
    const bool in = b < B && r < N;
    if (dir == 0) P[e] = in ? psi[(size_t)b * N + r] : cmk(0, 0);
    else if (in) psi[(size_t)b * N + r] = P[e];
  }
}

// k = sum_s slabs[s] (fixed order), then the (Horner-form) RK4 update of every padded element
__global__ void tdse_gemm_rk4_kernel(const c128* slabs, int S, size_t tot, c128* P, c128* x0, c128* x1, c128* acc,
                                     double dt, int stage) {
  (void)acc;   // Horner-form RK4: no accumulator
  c128* out = stage == 3 ? P : (stage & 1) ? x1 : x0;   // stage 0: x0, 1: x1, 2: x0, 3: P
  const double hc = rk4_horner_coef(dt, stage);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    c128 k = slabs[e];
    k = slab_sum(k, 1, S, [&](int q) { return slabs[(size_t)q * tot + e]; });
    out[e] = cadd(P[e], cscale(k, hc));
  }
}

// save0 / nsave_total: this launch's first save index and the run's number of saves (driven runs call it once
// per block of save_every steps, like the persistent kernel); obs row 0 (t0) only when save0 == 0.
int tdse_gemm_steps(const c128* H, c128* psi, int B, int N, double dt, int nsteps, hipStream_t st, int save_every,
                    const std::function<int(int)>& at_step);

int tdse_rows_run(const c128* H, c128* psi, int B, int N, double dt, int nsteps, int save_every, c128* snap,
                  const c128* E, int ne, c128* obs, hipStream_t st, int save0 = 0, int nsave_total = -1) {
  WsScope wss_(st);  // call-scoped scratch (qd_runtime.hip)
  const int nsave = nsave_total >= 0 ? nsave_total : (save_every > 0 ? nsteps / save_every : 0);
  void* w = nullptr;
  const size_t ws_elems = (size_t)B * 3 * N + (size_t)B * (ne ? ne : 0) * N;
  int rc = workspace(WS_MISC, ws_elems * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* ws = (c128*)w;
  c128* part = ws + (size_t)B * 3 * N;
  const dim3 rows((N + 3) / 4, B);
  auto observe = [&](int idx) -> int {
    if (ne && obs) {
      hipLaunchKernelGGL(tdse_obs_rows_kernel, dim3((N + 3) / 4, B * ne), dim3(256), 0, st, E, ne, (const c128*)psi, N,
                         part);
      QD_HIP(hipGetLastError());
      hipLaunchKernelGGL(tdse_obs_sum_kernel, dim3(B * ne), dim3(256), 0, st, (const c128*)part, ne, N, nsave, idx,
                         obs);
      QD_HIP(hipGetLastError());
    }
    return QD_OK;
  };
  QD_CHECK_ARG((size_t)B * (ne ? ne : 1) <= 65535, "qd_tdse_rk4: B * ne too large for the row path");
  if (save0 == 0 && (rc = observe(0))) return rc;
  auto save = [&](int s) -> int {  // after step s (0-based), psi [B][N] current
    if (save_every > 0 && (s + 1) % save_every == 0) {
      const int idx = save0 + (s + 1) / save_every;
      if (snap) {
        hipLaunchKernelGGL(tdse_snap_kernel, dim3((int)std::min<size_t>(((size_t)B * N + 255) / 256, 4096)), dim3(256),
                           0, st, (const c128*)psi, B, N, nsave, idx, snap);
        QD_HIP(hipGetLastError());
      }
      return observe(idx);
    }
    return QD_OK;
  };
  // batches: MFMA GEMM stages where they win (tools/tdse_bench.py, wavefunction-steps/s, rows -> GEMM:
  // N = 1024, B = 64: 230k -> 523k; N = 2048, B = 256: 31k -> 427k; N = 256, B = 64: 1.77M -> 1.08M, B = 256:
  // 2.42M -> 4.06M)
  if ((B >= 64 && N >= 512) || (B >= 128 && N >= 256)) {
    note_path("tdse_gemm");
    return tdse_gemm_steps(H, psi, B, N, dt, nsteps, st, save_every, save);
  }
  note_path("tdse_rows");
  for (int s = 0; s < nsteps; ++s) {
    for (int stage = 0; stage < 4; ++stage) {
      hipLaunchKernelGGL(tdse_row_stage_kernel<1>, rows, dim3(256), 0, st, H, psi, ws, N, B, dt, stage);
      QD_HIP(hipGetLastError());
    }
    if (save_every > 0 && (s + 1) % save_every == 0) {
      const int idx = save0 + (s + 1) / save_every;
      if (snap) {
        hipLaunchKernelGGL(tdse_snap_kernel, dim3((int)std::min<size_t>(((size_t)B * N + 255) / 256, 4096)), dim3(256),
                           0, st, (const c128*)psi, B, N, nsave, idx, snap);
        QD_HIP(hipGetLastError());
      }
      if ((rc = observe(idx))) return rc;
    }
  }
  return QD_OK;
}

int tdse_gemm_steps(const c128* H, c128* psi, int B, int N, double dt, int nsteps, hipStream_t st, int save_every,
                    const std::function<int(int)>& at_step) {
  WsScope wss_(st);  // call-scoped scratch (qd_runtime.hip)
  const int Bp = ceil_div(B, 128) * 128, Np = ceil_div(N, 128) * 128;
  const size_t NN = (size_t)Np * Np, BN = (size_t)Bp * Np;
  constexpr int MAXS = 16;
  void* w = nullptr;
  int rc = workspace(WS_TDSE_GEMM, (NN + 4 * BN + (size_t)MAXS * BN) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* mHTp = (c128*)w;
  c128* P = mHTp + NN;
  c128* x0 = P + BN;
  c128* x1 = x0 + BN;
  c128* acc = x1 + BN;
  c128* slabs = acc + BN;
  const int g1 = (int)std::min<size_t>((NN + 255) / 256, 8192), g2 = (int)std::min<size_t>((BN + 255) / 256, 8192);
  hipLaunchKernelGGL(tdse_pad_h_kernel, dim3(g1), dim3(256), 0, st, H, N, Np, mHTp);
  hipLaunchKernelGGL(tdse_pad_psi_kernel, dim3(g2), dim3(256), 0, st, psi, B, N, Bp, Np, P, 0);
  QD_HIP(hipGetLastError());
  for (int s = 0; s < nsteps; ++s) {
    for (int stage = 0; stage < 4; ++stage) {
      const c128* xin = stage == 0 ? P : ((stage & 1) ? x0 : x1);   // stage 1: x0, 2: x1, 3: x0
      int S = 1;
      if ((rc = cgemm_splitk_slabs(xin, mHTp, Bp, Np, Np, slabs, MAXS, &S, st))) return rc;
      hipLaunchKernelGGL(tdse_gemm_rk4_kernel, dim3(g2), dim3(256), 0, st, (const c128*)slabs, S, BN, P, x0, x1, acc,
                         dt, stage);
      QD_HIP(hipGetLastError());
    }
    if (save_every > 0 && (s + 1) % save_every == 0) {  // saves read psi [B][N]: unpad first
      hipLaunchKernelGGL(tdse_pad_psi_kernel, dim3(g2), dim3(256), 0, st, psi, B, N, Bp, Np, P, 1);
      QD_HIP(hipGetLastError());
      if ((rc = at_step(s))) return rc;
    }
  }
  hipLaunchKernelGGL(tdse_pad_psi_kernel, dim3(g2), dim3(256), 0, st, psi, B, N, Bp, Np, P, 1);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_tdse_rk4(const qd_c128* H, qd_c128* psi, int B, int N, double dt, int nsteps, int save_every,
                           qd_c128* snap, const qd_c128* E, int ne, qd_c128* obs, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(H && psi, "qd_tdse_rk4: null pointer");
  QD_CHECK_ARG(N >= 1 && B >= 1 && nsteps >= 0, "qd_tdse_rk4: bad sizes N=%d B=%d", N, B);
  QD_CHECK_ARG(ne >= 0 && (ne == 0 || (E && obs)), "qd_tdse_rk4: E/obs null but ne=%d", ne);
  QD_CHECK_ARG(!obs || save_every > 0 || nsteps == 0, "qd_tdse_rk4: observables need save_every > 0");
  hipStream_t st = (hipStream_t)stream;
  return tdse_rows_run((const c128*)H, (c128*)psi, B, N, dt, nsteps, save_every, (c128*)snap, (const c128*)E, ne,
                       ne ? (c128*)obs : nullptr, st);
}

extern "C" int qd_tdse_driven_rk4(const qd_c128* H0, const qd_c128* Hd, int nd, const qd_c128* fvals, qd_c128* psi,
                                  int B, int N, double dt, int nblocks, int nout, qd_c128* snap, const qd_c128* E,
                                  int ne, qd_c128* obs, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(H0 && psi && (nd == 0 || (Hd && fvals)), "qd_tdse_driven_rk4: null pointer");
  QD_CHECK_ARG(N >= 1 && B >= 1 && nblocks >= 0 && nout >= 1 && nd >= 0 && nd <= 16,
               "qd_tdse_driven_rk4: bad sizes N=%d B=%d nblocks=%d nout=%d nd=%d", N, B, nblocks, nout, nd);
  QD_CHECK_ARG(ne >= 0 && (ne == 0 || (E && obs)), "qd_tdse_driven_rk4: E/obs null but ne=%d", ne);
  hipStream_t st = (hipStream_t)stream;
  const size_t NN = (size_t)N * N, fl = (size_t)nblocks * nd;
  void* w = nullptr;
  int rc = workspace(WS_TDSE_H, (NN + fl) * sizeof(c128), &w, st);  // H(t) + drive values (WS_MISC: the row path)
  if (rc) return rc;
  c128* Ht = (c128*)w;
  c128* fdev = Ht + NN;
  if (fl) QD_TRY(upload(fdev, fvals, fl * sizeof(c128), st));
  const int blocks = (int)std::min<size_t>((NN + 255) / 256, 4096);
  if (nblocks == 0) {  // observables at t0 only
    return tdse_rows_run((const c128*)H0, (c128*)psi, B, N, dt, 0, nout, nullptr, (const c128*)E, ne,
                         ne ? (c128*)obs : nullptr, st, 0, 0);
  }
  // H constant within a block of nout steps (mol.py:1944-1951 evaluates calcH(t) once per block)
  for (int k = 0; k < nblocks; ++k) {
    hipLaunchKernelGGL(tdse_driven_h_kernel, dim3(blocks), dim3(256), 0, st, (const c128*)H0, (const c128*)Hd, nd,
                       (const c128*)fdev + (size_t)k * nd, N, Ht);
    QD_HIP(hipGetLastError());
    if ((rc = tdse_rows_run(Ht, (c128*)psi, B, N, dt, nout, nout, (c128*)snap, (const c128*)E, ne,
                            ne ? (c128*)obs : nullptr, st, k, nblocks)))
      return rc;
  }
  return QD_OK;
}
