// tdse.hip — batched RK4 for the time-dependent Schroedinger equation dpsi/dt = -i H psi.
//
// Replaces the loop of pyqed/mol.py:1653-1666 (_quantum_dynamics, reached from
// SESolver.run mol.py:1392 and Mol.run mol.py:628) with tdse = -1j H psi
// (phys.py:1322) and phys.rk4 (phys.py:1051-1064).  Observables are
// <psi|E_m|psi> (phys.obs, phys.py:1266-1283) at t0 and after every
// `save_every` steps.
//
// One workgroup per wavefunction, persistent over all steps: psi, the stage
// state and the RK4 accumulator live in LDS; (-iH)^T is streamed from L2/HBM
// each stage with lanes over rows (coalesced), so a stage is one GEMV.
#include "qd_common.hpp"

namespace qd {
namespace {

constexpr int TD_TPB = 256;
constexpr int TD_MAXN = 2048;

// mHT[j][r] = -i H[r][j] ; ET[m][j][r] = E_m[r][j]
__global__ void tdse_prep_kernel(const c128* H, const c128* E, int ne, int N, c128* mHT, c128* ET) {
  const size_t NN = (size_t)N * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / N), j = (int)(e % N);
    mHT[(size_t)j * N + r] = cmulmi(H[e]);
    for (int m = 0; m < ne; ++m) ET[m * NN + (size_t)j * N + r] = E[m * NN + e];
  }
}

// mHT[j][r] = -i (H0 - sum_d f_d Hd_d)[r][j]   (driven step block; f on the device)
__global__ void tdse_driven_prep_kernel(const c128* H0, const c128* Hd, int nd, const c128* f, int N, c128* mHT) {
  const size_t NN = (size_t)N * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / N), j = (int)(e % N);
    c128 h = H0[e];
    for (int d = 0; d < nd; ++d) h = csub(h, cmul(f[d], Hd[d * NN + e]));
    mHT[(size_t)j * N + r] = cmulmi(h);
  }
}

__global__ void tdse_et_kernel(const c128* E, int ne, int N, c128* ET) {
  const size_t NN = (size_t)N * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / N), j = (int)(e % N);
    for (int m = 0; m < ne; ++m) ET[m * NN + (size_t)j * N + r] = E[m * NN + e];
  }
}

__device__ void td_expect(const c128* psi, const c128* ET, int ne, int N, c128* out, c128* red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int m = 0; m < ne; ++m) {
    const c128* Em = ET + (size_t)m * N * N;
    double sr = 0, si = 0;
    for (int r = tid; r < N; r += TD_TPB) {
      c128 y = cmk(0, 0);
      for (int j = 0; j < N; ++j) y = cadd(y, cmul(Em[(size_t)j * N + r], psi[j]));
      const c128 v = cmul(cconj(psi[r]), y);
      sr += v.re;
      si += v.im;
    }
    for (int off = 32; off > 0; off >>= 1) {
      sr += __shfl_xor(sr, off, 64);
      si += __shfl_xor(si, off, 64);
    }
    if (lane == 0) red[wave] = cmk(sr, si);
    __syncthreads();
    if (tid == 0) {
      c128 s = red[0];
      for (int w = 1; w < TD_TPB / 64; ++w) s = cadd(s, red[w]);
      out[m] = s;
    }
    __syncthreads();
  }
}

// save0: index of this launch's first save in snap/obs (driven runs launch once per block of
// save_every steps); obs row 0 (t0) is written only when save0 == 0.
__global__ __launch_bounds__(TD_TPB) void tdse_rk4_kernel(const c128* mHT, c128* psi_g, int N, double dt, int nsteps,
                                                          int save_every, int nsave, int save0, c128* snap,
                                                          const c128* ET, int ne, c128* obs) {
  extern __shared__ c128 sm[];
  c128* psi = sm;          // N
  c128* xs = psi + N;      // N  stage input
  c128* acc = xs + N;      // N
  __shared__ c128 red[TD_TPB / 64];
  const int b = blockIdx.x;
  c128* pg = psi_g + (size_t)b * N;
  for (int r = threadIdx.x; r < N; r += TD_TPB) {
    psi[r] = pg[r];
    xs[r] = psi[r];
  }
  __syncthreads();
  c128* ob = obs ? obs + (size_t)b * (nsave + 1) * ne : nullptr;
  if (ob && save0 == 0) td_expect(psi, ET, ne, N, ob, red);
  const double dt2 = dt / 2.0;
  for (int s = 0; s < nsteps; ++s) {
    for (int stage = 0; stage < 4; ++stage) {
      // k = (-iH) xs ; each thread owns rows r
      constexpr int QMAX = TD_MAXN / TD_TPB;  // rows per thread; fully unrolled -> registers, not scratch
      c128 kreg[QMAX];
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        const int r = threadIdx.x + q * TD_TPB;
        c128 k = cmk(0, 0);
        if (r < N)
          for (int j = 0; j < N; ++j) k = cadd(k, cmul(mHT[(size_t)j * N + r], xs[j]));
        kreg[q] = k;
      }
      __syncthreads();  // all reads of xs done
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        const int r = threadIdx.x + q * TD_TPB;
        if (r >= N) break;
        const c128 k = kreg[q];
        if (stage == 0) {
          acc[r] = k;
          xs[r] = cadd(psi[r], cscale(k, dt2));
        } else if (stage == 1) {
          acc[r] = cadd(acc[r], cscale(k, 2.0));
          xs[r] = cadd(psi[r], cscale(k, dt2));
        } else if (stage == 2) {
          acc[r] = cadd(acc[r], cscale(k, 2.0));
          xs[r] = cadd(psi[r], cscale(k, dt));
        } else {
          const c128 a = cadd(acc[r], k);
          psi[r] = cadd(psi[r], cscale(cscale(a, 1.0 / 6.0), dt));
          xs[r] = psi[r];
        }
      }
      __syncthreads();
    }
    if (save_every > 0 && (s + 1) % save_every == 0) {
      const int idx = save0 + (s + 1) / save_every;  // 1..nsave
      if (snap)
        for (int r = threadIdx.x; r < N; r += TD_TPB) snap[((size_t)b * nsave + idx - 1) * N + r] = psi[r];
      if (ob) td_expect(psi, ET, ne, N, ob + (size_t)idx * ne, red);
    }
  }
  for (int r = threadIdx.x; r < N; r += TD_TPB) pg[r] = psi[r];
}

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_tdse_rk4(const qd_c128* H, qd_c128* psi, int B, int N, double dt, int nsteps, int save_every,
                           qd_c128* snap, const qd_c128* E, int ne, qd_c128* obs, void* stream) {
  QD_CHECK_ARG(H && psi, "qd_tdse_rk4: null pointer");
  QD_CHECK_ARG(N >= 1 && N <= TD_MAXN && B >= 1 && nsteps >= 0, "qd_tdse_rk4: bad sizes N=%d B=%d", N, B);
  QD_CHECK_ARG(ne >= 0 && (ne == 0 || (E && obs)), "qd_tdse_rk4: E/obs null but ne=%d", ne);
  QD_CHECK_ARG(!obs || save_every > 0 || nsteps == 0, "qd_tdse_rk4: observables need save_every > 0");
  hipStream_t st = (hipStream_t)stream;
  const size_t NN = (size_t)N * N;
  void* w = nullptr;
  int rc = workspace(WS_MISC, (1 + ne) * NN * sizeof(c128), &w);
  if (rc) return rc;
  c128* mHT = (c128*)w;
  c128* ET = mHT + NN;
  hipLaunchKernelGGL(tdse_prep_kernel, dim3((int)std::min<size_t>((NN + 255) / 256, 4096)), dim3(256), 0, st,
                     (const c128*)H, (const c128*)E, ne, N, mHT, ET);
  QD_HIP(hipGetLastError());
  const int nsave = save_every > 0 ? nsteps / save_every : 0;
  hipLaunchKernelGGL(tdse_rk4_kernel, dim3(B), dim3(TD_TPB), 3 * N * sizeof(c128), st, mHT, (c128*)psi, N, dt, nsteps,
                     save_every, nsave, 0, (c128*)snap, ET, ne, ne ? (c128*)obs : nullptr);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_tdse_driven_rk4(const qd_c128* H0, const qd_c128* Hd, int nd, const qd_c128* fvals, qd_c128* psi,
                                  int B, int N, double dt, int nblocks, int nout, qd_c128* snap, const qd_c128* E,
                                  int ne, qd_c128* obs, void* stream) {
  QD_CHECK_ARG(H0 && psi && (nd == 0 || (Hd && fvals)), "qd_tdse_driven_rk4: null pointer");
  QD_CHECK_ARG(N >= 1 && N <= TD_MAXN && B >= 1 && nblocks >= 0 && nout >= 1 && nd >= 0 && nd <= 16,
               "qd_tdse_driven_rk4: bad sizes N=%d B=%d nblocks=%d nout=%d nd=%d", N, B, nblocks, nout, nd);
  QD_CHECK_ARG(ne >= 0 && (ne == 0 || (E && obs)), "qd_tdse_driven_rk4: E/obs null but ne=%d", ne);
  hipStream_t st = (hipStream_t)stream;
  const size_t NN = (size_t)N * N;
  const size_t fl = (size_t)nblocks * nd;
  void* w = nullptr;
  int rc = workspace(WS_MISC, ((1 + ne) * NN + fl) * sizeof(c128), &w);
  if (rc) return rc;
  c128* mHT = (c128*)w;
  c128* ET = mHT + NN;
  c128* fdev = ET + ne * NN;
  const int blocks = (int)std::min<size_t>((NN + 255) / 256, 4096);
  if (ne) {
    hipLaunchKernelGGL(tdse_et_kernel, dim3(blocks), dim3(256), 0, st, (const c128*)E, ne, N, ET);
    QD_HIP(hipGetLastError());
  }
  if (fl) QD_HIP(hipMemcpyAsync(fdev, fvals, fl * sizeof(c128), hipMemcpyHostToDevice, st));
  if (nblocks == 0 && ne) {  // observables at t0 only
    hipLaunchKernelGGL(tdse_driven_prep_kernel, dim3(blocks), dim3(256), 0, st, (const c128*)H0, (const c128*)Hd, 0,
                       (const c128*)fdev, N, mHT);
    hipLaunchKernelGGL(tdse_rk4_kernel, dim3(B), dim3(TD_TPB), 3 * N * sizeof(c128), st, mHT, (c128*)psi, N, dt, 0,
                       nout, 0, 0, (c128*)nullptr, ET, ne, (c128*)obs);
    QD_HIP(hipGetLastError());
  }
  // one launch per block of nout steps: H is constant within a block (mol.py:1944-1951 evaluates
  // calcH(t) with t advanced only after the block)
  for (int k = 0; k < nblocks; ++k) {
    hipLaunchKernelGGL(tdse_driven_prep_kernel, dim3(blocks), dim3(256), 0, st, (const c128*)H0, (const c128*)Hd, nd,
                       (const c128*)fdev + (size_t)k * nd, N, mHT);
    QD_HIP(hipGetLastError());
    hipLaunchKernelGGL(tdse_rk4_kernel, dim3(B), dim3(TD_TPB), 3 * N * sizeof(c128), st, mHT, (c128*)psi, N, dt, nout,
                       nout, nblocks, k, (c128*)snap, ET, ne, ne ? (c128*)obs : nullptr);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}
