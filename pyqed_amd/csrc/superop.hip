// superop.hip — RK4 with a dense Liouville-space generator: d v/dt = L v.
//
// Replaces the csr GEMV loop of pyqed/oqs.py:436-459 (_redfield: rho = rk4(rho,
// rhs, dt, R), rhs = R.dot(rho), oqs.py:462-463) for an arbitrary dense
// superoperator (user-supplied R, Lindblad_solver.liouvillian(), ...).
// HBM-bound: every stage streams L once (16 N2^2 bytes); one wave per row with
// 16-byte lane-strided loads and several loads in flight, the RK4 bookkeeping
// fused into the row epilogue, up to 4 state vectors per pass over L.
#include "qd_common.hpp"

namespace qd {
namespace {

constexpr int SO_TPB = 256;
constexpr int SO_MAXB = 4;

template <int NB>
__global__ __launch_bounds__(SO_TPB) void superop_stage_kernel(const c128* L, int N2, const c128* xin, c128* xout,
                                                               c128* acc, c128* v, int vstride, int stage, double dt) {
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)SO_TPB + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * SO_TPB) >> 6;
  for (long i = wave; i < N2; i += nwaves) {
    const c128* Li = L + i * (long)N2;
    double sr[NB], si[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) sr[b] = si[b] = 0.0;
    int j = lane;
    for (; j + 192 < N2; j += 256) {
      const c128 l0 = Li[j], l1 = Li[j + 64], l2 = Li[j + 128], l3 = Li[j + 192];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const c128* x = xin + (long)b * vstride;
        const c128 x0 = x[j], x1 = x[j + 64], x2 = x[j + 128], x3 = x[j + 192];
        sr[b] += l0.re * x0.re - l0.im * x0.im + l1.re * x1.re - l1.im * x1.im + l2.re * x2.re - l2.im * x2.im +
                 l3.re * x3.re - l3.im * x3.im;
        si[b] += l0.re * x0.im + l0.im * x0.re + l1.re * x1.im + l1.im * x1.re + l2.re * x2.im + l2.im * x2.re +
                 l3.re * x3.im + l3.im * x3.re;
      }
    }
    for (; j < N2; j += 64) {
      const c128 l0 = Li[j];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const c128 x0 = xin[(long)b * vstride + j];
        sr[b] += l0.re * x0.re - l0.im * x0.im;
        si[b] += l0.re * x0.im + l0.im * x0.re;
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
      for (int off = 32; off > 0; off >>= 1) {
        sr[b] += __shfl_xor(sr[b], off, 64);
        si[b] += __shfl_xor(si[b], off, 64);
      }
    if (lane < NB) {
      // lane b finalises vector b (values are wave-uniform after the butterfly)
      double kr = 0, ki = 0;
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (b == lane) { kr = sr[b]; ki = si[b]; }
      const c128 k = cmk(kr, ki);
      const long idx = (long)lane * vstride + i;
      const c128 r0 = v[idx];
      if (stage == 0) {
        acc[idx] = k;
        xout[idx] = cadd(r0, cscale(k, dt / 2.0));
      } else if (stage == 1) {
        acc[idx] = cadd(acc[idx], cscale(k, 2.0));
        xout[idx] = cadd(r0, cscale(k, dt / 2.0));
      } else if (stage == 2) {
        acc[idx] = cadd(acc[idx], cscale(k, 2.0));
        xout[idx] = cadd(r0, cscale(k, dt));
      } else {
        v[idx] = cadd(r0, cscale(cscale(cadd(acc[idx], k), 1.0 / 6.0), dt));
      }
    }
  }
}

// obs[b][s][m] = sum_k W[m][k] v[b][k]  and optional snapshot copy
__global__ void superop_obs_kernel(const c128* v, int N2, const c128* W, int ne, c128* obs, int step, int nrec,
                                   c128* snap, int snap_idx, int nsnap) {
  const int b = blockIdx.y;
  const c128* vb = v + (long)b * N2;
  if (snap && blockIdx.x == 0)
    for (int k = threadIdx.x; k < N2; k += blockDim.x) snap[((long)b * nsnap + snap_idx) * N2 + k] = vb[k];
  __shared__ double red[2 * SO_TPB / 64];
  for (int m = blockIdx.x; m < ne; m += gridDim.x) {
    double sr = 0, si = 0;
    for (int k = threadIdx.x; k < N2; k += blockDim.x) {
      const c128 w = W[(long)m * N2 + k], x = vb[k];
      sr += w.re * x.re - w.im * x.im;
      si += w.re * x.im + w.im * x.re;
    }
    for (int off = 32; off > 0; off >>= 1) {
      sr += __shfl_xor(sr, off, 64);
      si += __shfl_xor(si, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      red[2 * (threadIdx.x >> 6)] = sr;
      red[2 * (threadIdx.x >> 6) + 1] = si;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double a = 0, c = 0;
      for (int w = 0; w < SO_TPB / 64; ++w) { a += red[2 * w]; c += red[2 * w + 1]; }
      obs[((long)b * nrec + step) * ne + m] = cmk(a, c);
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_superop_rk4(const qd_c128* L_, qd_c128* v_, int B, int N2, double dt, int nsteps, const qd_c128* W_,
                              int ne, qd_c128* obs_, qd_c128* snap_, int save_every, void* stream) {
  QD_CHECK_ARG(L_ && v_, "qd_superop_rk4: null pointer");
  QD_CHECK_ARG(B >= 1 && N2 >= 1 && nsteps >= 0, "qd_superop_rk4: bad sizes B=%d N2=%d", B, N2);
  QD_CHECK_ARG(ne == 0 || (W_ && obs_), "qd_superop_rk4: W/obs null but ne=%d", ne);
  hipStream_t st = (hipStream_t)stream;
  const c128* L = (const c128*)L_;
  c128* v = (c128*)v_;
  const c128* W = (const c128*)W_;
  c128* obs = (c128*)obs_;
  c128* snap = (c128*)snap_;
  const size_t tot = (size_t)B * N2;
  void* w = nullptr;
  int rc = workspace(WS_SUPEROP, 3 * tot * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* acc = (c128*)w;
  c128* xs[2] = {acc + tot, acc + 2 * tot};
  const int nsnap = save_every > 0 ? nsteps / save_every : 0;
  const int nrec = nsteps + 1;
  if (ne) {
    hipLaunchKernelGGL(superop_obs_kernel, dim3(std::min(ne, 64), B), dim3(SO_TPB), 0, st, v, N2, W, ne, obs, 0, nrec,
                       nullptr, 0, 0);
    QD_HIP(hipGetLastError());
  }
  const int waves_needed = N2;
  const int grid = std::max(1, std::min(8192, (waves_needed * 64 + SO_TPB - 1) / SO_TPB));
  for (int s = 0; s < nsteps; ++s) {
    for (int stage = 0; stage < 4; ++stage) {
      for (int b0 = 0; b0 < B; b0 += SO_MAXB) {
        const int nb = std::min(SO_MAXB, B - b0);
        const long off = (long)b0 * N2;
        const c128* xin = stage == 0 ? v + off : xs[(stage - 1) & 1] + off;
        c128* xo = xs[stage & 1] + off;
#define SOCALL(NB)                                                                                                 \
  hipLaunchKernelGGL(superop_stage_kernel<NB>, dim3(grid), dim3(SO_TPB), 0, st, L, N2, xin, xo, acc + off, v + off, \
                     N2, stage, dt)
        switch (nb) {
          case 1: SOCALL(1); break;
          case 2: SOCALL(2); break;
          case 3: SOCALL(3); break;
          default: SOCALL(4); break;
        }
#undef SOCALL
        QD_HIP(hipGetLastError());
      }
    }
    const bool take = snap && save_every > 0 && ((s + 1) % save_every == 0);
    if (ne || take) {
      hipLaunchKernelGGL(superop_obs_kernel, dim3(std::max(1, std::min(ne, 64)), B), dim3(SO_TPB), 0, st, v, N2, W,
                         ne, obs, s + 1, nrec, take ? snap : nullptr, take ? (s + 1) / save_every - 1 : 0, nsnap);
      QD_HIP(hipGetLastError());
    }
  }
  return QD_OK;
}
