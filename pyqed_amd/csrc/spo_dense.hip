// spo_dense.hip — SPO3 Strang steps with the kinetic propagator as three per-axis mode products on the f64 MFMAs.
//
// Linear coordinates (wpd.py:1255-1262): exp_K = exp(-i (kx^2/2mx + ky^2/2my + kz^2/2mz) dt) is the outer product
// e_x (x) e_y (x) e_z of per-axis factors, so the kinetic step of _KEO_linear (wpd.py:1418-1432: fftn, * exp_K,
// ifftn) equals M_x (x) M_y (x) M_z with the circulant M_a = F^-1 diag(e_a) F (n_a x n_a): three mode products, one
// pass per axis, each a complex GEMM with K = n_a.  For n_a <= 64 that GEMM is short enough (8 n_a flops per point
// per axis) that a pass runs at the MFMA rate instead of the dependent load -> LDS FFT stages -> store chain of the
// FFT passes, and any length works alike (no mixed-radix plan: 60^3 costs what 64^3 costs).
//
// One pass: psi[outer][i][inner] <- sum_k M[i][k] psi[outer][k][inner] with the circulant M[i][k] = m[(i - k) mod n],
// in place.  Column c = outer * st + inner (st = the axis stride); a workgroup owns 16 consecutive columns and all n
// output rows, one wave per 16 rows.  No LDS and no barrier before the MFMAs: every lane loads its A fragments (from
// the n-element vector m, L1-resident) and its B fragments (its column's element at k = 4 q + lane / 16, a fixed
// stride apart) straight into registers, in k order, so each k-step's MFMAs wait only for their own loads; the four
// waves' B loads of one column hit the same lines.  One barrier before the stores (the pass is in place).  The last
// pass of a step (z, st = ns) applies exp(-iV dt/2) per point in its epilogue -- and, between steps, the next step's
// half again after the snapshot -- the two states of a point sitting in neighbouring lanes.
#include "qd_common.hpp"

namespace qd {
namespace {

constexpr int SD_MAXN = 64;

struct SdPass {
  c128* psi;        // state, updated in place
  const c128* m;    // [n] first column of the circulant axis propagator
  unsigned C;       // columns (points x ns / n)
  unsigned st;      // axis stride in elements
  int n;
  const c128* Vh;   // last pass: [npts][ns][ns] point propagators, else null
  c128* snap;       // last pass: the state after the step's closing half (a snapshot step), else null
  int vh2;          // last pass: apply the next step's opening half too
};

// NS: 0 = plain pass; 1 / 2 = the z pass (st = NS) with its point epilogue for NS states
template <int NS>
__global__ __launch_bounds__(256) void spo_axis_kernel(SdPass p) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = p.n, nq = (n + 3) >> 2;
  const unsigned st = p.st;
  const unsigned c = blockIdx.x * 16 + (lane & 15);
  const bool live = c < p.C;
  const unsigned o = c / st, in = c - o * st;
  c128* col = p.psi + (size_t)o * n * st + in;   // this lane's column: element k at col[k * st]
  const int ai = 16 * w + (lane & 15), kl = lane >> 4;

  c128 a[SD_MAXN / 4], b[SD_MAXN / 4];
#pragma unroll
  for (int q = 0; q < SD_MAXN / 4; ++q) {
    if (q < nq) {
      const int k = 4 * q + kl;
      int d = ai - k;
      d += d < 0 ? n : 0;
      a[q] = (ai < n && k < n) ? p.m[d] : cmk(0.0, 0.0);
      b[q] = (live && k < n) ? col[(size_t)k * st] : cmk(0.0, 0.0);
    }
  }
  // one accumulator pair per wave: splitting K over more pairs (4: 72 us per 64^3 step, 8: 39) and the
  // three-multiplication form (42) were all slower than this (32; profiles/r06/spo/spo3_axes_ab.txt)
  d4 accr = d4{0.0, 0.0, 0.0, 0.0}, acci = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < SD_MAXN / 4; ++q) {
    if (q < nq) {   // uniform; the loops stay unrolled so a[q], b[q] are registers
      accr = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q].re, b[q].re, accr, 0, 0, 0);
      acci = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q].re, b[q].im, acci, 0, 0, 0);
      accr = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[q].im, b[q].im, accr, 0, 0, 0);
      acci = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q].im, b[q].re, acci, 0, 0, 0);
    }
  }
  __syncthreads();   // in place: every wave has consumed its loads of these columns

  // D: lane holds rows 16 w + lane / 16 + 4 r of its column
  if constexpr (NS == 0) {
    if (live) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * w + kl + 4 * r;
        if (i < n) col[(size_t)i * st] = cmk(accr[r], acci[r]);
      }
    }
  } else {
    // z pass: in = s; the other state of the point is in lane ^ 1 (NS = 2)
    const int s = (int)in;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * w + kl + 4 * r;
      const c128 own = cmk(accr[r], acci[r]);
      c128 u0 = own, u1 = own;
      if constexpr (NS == 2) {
        const c128 x = cmk(__shfl_xor(accr[r], 1), __shfl_xor(acci[r], 1));
        u0 = s ? x : own;
        u1 = s ? own : x;
      }
      if (!live || i >= n) continue;
      const size_t gp = (size_t)o * n + i;
      const c128* V = p.Vh + gp * NS * NS + s * NS;   // this lane's row of the point's operator
      const c128 v00 = V[0];
      const c128 v01 = NS == 2 ? V[NS == 2 ? 1 : 0] : v00;
      c128 v = cmul(v00, u0);
      if constexpr (NS == 2) v = cadd(v, cmul(v01, u1));
      if (p.snap) p.snap[gp * NS + s] = v;
      if (p.vh2) {
        if constexpr (NS == 2) {
          const c128 y = cmk(__shfl_xor(v.re, 1), __shfl_xor(v.im, 1));
          v = cadd(cmul(v00, s ? y : v), cmul(v01, s ? v : y));
        } else {
          v = cmul(v00, v);
        }
      }
      col[(size_t)i * st] = v;
    }
  }
}

// psi <- Vh psi per point (the first step's opening half)
template <int NS>
__global__ void spo_half_kernel(c128* psi, const c128* Vh, size_t npts) {
  for (size_t gp = (size_t)blockIdx.x * blockDim.x + threadIdx.x; gp < npts; gp += (size_t)gridDim.x * blockDim.x) {
    c128 u[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) u[s] = psi[gp * NS + s];
    const c128* V = Vh + gp * NS * NS;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      c128 acc = cmul(V[s * NS], u[0]);
#pragma unroll
      for (int q = 1; q < NS; ++q) acc = cadd(acc, cmul(V[s * NS + q], u[q]));
      psi[gp * NS + s] = acc;
    }
  }
}

template <int NS>
int run_axes(c128* psi, const c128* Vh, const c128* const m[3], const int d[3], int nsteps, int nout, c128* snap,
             hipStream_t st) {
  const size_t npts = (size_t)d[0] * d[1] * d[2];
  const int hb = (int)std::min<size_t>((npts + 255) / 256, 4096);
  hipLaunchKernelGGL(spo_half_kernel<NS>, dim3(hb), dim3(256), 0, st, psi, Vh, npts);
  QD_HIP(hipGetLastError());
  const unsigned tot = (unsigned)(npts * NS);
  const unsigned stride[3] = {(unsigned)(d[1] * d[2] * NS), (unsigned)(d[2] * NS), (unsigned)NS};
  for (int s = 0; s < nsteps; ++s) {
    for (int a = 0; a < 3; ++a) {
      SdPass p{};
      p.psi = psi;
      p.m = m[a];
      p.n = d[a];
      p.st = stride[a];
      p.C = tot / d[a];
      const dim3 grid((p.C + 15) / 16), block(64 * ((d[a] + 15) / 16));
      if (a < 2) {
        hipLaunchKernelGGL(spo_axis_kernel<0>, grid, block, 0, st, p);
      } else {
        p.Vh = Vh;
        p.snap = (snap && (s + 1) % nout == 0) ? snap + (size_t)((s + 1) / nout - 1) * npts * NS : nullptr;
        p.vh2 = s + 1 < nsteps;
        hipLaunchKernelGGL(spo_axis_kernel<NS>, grid, block, 0, st, p);
      }
      QD_HIP(hipGetLastError());
    }
  }
  return QD_OK;
}

}  // namespace

// spo.hip: 64^3 grids on the register transforms (three separable passes per step)
int spo3_sep64_run(c128* psi, const c128* Vh, const c128* const m[3], int ns, int nsteps, int nout, c128* snap,
                   hipStream_t st);
}  // namespace qd

using namespace qd;

extern "C" int qd_spo3_run_axes(qd_c128* psi, const qd_c128* expVh, const qd_c128* mx, const qd_c128* my,
                                const qd_c128* mz, int nx, int ny, int nz, int ns, int nsteps, int nout, qd_c128* snap,
                                void* stream) {
  QD_CHECK_ARG(psi && expVh && mx && my && mz, "qd_spo3_run_axes: null pointer");
  QD_CHECK_ARG(nx >= 1 && ny >= 1 && nz >= 1 && nx <= SD_MAXN && ny <= SD_MAXN && nz <= SD_MAXN,
               "qd_spo3_run_axes: nx=%d ny=%d nz=%d outside [1, %d]", nx, ny, nz, SD_MAXN);
  QD_CHECK_ARG(ns == 1 || ns == 2, "qd_spo3_run_axes: ns=%d (1 or 2)", ns);
  QD_CHECK_ARG(nsteps >= 0 && nout >= 1, "qd_spo3_run_axes: nsteps=%d nout=%d", nsteps, nout);
  if (nsteps == 0) return QD_OK;
  const c128* m[3] = {(const c128*)mx, (const c128*)my, (const c128*)mz};
  const int d[3] = {nx, ny, nz};
  hipStream_t st = (hipStream_t)stream;
  if (nx == 64 && ny == 64 && nz == 64) {
    WsScope wss_(st);
    note_path("spo3_sep64");
    return spo3_sep64_run((c128*)psi, (const c128*)expVh, m, ns, nsteps, nout, (c128*)snap, st);
  }
  note_path("spo3_axes");
  return ns == 1 ? run_axes<1>((c128*)psi, (const c128*)expVh, m, d, nsteps, nout, (c128*)snap, st)
                 : run_axes<2>((c128*)psi, (const c128*)expVh, m, d, nsteps, nout, (c128*)snap, st);
}
