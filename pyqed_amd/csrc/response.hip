// response.hip — Liouville-space response functions on the (t1, t2, t3) grid.
//
// Eigen (sum-over-states) form of the reference's SOS propagator
// (pyqed/oqs.py:160-214: eig(R), U = U1 diag(e^{lam t}) U1^-1, G = -iU) and of
// correlation_4op_3t (oqs.py:268-357):
//   S[i,j,k] = <<I| a G(tau_i) b G(tau_j) c G(tau_k) d |rho0>>
//            = (-i)^3 sum_pqr alpha_p e^{lam_p tau_i} B_pq e^{lam_q tau_j} C_qr e^{lam_r tau_k} beta_r
// with alpha = I^T a U1, B = U1^-1 b U1, C = U1^-1 c U1, beta = U1^-1 d rho0
// (host-side setup, like the reference's eig).  Kernels:
//   qd_sos_propagator     U[a][b][k]                  (oqs.py:210 contraction)
//   qd_response_cube      S[i][j][k], full n^3 cube   (oqs.py:339-357 tensordots)
//   qd_response2d_ensemble  sum over M disorder members of the (t3, t1) slice at
//                         fixed t2 — one complex GEMM
//                           S = X [n3 x K] * Z [K x n1],  K = M * nL,
//                           X[i][m*nL+p] = i * alpha_mp e^{lam_mp t3_i}
//                           Z[m*nL+p][k] = sum_q Mt_mpq beta_mq e^{lam_mq t1_k},
//                           Mt_m = B_m diag(e^{lam_m t2}) C_m  (host)
//                         run split-K over workgroups on the MFMA block engine
//                         with a deterministic slab reduction.
#include "cgemm_block.hpp"

namespace qd {
namespace {

__device__ __forceinline__ c128 cexp_t(c128 lam, double t) {
  // exp(lam * t) for real t, numpy's formula exp(re)*(cos im, sin im)
  const double er = exp(lam.re * t);
  double s, c;
  sincos(lam.im * t, &s, &c);
  return cmk(er * c, er * s);
}

__global__ void sos_propagator_kernel(const c128* U1, const c128* U2, const c128* lam, int nL, const double* t, int nt,
                                      c128* U) {
  const size_t tot = (size_t)nL * nL * nt;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % nt);
    const int b = (int)((e / nt) % nL);
    const int a = (int)(e / ((size_t)nt * nL));
    const double tk = t[k];
    c128 s = cmk(0, 0);
    for (int j = 0; j < nL; ++j) s = cadd(s, cmul(cmul(U1[(size_t)a * nL + j], cexp_t(lam[j], tk)), U2[(size_t)j * nL + b]));
    U[e] = s;
  }
}

// Y[k][q] = sum_r C[q][r] e^{lam_r t1_k} beta_r
__global__ void cube_y_kernel(const c128* C, const c128* beta, const c128* lam, int nL, const double* t1, int n1,
                              c128* Y) {
  const size_t tot = (size_t)n1 * nL;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int q = (int)(e % nL), k = (int)(e / nL);
    c128 s = cmk(0, 0);
    for (int r = 0; r < nL; ++r) s = cadd(s, cmul(C[(size_t)q * nL + r], cmul(cexp_t(lam[r], t1[k]), beta[r])));
    Y[e] = s;
  }
}

// W[j][p][k] = sum_q B[p][q] e^{lam_q t2_j} Y[k][q]
__global__ void cube_w_kernel(const c128* B, const c128* Y, const c128* lam, int nL, const double* t2, int n2, int n1,
                              c128* W) {
  const size_t tot = (size_t)n2 * nL * n1;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % n1);
    const int p = (int)((e / n1) % nL);
    const int j = (int)(e / ((size_t)n1 * nL));
    c128 s = cmk(0, 0);
    for (int q = 0; q < nL; ++q)
      s = cadd(s, cmul(cmul(B[(size_t)p * nL + q], cexp_t(lam[q], t2[j])), Y[(size_t)k * nL + q]));
    W[e] = s;
  }
}

// out[i][j][k] = i * sum_p alpha_p e^{lam_p t3_i} W[j][p][k]      ((-i)^3 = i)
// One block per (i, j) row; the p-loop coefficients are staged in LDS.
__global__ void cube_out_kernel(const c128* alpha, const c128* lam, const c128* W, int nL, const double* t3, int n3,
                                int n2, int n1, c128* out) {
  extern __shared__ c128 xs[];
  const int ij = blockIdx.x;
  const int i = ij / n2, j = ij % n2;
  for (int p = threadIdx.x; p < nL; p += blockDim.x) xs[p] = cmuli(cmul(alpha[p], cexp_t(lam[p], t3[i])));
  __syncthreads();
  const c128* Wj = W + (size_t)j * nL * n1;
  c128* o = out + ((size_t)i * n2 + j) * n1;
  for (int k = threadIdx.x; k < n1; k += blockDim.x) {
    c128 s = cmk(0, 0);
    for (int p = 0; p < nL; ++p) s = cadd(s, cmul(xs[p], Wj[(size_t)p * n1 + k]));
    o[k] = s;
  }
}

// ---------------------------------------------------------------- ensemble 2D slice
// One launch builds both GEMM operands (two bandwidth-bound writes of n x K c128 overlap):
//   blockIdx.y <  M : Z rows of member m (below)
//   blockIdx.y >= M : X [n3p][Kp], X[i][m*nL+p] = i * alpha_mp e^{lam_mp t3_i} (zero in the padding),
//                     grid-strided over the (blockIdx.y - M, blockIdx.x) blocks
// Z [Kp][n1p]: Z[m*nL+p][k] = sum_q Mt[m][p][q] y_q(k),  y_q(k) = beta[m][q] e^{lamz_mq t1_k}
// one thread per t1 point computes the nz exponentials once (registers, nz <= ZMAX) and emits the
// nL outputs of its column; Mt_m (nL x nz, rectangular when structurally zero alpha / beta columns
// were pruned on the host) staged in LDS.
constexpr int ZMAX = 16;
__global__ __launch_bounds__(256) void ens_xz_kernel(const c128* Mt, const c128* beta, const c128* lam, int M, int nL,
                                                     const double* t1, int n1, int n1p, int Kp, c128* Z,
                                                     const c128* alpha, const double* t3, int n3, int n3p, int xrows,
                                                     int K, c128* X, int nz, const c128* lamz) {
  __shared__ c128 sM[ZMAX * ZMAX];
  if ((int)blockIdx.y >= M) {
    const size_t tot = (size_t)n3p * Kp;
    const size_t nthr = (size_t)xrows * gridDim.x * blockDim.x;
    for (size_t e = ((size_t)(blockIdx.y - M) * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; e < tot;
         e += nthr) {
      const int kk = (int)(e % Kp), i = (int)(e / Kp);
      c128 v = cmk(0, 0);
      if (i < n3 && kk < K) v = cmuli(cmul(alpha[kk], cexp_t(lam[kk], t3[i])));
      X[e] = v;
    }
    return;
  }
  const int m = blockIdx.y;
  const int k = blockIdx.x * 256 + threadIdx.x;
  for (int e = threadIdx.x; e < nL * nz; e += 256) sM[e] = Mt[(size_t)m * nL * nz + e];
  __syncthreads();
  if (k >= n1p) return;
  c128 y[ZMAX];
  const double tk = k < n1 ? t1[k] : 0.0;
#pragma unroll
  for (int q = 0; q < ZMAX; ++q)
    y[q] = (q < nz && k < n1) ? cmul(beta[(size_t)m * nz + q], cexp_t(lamz[(size_t)m * nz + q], tk)) : cmk(0, 0);
  for (int p = 0; p < nL; ++p) {
    c128 v = cmk(0, 0);
#pragma unroll
    for (int q = 0; q < ZMAX; ++q)
      if (q < nz) v = cadd(v, cmul(sM[p * nz + q], y[q]));
    Z[((size_t)m * nL + p) * n1p + k] = v;
  }
}

// ---- uniform time grids (t = t0 + j dt): exponentials from two-level tables,
// e^{lam (t0 + (16 l + j) dt)} = e^{lam (t0 + 16 l dt)} * e^{lam j dt}; the coarse factor is a direct
// exponential, the fine table a product chain of e^{lam dt} (<= 15 products).  A handful of
// transcendentals per 16-64 outputs instead of one per output; relative error ~1e-14.
constexpr int UNI_ROWS = 64;  // P rows per block (t2 scan)
constexpr int XU_ROWS = 16;   // materialised uniform X: rows per block (one 16-row group: more, shorter blocks)
__device__ __forceinline__ void ens_x_uniform_block(int bx, int by, const c128* alpha, const c128* lam, int K, int Kp,
                                                    double t0, double dt, int n3, int n3p, c128* X) {
  const int kk = bx * 256 + threadIdx.x;
  const int i0 = by * XU_ROWS;
  if (kk >= Kp) return;
  const bool col = kk < K;
  const c128 l = col ? lam[kk] : cmk(0, 0);
  const c128 a = col ? cmuli(alpha[kk]) : cmk(0, 0);
  c128 T1[16];
  T1[0] = cmk(1, 0);
  const c128 st = cexp_t(l, dt);
#pragma unroll
  for (int j = 1; j < 16; ++j) T1[j] = cmul(T1[j - 1], st);
  for (int g = 0; g < XU_ROWS / 16; ++g) {
    const int ib = i0 + 16 * g;
    const c128 base = cmul(a, cexp_t(l, t0 + (double)ib * dt));
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = ib + j;
      if (i >= n3p) break;
      X[(size_t)i * Kp + kk] = (col && i < n3) ? cmul(base, T1[j]) : cmk(0, 0);
    }
  }
}

// Z rows of member m = blockIdx.y, uniform t1: tables of e^{lam_q t} in LDS (nL x (16 + n1p/16)).
constexpr int UNI_MAXC = 1024 / 16;
// One launch, both operands: blockIdx.y < M -> Z rows of member blockIdx.y (blockIdx.x = column
// block); blockIdx.y >= M -> X block (blockIdx.y - M) in a (Kp/256) x (n3p/XU_ROWS) tiling.
__global__ __launch_bounds__(256) void ens_xz_uniform_kernel(const c128* Mt, const c128* beta, const c128* lam, int M,
                                                             int nL, double t0, double dt, int n1, int n1p, int Kp,
                                                             c128* Z, const c128* alpha, int K, double t3_0,
                                                             double dt3, int n3, int n3p, int xbx, c128* X, int nz,
                                                             const c128* lamz) {
  __shared__ c128 sM[ZMAX * ZMAX];
  __shared__ c128 sF[ZMAX * 16];        // e^{lam_q j dt}
  __shared__ c128 sC[ZMAX * UNI_MAXC];  // beta_q e^{lam_q (t0 + 16 l dt)}
  if ((int)blockIdx.y >= M) {
    if (blockIdx.x != 0) return;
    const int xb = blockIdx.y - M;
    ens_x_uniform_block(xb % xbx, xb / xbx, alpha, lam, K, Kp, t3_0, dt3, n3, n3p, X);
    return;
  }
  const int m = blockIdx.y;
  const int nC = n1p / 16;
  const c128* lm = lamz + (size_t)m * nz;
  for (int e = threadIdx.x; e < nL * nz; e += 256) sM[e] = Mt[(size_t)m * nL * nz + e];
  for (int e = threadIdx.x; e < nz * 16; e += 256) sF[e] = cexp_t(lm[e / 16], (double)(e % 16) * dt);
  for (int e = threadIdx.x; e < nz * nC; e += 256)
    sC[e] = cmul(beta[(size_t)m * nz + e / nC], cexp_t(lm[e / nC], t0 + 16.0 * (double)(e % nC) * dt));
  __syncthreads();
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n1p) return;
  c128 y[ZMAX];
#pragma unroll
  for (int q = 0; q < ZMAX; ++q)
    y[q] = (q < nz && k < n1) ? cmul(sC[q * nC + (k >> 4)], sF[q * 16 + (k & 15)]) : cmk(0, 0);
  for (int p = 0; p < nL; ++p) {
    c128 v = cmk(0, 0);
#pragma unroll
    for (int q = 0; q < ZMAX; ++q)
      if (q < nz) v = cadd(v, cmul(sM[p * nz + q], y[q]));
    Z[((size_t)m * nL + p) * n1p + k] = v;
  }
}

// Z rows of G members per block (uniform t1), tables in dynamic LDS: per member Mt_m (nL x nz), the fine
// table e^{lamz_q j dt} (nz x 16) and the coarse one beta_q e^{lamz_q (t0 + 16 l dt)} (nz x nC).  Every
// wave takes part in the table phase (G nz (16 + nC) exponentials per block instead of nz (16 + nC) per
// 256-thread block), and a block then streams G nL full Z rows.  Blocks blockIdx.y >= ceil(M / G) build
// X blocks instead (materialised uniform X, when the A operand is not generated in the GEMM).
__global__ __launch_bounds__(256) void ens_z_uniform_kernel(const c128* Mt, const c128* beta, const c128* lamz, int M,
                                                            int nL, int nz, int G, double t0, double dt, int n1,
                                                            int n1p, c128* Z, const c128* alpha, const c128* lamx,
                                                            int K, int Kp, double t3_0, double dt3, int n3, int n3p,
                                                            int xbx, c128* X) {
  extern __shared__ c128 zs[];
  const int nMB = (M + G - 1) / G;
  if ((int)blockIdx.y >= nMB) {
    if (blockIdx.x != 0) return;
    const int xb = blockIdx.y - nMB;
    ens_x_uniform_block(xb % xbx, xb / xbx, alpha, lamx, K, Kp, t3_0, dt3, n3, n3p, X);
    return;
  }
  const int nC = n1p / 16;
  const int per = nL * nz + nz * (16 + nC);
  const int m0 = blockIdx.y * G;
  const int g = min(G, M - m0);
  // round 1: every input of the block's members (Mt, lamz, beta) in one parallel load round into LDS
  c128* sLam = zs + G * per;
  c128* sBeta = sLam + G * nz;
  for (int e = threadIdx.x; e < g * nL * nz; e += 256)
    zs[(e / (nL * nz)) * per + e % (nL * nz)] = Mt[(size_t)m0 * nL * nz + e];
  for (int e = threadIdx.x; e < g * nz; e += 256) {
    sLam[e] = lamz[(size_t)m0 * nz + e];
    sBeta[e] = beta[(size_t)m0 * nz + e];
  }
  __syncthreads();
  // round 2: the exponential tables from LDS operands (no global latency inside the loop)
  // one thread per (member, q): fine[j] = e^{lam j dt} as powers of e^{lam dt}, coarse[l] = beta e^{lam t0} times
  // powers of e^{16 lam dt} (3 exponentials instead of 16 + nC; relative error ~1e-14)
  for (int e = threadIdx.x; e < g * nz; e += 256) {
    const int gi = e / nz, q = e - gi * nz;
    const c128 l = sLam[gi * nz + q];
    c128* fine = zs + gi * per + nL * nz + q * 16;
    c128* coarse = zs + gi * per + nL * nz + nz * 16 + q * nC;
    const c128 e1 = cexp_t(l, dt);
    c128 f = cmk(1.0, 0.0);
    fine[0] = f;
    for (int j = 1; j < 16; ++j) {
      f = cmul(f, e1);
      fine[j] = f;
    }
    const c128 e16 = cexp_t(l, 16.0 * dt);
    c128 c = cmul(sBeta[gi * nz + q], cexp_t(l, t0));
    for (int u = 0; u < nC; ++u) {
      coarse[u] = c;
      c = cmul(c, e16);
    }
  }
  __syncthreads();
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n1p) return;
  for (int gi = 0; gi < g; ++gi) {
    const c128* sM = zs + gi * per;
    const c128* sF = sM + nL * nz;
    const c128* sC = sF + nz * 16;
    c128 y[ZMAX];
#pragma unroll
    for (int q = 0; q < ZMAX; ++q)
      y[q] = (q < nz && k < n1) ? cmul(sC[q * nC + (k >> 4)], sF[q * 16 + (k & 15)]) : cmk(0, 0);
    for (int p = 0; p < nL; ++p) {
      c128 v = cmk(0, 0);
#pragma unroll
      for (int q = 0; q < ZMAX; ++q)
        if (q < nz) v = cadd(v, cmul(sM[p * nz + q], y[q]));
      Z[((size_t)(m0 + gi) * nL + p) * n1p + k] = v;
    }
  }
}

// members per block of ens_z_uniform_kernel: tables of <= 32 KB LDS, at most 32 members
// and at least 1024 member blocks when M allows (M = 4096: 0.128 -> 0.116 ms per 256 x 256 grid; no change at
// M = 32k, where the LDS cap binds; tools/zblocks_ab.sh)
int z_group(int nL, int nz, int n1p, int M) {
  const int per = nL * nz + nz * (16 + n1p / 16) + 2 * nz;
  const int G = std::max(1, std::min(32, 2048 / per));
  return std::max(1, std::min(G, M / 1024));
}
// its dynamic LDS bytes
size_t z_lds(int G, int nL, int nz, int n1p) {
  return (size_t)G * (nL * nz + nz * (16 + n1p / 16) + 2 * nz) * sizeof(c128);
}

// rows K..Kp-1 of Z are padding
__global__ void ens_z_pad_kernel(int K, int Kp, int n1p, c128* Z) {
  const size_t tot = (size_t)(Kp - K) * n1p;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x)
    Z[(size_t)K * n1p + e] = cmk(0, 0);
}

// Generic fallback for nL > ZMAX (one thread per output element).
__global__ void ens_z_generic_kernel(const c128* Mt, const c128* beta, const c128* lam, int M, int nL,
                                     const double* t1, int n1, int n1p, int Kp, c128* Z, int nz) {
  const size_t tot = (size_t)Kp * n1p;
  const int K = M * nL;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % n1p), row = (int)(e / n1p);
    c128 v = cmk(0, 0);
    if (row < K && k < n1) {
      const int m = row / nL, p = row % nL;
      const c128* Mr = Mt + ((size_t)m * nL + p) * nz;
      for (int q = 0; q < nz; ++q)
        v = cadd(v, cmul(Mr[q], cmul(beta[(size_t)m * nz + q], cexp_t(lam[(size_t)m * nz + q], t1[k]))));
    }
    Z[e] = v;
  }
}

// Uniform t3 without materialising X: X[i][kk] = coarse[i >> 4][kk] * fine[i & 15][kk] with
//   coarse[c][kk] = i alpha_kk e^{lam_kk (t0 + 16 c dt)},  fine[j][kk] = (e^{lam_kk dt})^j (product chain),
// the same factors (and roundings) ens_x_uniform_block multiplies, formed by the GEMM's A staging instead
// (tables: (n3p/16 + 16) x Kp, 1/8 of X at n3p = 256).  Columns kk >= K are zero; rows past n3 inside the
// last 16-row group are finite and only reach output rows the reduction never reads.
__global__ __launch_bounds__(256) void ens_xtab_kernel(const c128* alpha, const c128* lam, int K, int Kp, double t0,
                                                       double dt, int n3, int n3p, c128* coarse, c128* fine) {
  const int kk = blockIdx.x * 256 + threadIdx.x;
  if (kk >= Kp) return;
  const bool col = kk < K;
  const c128 l = col ? lam[kk] : cmk(0, 0);
  const c128 a = col ? cmuli(alpha[kk]) : cmk(0, 0);
  const c128 st = cexp_t(l, dt);
  c128 f = cmk(1, 0);
  for (int j = 0; j < 16; ++j) {
    fine[(size_t)j * Kp + kk] = f;
    f = cmul(f, st);
  }
  for (int c = 0; c < n3p / 16; ++c)
    coarse[(size_t)c * Kp + kk] = (col && 16 * c < n3) ? cmul(a, cexp_t(l, t0 + (double)(16 * c) * dt)) : cmk(0, 0);
}

constexpr int ENS_BT = 128;
#ifndef ENS_PIPE
#define ENS_PIPE false  // fragment double-buffering (PIPE) fits (250 VGPRs, no scratch) but measured neutral here
#endif

// A operand X [n3p][Kp] (materialised by ens_xz_kernel), streamed one tile ahead.
struct EnsXA {
  using Raw = cg_v2;
  const c128* X;
  int Kp, row0, k0;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    return cg_ld(X + (size_t)(row0 + (e >> 4)) * Kp + k0 + t * CG_KT + (e & 15));
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int, int, int) const { return r; }
};

struct EnsXTab {
  struct Raw {
    cg_v2 c, f;
  };
  const c128* coarse;
  const c128* fine;
  int Kp, row0, k0;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    const int row = row0 + (e >> 4);
    const size_t kk = (size_t)k0 + t * CG_KT + (e & 15);
    return Raw{cg_ld(coarse + (size_t)(row >> 4) * Kp + kk), cg_ld(fine + (size_t)(row & 15) * Kp + kk)};
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int, int, int) const {
    const c128 v = cmul(cmk(r.c.x, r.c.y), cmk(r.f.x, r.f.y));
    return cg_v2{v.re, v.im};
  }
};

template <int BT = ENS_BT>
struct EnsZB {
  using Raw = cg_v2;
  const c128* Z;
  int n1p, col0, k0;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    return cg_ld(Z + (size_t)(k0 + t * CG_KT + e / BT) * n1p + col0 + (e % BT));
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int, int, int) const { return r; }
};

// XCD-aware tile order for the split-K GEMMs (speed only: any placement computes the same tiles).
// Workgroups are dealt round-robin over the 8 XCDs, so linear id L runs on XCD L % 8.  Tile u (column
// block fastest, then row block, then K split) is given to L with u = (L % 8) * (T / 8) + L / 8: each
// XCD owns a contiguous run of tiles, i.e. whole rows of column blocks that share one A (P / X) K-range
// and neighbouring row blocks that share B (Q / Z) tiles, in its own L2.  Identity when T % 8 != 0.
__device__ __forceinline__ void ens_tile(int& bn, int& bm, int& s) {
  const int NX = gridDim.x, NY = gridDim.y, T = NX * NY * gridDim.z;
  const int L = blockIdx.x + NX * (blockIdx.y + NY * blockIdx.z);
  const int u = (T % 8 == 0) ? (L % 8) * (T / 8) + L / 8 : L;
  bn = u % NX;
  bm = (u / NX) % NY;
  s = u / (NX * NY);
}

// grid: (n1p/BT) x (n3p/BT) x S ; each workgroup accumulates K-tiles [t0, t1) of its block.  BT = 64 for
// problems whose 128-blocks cannot fill the chip with >= 4 K-tiles per workgroup (4x the blocks, 1/4 the
// split-K slabs to write and reduce).
template <int BT, bool XTAB, int DEPTH = 1>
__global__ __launch_bounds__(CG_WG) void ens_gemm_kernel(const c128* X, int Kp, const c128* Z, int n1p, int tiles,
                                                         int S, c128* slabs, int n3p, const c128* fine) {
  __shared__ CgLds<BT> L;
  int bn, bm, s;
  ens_tile(bn, bm, s);
  const int t0 = (int)((long)tiles * s / S), t1 = (int)((long)tiles * (s + 1) / S);
  CgAcc<BT> A;
  c128* slab = slabs + (size_t)s * n3p * n1p;
  if (t1 > t0) {
    EnsZB<BT> pb{Z, n1p, bn * BT, t0 * CG_KT};
    if constexpr (XTAB) {
      EnsXTab pa{X, fine, Kp, bm * BT, t0 * CG_KT};  // X = the coarse table
      cg_block_gemm_gen<BT, ENS_PIPE>(t1 - t0, pa, pb, L, A);
    } else {
      EnsXA pa{X, Kp, bm * BT, t0 * CG_KT};
      if constexpr (DEPTH == 2)   // fragment double-buffering for the 64-blocks (shard: 0.1630 vs 0.1653 ms per grid;
                                  // the 128-blocks slow down with it, 1.53 vs 1.19 ms: profiles/r06/2des/knobs_ab.txt)
        cg_block_gemm_gen2<BT, ENS_PIPE || BT == 64>(t1 - t0, pa, pb, L, A);
      else
        cg_block_gemm_gen<BT, ENS_PIPE>(t1 - t0, pa, pb, L, A);
    }
    cg_epilogue<BT>(A, [&](int row, int col, c128 v) {
      slab[(size_t)(bm * BT + row) * n1p + bn * BT + col] = v;
    });
  } else {
    for (int e = threadIdx.x; e < BT * BT; e += CG_WG)
      slab[(size_t)(bm * BT + e / BT) * n1p + bn * BT + e % BT] = cmk(0, 0);
  }
}

// (BT, S) for a split-K GEMM of Mp x Np (multiples of 128) over `tiles` K-tiles: 128-blocks with enough
// splits to cover the 256 CUs once at >= 4 K-tiles per workgroup; 64-blocks when that leaves the chip
// under-filled or gives a workgroup fewer than 32 K-tiles (the S partial slabs to write and reduce then
// cost more than the 64-block's lower operand reuse; measured on the 256 x 256 2DES grid: 64-blocks
// win at K <= 8k, 128-blocks from K = 32k).  QD_ENS_BT=64/128 forces the block size (A/B runs).
struct SplitPlan {
  int bt, S;
};
SplitPlan split_plan(int Mp, int Np, int tiles) {
  // 64-blocks: two workgroups per CU (69.6 KB of LDS each), 512 in all (8,192-member shard: 0.169-0.170 vs 0.172-0.173
  // ms per grid at 256; 384 and 768 slower, profiles/r05/2des/wg64_splits_ab.txt); 128-blocks hold one per CU
  auto splits = [&](int bt) {
    const int blocks = (Mp / bt) * (Np / bt);
    return std::max(1, std::min(ceil_div(bt == 64 ? 512 : 256, blocks), std::max(1, tiles / 4)));
  };
  const int S128 = splits(128);
#ifndef ENS_MIN_TILES128
#define ENS_MIN_TILES128 32
#endif
  const bool small = (Mp / 128) * (Np / 128) * S128 < 256 || tiles / S128 < ENS_MIN_TILES128;
  const int bt = small ? 64 : 128;
  return {bt, splits(bt)};
}

// fine != nullptr: X is the coarse table of ens_xtab_kernel (generated A operand)
void launch_ens_gemm(const SplitPlan& pl, const c128* X, int Kp, const c128* Z, int Mp, int Np, int tiles,
                     c128* slabs, hipStream_t st, const c128* fine = nullptr) {
  const dim3 g(Np / pl.bt, Mp / pl.bt, pl.S);
  // the 64-block path keeps two K-tiles of global loads in flight (4,096-member shard: 0.111 ms per grid at 2 vs
  // 0.113 at 1, tools/ens_depth_ab.sh)
  note_path(pl.bt == 64 ? (fine ? "ens_gemm64_xtab" : "ens_gemm64") : (fine ? "ens_gemm128_xtab" : "ens_gemm128"));
  if (pl.bt == 64) {
    if (fine)
      hipLaunchKernelGGL((ens_gemm_kernel<64, true>), g, dim3(CG_WG), 0, st, X, Kp, Z, Np, tiles, pl.S, slabs, Mp, fine);
    else
      hipLaunchKernelGGL((ens_gemm_kernel<64, false, 2>), g, dim3(CG_WG), 0, st, X, Kp, Z, Np, tiles, pl.S, slabs, Mp, fine);
  } else {
    if (fine)
      hipLaunchKernelGGL((ens_gemm_kernel<128, true>), g, dim3(CG_WG), 0, st, X, Kp, Z, Np, tiles, pl.S, slabs, Mp, fine);
    else
      hipLaunchKernelGGL((ens_gemm_kernel<128, false>), g, dim3(CG_WG), 0, st, X, Kp, Z, Np, tiles, pl.S, slabs, Mp, fine);
  }
}

// out[i][k] (+)= sum_s slab[s][i][k], fixed order -> deterministic
__global__ void ens_reduce_kernel(const c128* slabs, int S, int n3, int n1, int n3p, int n1p, c128* out,
                                  int accumulate) {
  const size_t tot = (size_t)n3 * n1;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / n1), k = (int)(e % n1);
    c128 v = accumulate ? out[e] : cmk(0, 0);
    v = slab_sum(v, 0, S, [&](int s) { return slabs[((size_t)s * n3p + i) * n1p + k]; });
    out[e] = v;
  }
}

// out[k][i] (+)= sum_s slab[s][i][k] (out is n1 x n3): 16 x 16 tiles through LDS, coalesced on both sides
__global__ __launch_bounds__(256) void ens_reduce_trans_kernel(const c128* slabs, int S, int n3, int n1, int n3p,
                                                               int n1p, c128* out, int accumulate) {
  __shared__ c128 tile[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int k0 = blockIdx.x * 16, i0 = blockIdx.y * 16;
  {
    const int i = i0 + ty, k = k0 + tx;
    c128 v = cmk(0, 0);
    if (i < n3 && k < n1) v = slab_sum(v, 0, S, [&](int s) { return slabs[((size_t)s * n3p + i) * n1p + k]; });
    tile[ty][tx] = v;
  }
  __syncthreads();
  const int k = k0 + ty, i = i0 + tx;
  if (i < n3 && k < n1) {
    const size_t e = (size_t)k * n3 + i;
    const c128 v = tile[tx][ty];
    out[e] = accumulate ? cadd(out[e], v) : v;
  }
}

// out[j][i][k] (+)= sum_s slab[s][i][j*n1p + k]   (slab leading dimension ldz = n2*n1p), fixed order
__global__ void ens_reduce_t2_kernel(const c128* slabs, int S, int n2, int n3, int n1, int n3p, int n1p, c128* out,
                                     int accumulate) {
  const size_t tot = (size_t)n2 * n3 * n1;
  const size_t ldz = (size_t)n2 * n1p;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % n1);
    const int i = (int)((e / n1) % n3);
    const int j = (int)(e / ((size_t)n1 * n3));
    c128 v = accumulate ? out[e] : cmk(0, 0);
    v = slab_sum(v, 0, S, [&](int s) { return slabs[((size_t)s * n3p + i) * ldz + (size_t)j * n1p + k]; });
    out[e] = v;
  }
}

// ---- t2 scan without a per-t2 operand: with P_m = X_m B_m and Q_m = C_m Y_m,
//   S_j = sum_m P_m diag(e^{lam_m t2_j}) Q_m = P * diag(E_j) * Q,   E_j[(m,r)] = e^{lam_mr t2_j},
// so P [n3p][Kp] and Q [Kp][n1p] are built once per scan and the GEMM's B operand for waiting time j is
// Q with its rows scaled by E_j, formed in the staging step (one complex multiply per staged element).
// P block: MB = floor(256 / max(np, nr)) members; thread c < MB np computes x_{m p}(t) for (m, p) =
// (m0 + c / np, c % np), the X values of a 16-row group go through LDS, and output thread c < MB nr,
// (m, r) = (m0 + c / nr, c % nr), contracts its member's np values with B_m[:, r] (registers).
// np = nr = nL and lamp = lam in the unpruned form; the host passes the compact index sets otherwise.
__global__ __launch_bounds__(256) void ens_p_uniform_kernel(const c128* alpha, const c128* Bm, const c128* lamp, int M,
                                                            int np, int nr, double t0, double dt, int n3, int n3p,
                                                            int Kp, c128* P) {
  __shared__ c128 sX[16 * 256];
  const int MB = 256 / (np > nr ? np : nr);
  const int m0 = blockIdx.x * MB;
  const int c = threadIdx.x;
  // X part: x_{m p}(t) = i alpha_mp e^{lamp_mp t} for (m, p) = (m0 + c / np, c % np)
  const int mx = m0 + c / np, px = c % np;
  const bool xcol = c < MB * np && mx < M;
  const int kx = mx * np + px;
  const c128 l = xcol ? lamp[kx] : cmk(0, 0);
  const c128 a = xcol ? cmuli(alpha[kx]) : cmk(0, 0);
  // output column (m, r) = (m0 + c / nr, c % nr), P column kk = m nr + r
  const int m = m0 + c / nr, r = c % nr;
  const bool col = c < MB * nr && m < M;
  const int kk = m * nr + r;
  c128 T1[16];
  T1[0] = cmk(1, 0);
  const c128 st = cexp_t(l, dt);
#pragma unroll
  for (int j = 1; j < 16; ++j) T1[j] = cmul(T1[j - 1], st);
  c128 b[ZMAX];
#pragma unroll
  for (int p = 0; p < ZMAX; ++p) b[p] = (col && p < np) ? Bm[((size_t)m * np + p) * nr + r] : cmk(0, 0);
  const int mc0 = (c / nr) * np;             // first sX column of this output thread's member
  for (int g = 0; g < UNI_ROWS / 16; ++g) {
    const int ib = (int)blockIdx.y * UNI_ROWS + 16 * g;
    const c128 base = cmul(a, cexp_t(l, t0 + (double)ib * dt));
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) sX[j * 256 + c] = cmul(base, T1[j]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = ib + j;
      if (i >= n3p) break;
      c128 v = cmk(0, 0);
      if (col && i < n3) {
#pragma unroll
        for (int p = 0; p < ZMAX; ++p)
          if (p < np) v = cadd(v, cmul(sX[j * 256 + mc0 + p], b[p]));
      }
      if (col && kk < Kp) P[(size_t)i * Kp + kk] = v;
    }
  }
}

// columns K..Kp-1 of P are padding (the member blocks cover columns < K only)
__global__ void ens_p_pad_kernel(int K, int Kp, int n3p, c128* P) {
  const int w = Kp - K;
  const size_t tot = (size_t)n3p * w;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x)
    P[(e / w) * Kp + K + e % w] = cmk(0, 0);
}

// E [n2][Kp]: e^{lam_kk t2_j}, zero in the padding
__global__ void ens_e_kernel(const c128* lam, int K, int Kp, const double* t2, int n2, c128* E) {
  const size_t tot = (size_t)n2 * Kp;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int kk = (int)(e % Kp), j = (int)(e / Kp);
    E[e] = kk < K ? cexp_t(lam[kk], t2[j]) : cmk(0, 0);
  }
}

struct EnsQEB {
  struct Raw { cg_v2 q, e; };
  const c128* Q;
  const c128* Ej;   // E row of this column block's waiting time
  int n1p, col0, k0;
  __device__ __forceinline__ Raw fetch(int t, int e, int) const {
    const int row = k0 + t * CG_KT + e / ENS_BT;
    return Raw{cg_ld(Q + (size_t)row * n1p + col0 + (e % ENS_BT)), cg_ld(Ej + row)};
  }
  __device__ __forceinline__ cg_v2 finish(const Raw& r, int, int, int) const {
    const c128 v = cmul(cmk(r.e.x, r.e.y), cmk(r.q.x, r.q.y));
    return cg_v2{v.re, v.im};
  }
};

// grid: (n2 * n1p / BT) x (n3p / BT) x S; column block bn is waiting time (bn * BT) / n1p
__global__ __launch_bounds__(CG_WG) void ens_t2_gemm_kernel(const c128* P, int Kp, const c128* Q, int n1p,
                                                            const c128* E, int tiles, int S, c128* slabs, int n3p,
                                                            int ldz) {
  __shared__ CgLds<ENS_BT> L;
  int bn, bm, s;
  ens_tile(bn, bm, s);
  const int t0 = (int)((long)tiles * s / S), t1 = (int)((long)tiles * (s + 1) / S);
  const int j = (bn * ENS_BT) / n1p, colq = (bn * ENS_BT) % n1p;
  CgAcc<ENS_BT> A;
  c128* slab = slabs + (size_t)s * n3p * ldz;
  if (t1 > t0) {
    EnsXA pa{P, Kp, bm * ENS_BT, t0 * CG_KT};
    EnsQEB pb{Q, E + (size_t)j * Kp, n1p, colq, t0 * CG_KT};
    cg_block_gemm_gen<ENS_BT>(t1 - t0, pa, pb, L, A);
    cg_epilogue<ENS_BT>(A, [&](int row, int col, c128 v) {
      slab[(size_t)(bm * ENS_BT + row) * ldz + bn * ENS_BT + col] = v;
    });
  } else {
    for (int e = threadIdx.x; e < ENS_BT * ENS_BT; e += CG_WG)
      slab[(size_t)(bm * ENS_BT + e / ENS_BT) * ldz + bn * ENS_BT + e % ENS_BT] = cmk(0, 0);
  }
}

// ---- frequency-domain bilinear grids (DEOMSolver.correlation_4op_3t, heom/deom.py:1127-1209):
//   out[i][j] = sum_pq x_p(wx_i) M_pq z_q(wy_j),  x_p(w) = a_p / (-lam_p - i w),  z_q(w) = v_q / (-lam_q - i w)
// as two split-K MFMA GEMMs: W = M Z (n x n x ny), out = X W (nx x n x ny).
__device__ __forceinline__ c128 cdiv(c128 a, c128 b) {
  // Smith's algorithm (scaled, as numpy's complex division)
  if (fabs(b.re) >= fabs(b.im)) {
    const double r = b.im / b.re, d = b.re + b.im * r;
    return cmk((a.re + a.im * r) / d, (a.im - a.re * r) / d);
  }
  const double r = b.re / b.im, d = b.im + b.re * r;
  return cmk((a.re * r + a.im) / d, (a.im * r - a.re) / d);
}

// rows_w = 1: out[i][p] (ld = Kp) = coef_p / (-lam_p - i w_i) for i < nw, p < n, zero padding up to [rows][Kp]
// rows_w = 0: out[q][j] (ld = nwp) = coef_q / (-lam_q - i w_j), [Kp][nwp]
__global__ void resolvent_operand_kernel(const c128* coef, const c128* lam, int n, const double* w, int nw, int rows_w,
                                         int R, int C, c128* out) {
  const size_t tot = (size_t)R * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / C), c = (int)(e % C);
    const int iw = rows_w ? r : c, p = rows_w ? c : r;
    c128 v = cmk(0, 0);
    if (iw < nw && p < n) v = cdiv(coef[p], cmk(-lam[p].re, -lam[p].im - w[iw]));
    out[e] = v;
  }
}

// dst [R][C] = src [n][n] zero-padded
__global__ void pad_square_kernel(const c128* src, int n, int R, int C, c128* dst) {
  const size_t tot = (size_t)R * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / C), c = (int)(e % C);
    dst[e] = (r < n && c < n) ? src[(size_t)r * n + c] : cmk(0, 0);
  }
}

// out[i] = sum_n -c_n / (lam_n + i w_i)   (Lindblad_solver.correlation_*_1w, superoperator.py:603-700)
__global__ void resolvent_sum_kernel(const c128* c, const c128* lam, int n, const double* w, int nw, c128* out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
    c128 s = cmk(0, 0);
    for (int k = 0; k < n; ++k) {
      const c128 den = cmk(lam[k].re, lam[k].im + w[i]);
      const double d2 = den.re * den.re + den.im * den.im;
      const c128 inv = cmk(den.re / d2, -den.im / d2);
      s = csub(s, cmul(c[k], inv));
    }
    out[i] = s;
  }
}

int grid_for(size_t n, int threads) { return (int)std::min<size_t>((n + threads - 1) / threads, 16384); }

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_sos_propagator(const qd_c128* U1, const qd_c128* U2, const qd_c128* lam, int nL, const double* t,
                                 int nt, qd_c128* U, void* stream) {
  QD_CHECK_ARG(U1 && U2 && lam && t && U, "qd_sos_propagator: null pointer");
  QD_CHECK_ARG(nL >= 1 && nt >= 1, "qd_sos_propagator: nL=%d nt=%d must be >= 1", nL, nt);
  const size_t tot = (size_t)nL * nL * nt;
  hipLaunchKernelGGL(sos_propagator_kernel, dim3(grid_for(tot, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const c128*)U1, (const c128*)U2, (const c128*)lam, nL, t, nt, (c128*)U);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_response_cube(const qd_c128* alpha, const qd_c128* B, const qd_c128* C, const qd_c128* beta,
                                const qd_c128* lam, int nL, const double* t3, int n3, const double* t2, int n2,
                                const double* t1, int n1, qd_c128* out, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(alpha && B && C && beta && lam && t3 && t2 && t1 && out, "qd_response_cube: null pointer");
  QD_CHECK_ARG(nL >= 1 && nL <= 4096 && n3 >= 1 && n2 >= 1 && n1 >= 1, "qd_response_cube: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  void* w = nullptr;
  const size_t ny = (size_t)n1 * nL, nw = (size_t)n2 * nL * n1;
  int rc = workspace(WS_2DES, (ny + nw) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* Y = (c128*)w;
  c128* W = Y + ny;
  hipLaunchKernelGGL(cube_y_kernel, dim3(grid_for(ny, 256)), dim3(256), 0, st, (const c128*)C, (const c128*)beta,
                     (const c128*)lam, nL, t1, n1, Y);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(cube_w_kernel, dim3(grid_for(nw, 256)), dim3(256), 0, st, (const c128*)B, Y, (const c128*)lam,
                     nL, t2, n2, n1, W);
  QD_HIP(hipGetLastError());
  QD_CHECK_ARG((size_t)n3 * n2 < (1u << 31), "qd_response_cube: n3*n2 too large");
  hipLaunchKernelGGL(cube_out_kernel, dim3(n3 * n2), dim3(256), nL * sizeof(c128), st, (const c128*)alpha,
                     (const c128*)lam, W, nL, t3, n3, n2, n1, (c128*)out);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

namespace {
// Shared driver.  Time grids are either device arrays (t3 / t1) or uniform (t0 + j dt, when the
// array pointer is null): the uniform form builds the GEMM operands from exponential tables.
// nL / lam: the t3 (X, GEMM K) side; nz / lamz: the t1 side (Mt is [M][nL][nz]).  trans != 0 writes
// out[k][i] = S[i][k] (the host's swapped form, which puts the smaller pruned index set on K).
int ens_run(const char* fn, const qd_c128* alpha, const qd_c128* Mt, const qd_c128* beta, const qd_c128* lam, int M,
            int nL, const double* t3, double t3_0, double dt3, int n3, const double* t1, double t1_0, double dt1,
            int n1, qd_c128* out, int accumulate, void* stream, int nz = 0, const qd_c128* lamz_ = nullptr,
            int trans = 0) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  if (nz == 0) nz = nL;
  const c128* lamz = (const c128*)(lamz_ ? lamz_ : lam);
  QD_CHECK_ARG(alpha && Mt && beta && lam && out, "%s: null pointer", fn);
  QD_CHECK_ARG(M >= 1 && nL >= 1 && nz >= 1 && n3 >= 1 && n1 >= 1, "%s: bad sizes", fn);
  QD_CHECK_ARG((long)M * nL < (1L << 30) && M < 65536 * 1024, "%s: M*nL too large", fn);
  hipStream_t st = (hipStream_t)stream;
  const int BT = ENS_BT;
  const int n3p = ceil_div(n3, BT) * BT, n1p = ceil_div(n1, BT) * BT;
  const int K = M * nL;
  const int tiles = ceil_div(K, CG_KT);
  const int Kp = tiles * CG_KT;
  const SplitPlan plan = split_plan(n3p, n1p, tiles);
  const int S = plan.S;
  const size_t nXe = (size_t)n3p * Kp, nZe = (size_t)Kp * n1p, nsl = (size_t)S * n3p * n1p;
  void* w = nullptr;
  int rc = workspace(WS_2DES, (nXe + nZe + nsl) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* X = (c128*)w;
  c128* Z = X + nXe;
  c128* slabs = Z + nZe;
  const int zbx = n1p / 256 + (n1p % 256 != 0);
  const bool zfast = nL <= ZMAX && nz <= ZMAX && M <= 65535 - 4096;
  const int xbx = ceil_div(Kp, 256), xblocks = xbx * (n3p / XU_ROWS);
  // uniform t3: the A operand is generated in the GEMM staging from (n3p/16 + 16) x Kp tables held in
  // the X buffer (round 3)
  const bool xtab = !t3 && plan.bt == 128;  // 64-blocks are already load-bound in the staging
  c128* coarse = X;
  c128* fine = X + (size_t)(n3p / 16) * Kp;
  if (xtab) {
    hipLaunchKernelGGL(ens_xtab_kernel, dim3(xbx), dim3(256), 0, st, (const c128*)alpha, (const c128*)lam, K, Kp,
                       t3_0, dt3, n3, n3p, coarse, fine);
    QD_HIP(hipGetLastError());
  }
  const int G = z_group(nL, nz, n1p, M);
  const int nMB = ceil_div(M, G);
  if (!t1 && nL <= ZMAX && nz <= ZMAX && n1p <= 16 * UNI_MAXC && (long)nMB + xblocks <= 65535) {
    // Z (uniform t1), G members per block; a materialised uniform X (when not generated in the GEMM) in
    // the same launch
    const bool xin = !t3 && !xtab;
    hipLaunchKernelGGL(ens_z_uniform_kernel, dim3(zbx, nMB + (xin ? xblocks : 0)), dim3(256),
                       z_lds(G, nL, nz, n1p), st, (const c128*)Mt, (const c128*)beta, lamz, M, nL, nz, G, t1_0,
                       dt1, n1, n1p, Z, (const c128*)alpha, (const c128*)lam, K, Kp, t3_0, dt3, n3, n3p, xbx, X);
    QD_HIP(hipGetLastError());
    if (Kp > K) {
      hipLaunchKernelGGL(ens_z_pad_kernel, dim3(64), dim3(256), 0, st, K, Kp, n1p, Z);
      QD_HIP(hipGetLastError());
    }
    if (t3) {  // X from the array (X part of the combined kernel only)
      hipLaunchKernelGGL(ens_xz_kernel, dim3(zbx, 4096), dim3(256), 0, st, (const c128*)Mt, (const c128*)beta,
                         (const c128*)lam, 0, nL, t1, n1, n1p, Kp, Z, (const c128*)alpha, t3, n3, n3p, 4096, K, X, nz, lamz);
      QD_HIP(hipGetLastError());
    }
  } else {
    QD_CHECK_ARG(t1, "%s: uniform t1 needs nL <= %d and n1 <= %d", fn, ZMAX, 16 * UNI_MAXC);
    if (!t3 && !xtab) {  // uniform t3 with an array t1: X blocks only
      hipLaunchKernelGGL(ens_xz_uniform_kernel, dim3(1, xblocks), dim3(256), 0, st, (const c128*)Mt,
                         (const c128*)beta, (const c128*)lam, 0, nL, 0.0, 0.0, n1, n1p, Kp, Z, (const c128*)alpha, K,
                         t3_0, dt3, n3, n3p, xbx, X, nz, lamz);
      QD_HIP(hipGetLastError());
    }
    if (zfast) {
      // X (when from an array) gets as many block rows as Z has (capped): one launch, both writes
      const int xrows = t3 ? std::max(1, std::min(M, 4096)) : 0;
      hipLaunchKernelGGL(ens_xz_kernel, dim3(zbx, M + xrows), dim3(256), 0, st, (const c128*)Mt, (const c128*)beta,
                         (const c128*)lam, M, nL, t1, n1, n1p, Kp, Z, (const c128*)alpha, t3, n3, n3p, xrows, K, X, nz, lamz);
      QD_HIP(hipGetLastError());
      if (Kp > K) {
        hipLaunchKernelGGL(ens_z_pad_kernel, dim3(64), dim3(256), 0, st, K, Kp, n1p, Z);
        QD_HIP(hipGetLastError());
      }
    } else {
      if (t3) {
        hipLaunchKernelGGL(ens_xz_kernel, dim3(zbx, 4096), dim3(256), 0, st, (const c128*)Mt, (const c128*)beta,
                           (const c128*)lam, 0, nL, t1, n1, n1p, Kp, Z, (const c128*)alpha, t3, n3, n3p, 4096, K, X, nz, lamz);
        QD_HIP(hipGetLastError());
      }
      hipLaunchKernelGGL(ens_z_generic_kernel, dim3(grid_for(nZe, 256)), dim3(256), 0, st, (const c128*)Mt,
                         (const c128*)beta, lamz, M, nL, t1, n1, n1p, Kp, Z, nz);
      QD_HIP(hipGetLastError());
    }
  }
  launch_ens_gemm(plan, X, Kp, Z, n3p, n1p, tiles, slabs, st, xtab ? fine : nullptr);
  QD_HIP(hipGetLastError());
  if (trans)
    hipLaunchKernelGGL(ens_reduce_trans_kernel, dim3(ceil_div(n1, 16), ceil_div(n3, 16)), dim3(256), 0, st, slabs, S,
                       n3, n1, n3p, n1p, (c128*)out, accumulate);
  else
    hipLaunchKernelGGL(ens_reduce_kernel, dim3(grid_for((size_t)n3 * n1, 256)), dim3(256), 0, st, slabs, S, n3, n1,
                       n3p, n1p, (c128*)out, accumulate);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
}  // namespace

extern "C" int qd_response2d_ensemble(const qd_c128* alpha, const qd_c128* Mt, const qd_c128* beta,
                                      const qd_c128* lam, int M, int nL, const double* t3, int n3, const double* t1,
                                      int n1, qd_c128* out, int accumulate, void* stream) {
  QD_CHECK_ARG(t3 && t1, "qd_response2d_ensemble: null time grid");
  return ens_run("qd_response2d_ensemble", alpha, Mt, beta, lam, M, nL, t3, 0, 0, n3, t1, 0, 0, n1, out, accumulate,
                 stream);
}

extern "C" int qd_response2d_ensemble_uniform(const qd_c128* alpha, const qd_c128* Mt, const qd_c128* beta,
                                              const qd_c128* lam, int M, int nL, double t3_0, double dt3, int n3,
                                              double t1_0, double dt1, int n1, qd_c128* out, int accumulate,
                                              void* stream) {
  QD_CHECK_ARG(nL <= ZMAX && n1 <= 16 * UNI_MAXC, "qd_response2d_ensemble_uniform: nL=%d (<= %d), n1=%d (<= %d)", nL,
               ZMAX, n1, 16 * UNI_MAXC);
  return ens_run("qd_response2d_ensemble_uniform", alpha, Mt, beta, lam, M, nL, nullptr, t3_0, dt3, n3, nullptr, t1_0,
                 dt1, n1, out, accumulate, stream);
}

extern "C" int qd_response2d_ensemble_rect(const qd_c128* alpha, const qd_c128* lamx, int nx, const qd_c128* Mt,
                                           const qd_c128* beta, const qd_c128* lamz, int nz, int M, const double* t3,
                                           double t3_0, double dt3, int n3, const double* t1, double t1_0, double dt1,
                                           int n1, int transpose_out, qd_c128* out, int accumulate, void* stream) {
  QD_CHECK_ARG(lamz, "qd_response2d_ensemble_rect: null pointer");
  QD_CHECK_ARG(t1 || (nz <= ZMAX && nx <= ZMAX && n1 <= 16 * UNI_MAXC),
               "qd_response2d_ensemble_rect: uniform t1 needs nx, nz <= %d and n1 <= %d", ZMAX, 16 * UNI_MAXC);
  return ens_run("qd_response2d_ensemble_rect", alpha, Mt, beta, lamx, M, nx, t3, t3_0, dt3, n3, t1, t1_0, dt1, n1, out,
                 accumulate, stream, nz, lamz, transpose_out ? 1 : 0);
}

namespace {
struct T2Dims {
  int n3p, n1p, K, Kp, tiles;
};
T2Dims t2_dims(int M, int nL, int n3, int n1) {
  T2Dims d;
  d.n3p = ceil_div(n3, ENS_BT) * ENS_BT;
  d.n1p = ceil_div(n1, ENS_BT) * ENS_BT;
  d.K = M * nL;
  d.tiles = ceil_div(d.K, CG_KT);
  d.Kp = d.tiles * CG_KT;
  return d;
}
}  // namespace

extern "C" int qd_response2d_t2_dims(int M, int nL, int n3, int n1, int* n3p, int* n1p, int* Kp) {
  QD_CHECK_ARG(n3p && n1p && Kp, "qd_response2d_t2_dims: null pointer");
  QD_CHECK_ARG(M >= 1 && nL >= 1 && n3 >= 1 && n1 >= 1, "qd_response2d_t2_dims: bad sizes");
  const T2Dims d = t2_dims(M, nL, n3, n1);
  *n3p = d.n3p;
  *n1p = d.n1p;
  *Kp = d.Kp;
  return QD_OK;
}

extern "C" int qd_response2d_t2_operands_rect(const qd_c128* alpha, const qd_c128* lamp, int np,
                                              const qd_c128* Bm, const qd_c128* lamr, int nr, const qd_c128* Cm,
                                              const qd_c128* beta, const qd_c128* lamq, int nq, int M, double t3_0,
                                              double dt3, int n3, double t1_0, double dt1, int n1, qd_c128* P_,
                                              qd_c128* Q_, void* stream) {
  const char* fn = "qd_response2d_t2_operands_rect";
  QD_CHECK_ARG(alpha && lamp && Bm && lamr && Cm && beta && lamq && P_ && Q_, "%s: null pointer", fn);
  QD_CHECK_ARG(M >= 1 && np >= 1 && nr >= 1 && nq >= 1 && n3 >= 1 && n1 >= 1, "%s: bad sizes", fn);
  QD_CHECK_ARG(np <= ZMAX && nr <= ZMAX && nq <= ZMAX && n1 <= 16 * UNI_MAXC,
               "%s: np=%d nr=%d nq=%d (<= %d), n1=%d (<= %d)", fn, np, nr, nq, ZMAX, n1, 16 * UNI_MAXC);
  QD_CHECK_ARG((long)M * nr < (1L << 30), "%s: M=%d too large", fn, M);
  hipStream_t st = (hipStream_t)stream;
  const T2Dims d = t2_dims(M, nr, n3, n1);
  // the Z-build grid's y extent is the number of member groups (<= 65535)
  QD_CHECK_ARG(ceil_div(M, z_group(nr, nq, d.n1p, M)) <= 65535, "%s: M=%d too large", fn, M);
  c128* P = (c128*)P_;
  c128* Q = (c128*)Q_;
  const int MB = 256 / std::max(np, nr);
  hipLaunchKernelGGL(ens_p_uniform_kernel, dim3(ceil_div(M, MB), d.n3p / UNI_ROWS), dim3(256), 0, st,
                     (const c128*)alpha, (const c128*)Bm, (const c128*)lamp, M, np, nr, t3_0, dt3, n3, d.n3p, d.Kp, P);
  QD_HIP(hipGetLastError());
  if (d.Kp > d.K) {
    hipLaunchKernelGGL(ens_p_pad_kernel, dim3(64), dim3(256), 0, st, d.K, d.Kp, d.n3p, P);
    QD_HIP(hipGetLastError());
  }
  // Q = C_m Y_m: the uniform Z build with Mt := C [M][nr][nq] (Z rows only)
  const int G = z_group(nr, nq, d.n1p, M);
  hipLaunchKernelGGL(ens_z_uniform_kernel, dim3(ceil_div(d.n1p, 256), ceil_div(M, G)), dim3(256),
                     z_lds(G, nr, nq, d.n1p), st, (const c128*)Cm,
                     (const c128*)beta, (const c128*)lamq, M, nr, nq, G, t1_0, dt1, n1, d.n1p, Q, (const c128*)nullptr,
                     (const c128*)nullptr, d.K, d.Kp, 0.0, 0.0, n3, d.n3p, 1, (c128*)nullptr);
  QD_HIP(hipGetLastError());
  if (d.Kp > d.K) {
    hipLaunchKernelGGL(ens_z_pad_kernel, dim3(64), dim3(256), 0, st, d.K, d.Kp, d.n1p, Q);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}

extern "C" int qd_response2d_t2_operands(const qd_c128* alpha, const qd_c128* Bm, const qd_c128* Cm,
                                         const qd_c128* beta, const qd_c128* lam, int M, int nL, double t3_0,
                                         double dt3, int n3, double t1_0, double dt1, int n1, qd_c128* P_,
                                         qd_c128* Q_, void* stream) {
  return qd_response2d_t2_operands_rect(alpha, lam, nL, Bm, lam, nL, Cm, beta, lam, nL, M, t3_0, dt3, n3, t1_0, dt1,
                                        n1, P_, Q_, stream);
}

extern "C" int qd_response2d_t2_apply(const qd_c128* P, const qd_c128* Q, const qd_c128* lam, int M, int nL, int n3,
                                      int n1, const double* t2, int n2, qd_c128* out, int accumulate, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  const char* fn = "qd_response2d_t2_apply";
  QD_CHECK_ARG(P && Q && lam && t2 && out, "%s: null pointer", fn);
  QD_CHECK_ARG(M >= 1 && nL >= 1 && n3 >= 1 && n1 >= 1 && n2 >= 1 && n2 <= 65535, "%s: bad sizes", fn);
  hipStream_t st = (hipStream_t)stream;
  const T2Dims d = t2_dims(M, nL, n3, n1);
  const long ldz = (long)n2 * d.n1p;
  QD_CHECK_ARG(ldz / ENS_BT <= 65535, "%s: n2*n1 too large", fn);
  const int blocks2d = (int)((d.n3p / ENS_BT) * (ldz / ENS_BT));
  const int S = std::max(1, std::min(ceil_div(256, blocks2d), std::max(1, d.tiles / 4)));
  const size_t nE = (size_t)n2 * d.Kp, nsl = (size_t)S * d.n3p * ldz;
  void* w = nullptr;
  int rc = workspace(WS_2DES, (nE + nsl) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* E = (c128*)w;
  c128* slabs = E + nE;
  hipLaunchKernelGGL(ens_e_kernel, dim3(grid_for(nE, 256)), dim3(256), 0, st, (const c128*)lam, d.K, d.Kp, t2, n2, E);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(ens_t2_gemm_kernel, dim3((int)(ldz / ENS_BT), d.n3p / ENS_BT, S), dim3(CG_WG), 0, st,
                     (const c128*)P, d.Kp, (const c128*)Q, d.n1p, (const c128*)E, d.tiles, S, slabs, d.n3p, (int)ldz);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(ens_reduce_t2_kernel, dim3(grid_for((size_t)n2 * n3 * n1, 256)), dim3(256), 0, st, slabs, S, n2,
                     n3, n1, d.n3p, d.n1p, (c128*)out, accumulate);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_response2d_t2scan(const qd_c128* alpha, const qd_c128* Bm, const qd_c128* Cm, const qd_c128* beta,
                                    const qd_c128* lam, int M, int nL, double t3_0, double dt3, int n3,
                                    const double* t2, int n2, double t1_0, double dt1, int n1, qd_c128* out,
                                    int accumulate, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  const char* fn = "qd_response2d_t2scan";
  QD_CHECK_ARG(alpha && Bm && Cm && beta && lam && t2 && out, "%s: null pointer", fn);
  QD_CHECK_ARG(M >= 1 && nL >= 1 && n3 >= 1 && n1 >= 1 && n2 >= 1, "%s: bad sizes", fn);
  const T2Dims d = t2_dims(M, nL, n3, n1);
  void* w = nullptr;
  int rc = workspace(WS_2DES_OPS, ((size_t)d.n3p * d.Kp + (size_t)d.Kp * d.n1p) * sizeof(c128), &w, (hipStream_t)stream);
  if (rc) return rc;
  qd_c128* P = (qd_c128*)w;
  qd_c128* Q = P + (size_t)d.n3p * d.Kp;
  if ((rc = qd_response2d_t2_operands(alpha, Bm, Cm, beta, lam, M, nL, t3_0, dt3, n3, t1_0, dt1, n1, P, Q, stream)))
    return rc;
  return qd_response2d_t2_apply(P, Q, lam, M, nL, n3, n1, t2, n2, out, accumulate, stream);
}

namespace {
// C[m][k] (m < Mo, k < No, leading dimension No) = A [Mp][Kp] * B [Kp][Np]; padded operands, split-K MFMA GEMM
int splitk_gemm(const c128* A, const c128* B, int Mp, int Kp, int Np, int Mo, int No, c128* C, c128* slabs, int S,
                hipStream_t st) {
  const int tiles = Kp / CG_KT;
  launch_ens_gemm(SplitPlan{ENS_BT, S}, A, Kp, B, Mp, Np, tiles, slabs, st);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(ens_reduce_kernel, dim3(grid_for((size_t)Mo * No, 256)), dim3(256), 0, st, slabs, S, Mo, No, Mp,
                     Np, C, 0);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
int splits_for(int Mp, int Np, int Kp) {
  const int blocks = (Mp / ENS_BT) * (Np / ENS_BT), tiles = Kp / CG_KT;
  return std::max(1, std::min(ceil_div(256, blocks), std::max(1, tiles / 4)));
}
}  // namespace

// Split-K complex GEMM for other translation units (TDSE batches): partial products of A [Mp][Kp] * B [Kp][Np]
// (row-major, Mp and Np multiples of 128, Kp of 16) into S slabs [S][Mp][Np]; S is returned through *S_out
// (<= max_S).  The caller sums the slabs in order s = 0 .. S-1.
int qd::cgemm_splitk_slabs(const c128* A, const c128* B, int Mp, int Kp, int Np, c128* slabs, int max_S, int* S_out,
                           hipStream_t st) {
  QD_CHECK_ARG(Mp % 128 == 0 && Np % 64 == 0 && Kp % CG_KT == 0, "cgemm_splitk_slabs: bad padding");
  const int tiles = Kp / CG_KT;
  SplitPlan pl;
  if (Np % 128 == 0) {
    pl = split_plan(Mp, Np, tiles);
  } else {  // 64-wide column blocks (skinny B, e.g. a batch of <= 64 vectors): >= 512 workgroups, >= 8 K-tiles each
    const int blocks = (Mp / 64) * (Np / 64);
    pl = {64, std::max(1, std::min(ceil_div(512, blocks), std::max(1, tiles / 8)))};
  }
  pl.S = std::min(pl.S, max_S);
  launch_ens_gemm(pl, A, Kp, B, Mp, Np, Kp / CG_KT, slabs, st);
  QD_HIP(hipGetLastError());
  *S_out = pl.S;
  return QD_OK;
}

extern "C" int qd_resolvent_grid2d(const qd_c128* a, const qd_c128* M, const qd_c128* v, const qd_c128* lam, int n,
                                   const double* wx, int nx, const double* wy, int ny, qd_c128* out, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  const char* fn = "qd_resolvent_grid2d";
  QD_CHECK_ARG(a && M && v && lam && wx && wy && out, "%s: null pointer", fn);
  QD_CHECK_ARG(n >= 1 && nx >= 1 && ny >= 1 && n <= 65536 && nx <= 65536 && ny <= 65536, "%s: bad sizes", fn);
  hipStream_t st = (hipStream_t)stream;
  const int BT = ENS_BT;
  const int np_ = ceil_div(n, BT) * BT;  // n as a row / column block dimension and as K (multiple of 16 too)
  const int nxp = ceil_div(nx, BT) * BT, nyp = ceil_div(ny, BT) * BT;
  const int S1 = splits_for(np_, nyp, np_), S2 = splits_for(nxp, nyp, np_);
  const size_t nM = (size_t)np_ * np_, nZ = (size_t)np_ * nyp, nW = (size_t)np_ * nyp, nX = (size_t)nxp * np_;
  const size_t nsl = std::max((size_t)S1 * np_ * nyp, (size_t)S2 * nxp * nyp);
  void* w = nullptr;
  int rc = workspace(WS_2DES, (nM + nZ + nW + nX + nsl) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* Mp = (c128*)w;
  c128* Z = Mp + nM;
  c128* W = Z + nZ;
  c128* X = W + nW;
  c128* slabs = X + nX;
  hipLaunchKernelGGL(pad_square_kernel, dim3(grid_for(nM, 256)), dim3(256), 0, st, (const c128*)M, n, np_, np_, Mp);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(resolvent_operand_kernel, dim3(grid_for(nZ, 256)), dim3(256), 0, st, (const c128*)v,
                     (const c128*)lam, n, wy, ny, 0, np_, nyp, Z);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(resolvent_operand_kernel, dim3(grid_for(nX, 256)), dim3(256), 0, st, (const c128*)a,
                     (const c128*)lam, n, wx, nx, 1, nxp, np_, X);
  QD_HIP(hipGetLastError());
  if ((rc = splitk_gemm(Mp, Z, np_, np_, nyp, np_, nyp, W, slabs, S1, st))) return rc;      // W = M Z (padded)
  return splitk_gemm(X, W, nxp, np_, nyp, nx, ny, (c128*)out, slabs, S2, st);              // out = X W
}

extern "C" int qd_resolvent_sum(const qd_c128* coeff, const qd_c128* lam, int n, const double* w, int nw,
                                qd_c128* out, void* stream) {
  QD_CHECK_ARG(coeff && lam && w && out, "qd_resolvent_sum: null pointer");
  QD_CHECK_ARG(n >= 1 && nw >= 1, "qd_resolvent_sum: bad sizes");
  hipLaunchKernelGGL(resolvent_sum_kernel, dim3(grid_for(nw, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const c128*)coeff, (const c128*)lam, n, w, nw, (c128*)out);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
