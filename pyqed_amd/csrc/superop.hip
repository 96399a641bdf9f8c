// superop.hip — RK4 with a dense Liouville-space generator: d v/dt = L v.
//
// Replaces the csr GEMV loop of pyqed/oqs.py:436-459 (_redfield: rho = rk4(rho,
// rhs, dt, R), rhs = R.dot(rho), oqs.py:462-463) for an arbitrary dense
// superoperator (user-supplied R, Lindblad_solver.liouvillian(), ...).
// HBM-bound for small batches: every stage streams L once per group of <= 8 vectors (16 N2^2 bytes), the RK4
// bookkeeping fused into the row epilogue; MFMA-bound GEMM stages for batches >= 48 (L once per stage).
#include "qd_common.hpp"

namespace qd {
namespace {

constexpr int SO_TPB = 256;

typedef double d2v __attribute__((ext_vector_type(2)));

// One RK4 stage for NB state vectors, VALU GEMV path (small batches).  Each wave owns R consecutive rows of L and
// streams them once with 16-B lane-contiguous loads (1 KB per wave instruction, nontemporal: L is read once per
// stage and must not evict x); each x chunk it loads is reused for its R rows, so x's L2 traffic is 1/R of L's.
// U column chunks per iteration keep R*U independent 16-B loads of L in flight per lane.  A butterfly finishes
// the R*NB row sums; lane t < R*NB runs the fused RK4 bookkeeping of (row t / NB, vector t % NB).
template <int NB, int R, int U>
__global__ __launch_bounds__(SO_TPB) void superop_rows_kernel(const c128* __restrict__ L, int N2,
                                                              const c128* __restrict__ xin, c128* xout, c128* acc,
                                                              c128* v, int vstride, int stage, double dt) {
  const int lane = threadIdx.x & 63;
  const long r0 = ((blockIdx.x * (long)SO_TPB + threadIdx.x) >> 6) * R;
  if (r0 >= N2) return;
  double sr[R][NB], si[R][NB];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) sr[r][b] = si[r][b] = 0.0;
  const d2v* Lrow[R];
#pragma unroll
  for (int r = 0; r < R; ++r) Lrow[r] = (const d2v*)(L + std::min<long>(r0 + r, N2 - 1) * (long)N2);
  for (int j0 = 0; j0 < N2; j0 += 64 * U) {
    d2v l[R][U];
    c128 x[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + lane + 64 * u;
      const bool in = j < N2;
#pragma unroll
      for (int r = 0; r < R; ++r) l[r][u] = in ? __builtin_nontemporal_load(Lrow[r] + j) : d2v{0.0, 0.0};
#pragma unroll
      for (int b = 0; b < NB; ++b) x[b][u] = in ? xin[(long)b * vstride + j] : cmk(0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          sr[r][b] = fma(l[r][u].x, x[b][u].re, fma(-l[r][u].y, x[b][u].im, sr[r][b]));
          si[r][b] = fma(l[r][u].x, x[b][u].im, fma(l[r][u].y, x[b][u].re, si[r][b]));
        }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        sr[r][b] += __shfl_xor(sr[r][b], off, 64);
        si[r][b] += __shfl_xor(si[r][b], off, 64);
      }
  if (lane < R * NB) {
    double kr = 0, ki = 0;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (r * NB + b == lane) {
          kr = sr[r][b];
          ki = si[r][b];
        }
    const int r = lane / NB, b = lane % NB;
    const long row = r0 + r;
    if (row < N2) {
      const c128 k = cmk(kr, ki);
      const long idx = (long)b * vstride + row;
      // Horner-form RK4 (rk4_horner_coef): L is constant over the step; no accumulator
      (stage == 3 ? v : xout)[idx] = cadd(v[idx], cscale(k, rk4_horner_coef(dt, stage)));
    }
  }
}

// GEMM path state layout: X [N2p][Bp] (vector index fastest), zero padding.  dir 0: pack v [B][N2] -> X;
// dir 1: unpack X -> v.
__global__ void superop_pack_kernel(c128* v, int B, int N2, int Bp, int N2p, c128* X, int dir) {
  const size_t tot = (size_t)N2p * Bp;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / Bp), b = (int)(e % Bp);
    const bool in = b < B && r < N2;
    if (dir == 0) X[e] = in ? v[(size_t)b * N2 + r] : cmk(0, 0);
    else if (in) v[(size_t)b * N2 + r] = X[e];
  }
}

// L [N2][N2] -> Lp [N2p][N2p] zero-padded (GEMM path when N2 is not a multiple of 128)
__global__ void superop_pad_l_kernel(const c128* L, int N2, int N2p, c128* Lp) {
  const size_t tot = (size_t)N2p * N2p;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / N2p), c = (int)(e % N2p);
    Lp[e] = (r < N2 && c < N2) ? L[(size_t)r * N2 + c] : cmk(0, 0);
  }
}

// k = sum_s slabs[s] (fixed order: deterministic), then the Horner-form RK4 update of every element (rk4_horner_coef)
__global__ void superop_gemm_rk4_kernel(const c128* slabs, int S, size_t tot, c128* X, c128* x0, c128* x1, c128* acc,
                                        double dt, int stage) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    c128 k = slabs[e];
    k = slab_sum(k, 1, S, [&](int q) { return slabs[(size_t)q * tot + e]; });
    // Horner-form RK4: stage 0 -> x0, 1 -> x1, 2 -> x0, 3 -> X
    (stage == 3 ? X : (stage & 1) ? x1 : x0)[e] = cadd(X[e], cscale(k, rk4_horner_coef(dt, stage)));
  }
}

// Dense superoperator of the generalised Lindblad form d rho/dt = P rho + rho Q + sum_c L_c rho R_c acting on
// row-major vec(rho) (superoperator.py:29-58, 200-270 conventions: left kron(A, I), right kron(I, A^T)):
//   Lsup[(a,b),(c,d)] = P[a][c] d_bd + d_ac Q[d][b] + sum_c L_c[a][c] R_c[d][b].
// Lindblad: P = -i(H - (i/2) S), Q = iH - S/2, L_c = C_c, R_c = C_c^+ (oqs.liouvillian, oqs.py:697-714).
__global__ void superop_from_glf_kernel(const c128* P, const c128* Q, const c128* Lop, const c128* Rop, int nc, int N,
                                        c128* out) {
  const size_t N2 = (size_t)N * N, tot = N2 * N2;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const size_t row = e / N2, col = e % N2;
    const int a = (int)(row / N), b = (int)(row % N), c = (int)(col / N), d = (int)(col % N);
    c128 v = cmk(0, 0);
    if (b == d) v = cadd(v, P[(size_t)a * N + c]);
    if (a == c) v = cadd(v, Q[(size_t)d * N + b]);
    for (int k = 0; k < nc; ++k)
      v = cadd(v, cmul(Lop[(size_t)k * N2 + (size_t)a * N + c], Rop[(size_t)k * N2 + (size_t)d * N + b]));
    out[e] = v;
  }
}

// P = -i(H - (i/2) S), Q = iH - S/2, R_c = C_c^+, S = sum_c C_c^+ C_c (one thread per element, N^3 nc work)
__global__ void lindblad_glf_ops_kernel(const c128* H, const c128* C, int nc, int N, c128* P, c128* Q, c128* Rd) {
  const size_t NN = (size_t)N * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < NN; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / N), j = (int)(e % N);
    c128 s = cmk(0, 0);
    for (int c = 0; c < nc; ++c) {
      const c128* Cc = C + (size_t)c * NN;
      for (int k = 0; k < N; ++k) s = cadd(s, cmul(cconj(Cc[(size_t)k * N + i]), Cc[(size_t)k * N + j]));
      Rd[(size_t)c * NN + e] = cconj(Cc[(size_t)j * N + i]);
    }
    const c128 h = H[e];
    P[e] = cmulmi(csub(h, cmuli(cscale(s, 0.5))));
    Q[e] = csub(cmuli(h), cscale(s, 0.5));
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

namespace {
// VALU GEMV stage for a group of nb <= 8 vectors (rows per wave R and column unroll U sized so that the loads of
// L in flight per lane stay ~16 and the registers under 128)
int launch_rows(int nb, const c128* L, int N2, const c128* xin, c128* xo, c128* acc, c128* v, int vstride, int stage,
                double dt, hipStream_t st) {
  auto go = [&](auto kern, int R) {
    const long waves = (N2 + R - 1) / R;
    const int grid = (int)((waves * 64 + SO_TPB - 1) / SO_TPB);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(SO_TPB), 0, st, L, N2, xin, xo, acc, v, vstride, stage, dt);
  };
  switch (nb) {
    case 1: go(superop_rows_kernel<1, 4, 4>, 4); break;
    case 2: go(superop_rows_kernel<2, 4, 4>, 4); break;
    case 3: go(superop_rows_kernel<3, 2, 4>, 2); break;
    case 4: go(superop_rows_kernel<4, 2, 4>, 2); break;
    case 5: go(superop_rows_kernel<5, 2, 2>, 2); break;
    case 6: go(superop_rows_kernel<6, 2, 2>, 2); break;
    case 7: go(superop_rows_kernel<7, 2, 2>, 2); break;
    default: go(superop_rows_kernel<8, 2, 2>, 2); break;
  }
  QD_HIP(hipGetLastError());
  return QD_OK;
}
}  // namespace

// Batches of >= QD_SUPEROP_GEMM_MIN vectors (default 48) run each stage as one complex-fp64 MFMA GEMM,
// K[N2p][Bp] = L[N2p][N2p] X[N2p][Bp], on the split-K block engine (cgemm_splitk_slabs, 64- or 128-wide column
// blocks), then one elementwise kernel sums the slabs in fixed order and does the RK4 update.  L is streamed once
// per stage for the whole batch; below the threshold the VALU GEMV streams L once per group of <= 8 vectors.
extern "C" int qd_superop_rk4(const qd_c128* L_, qd_c128* v_, int B, int N2, double dt, int nsteps, const qd_c128* W_,
                              int ne, qd_c128* obs_, qd_c128* snap_, int save_every, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(L_ && v_, "qd_superop_rk4: null pointer");
  QD_CHECK_ARG(B >= 1 && N2 >= 1 && nsteps >= 0, "qd_superop_rk4: bad sizes B=%d N2=%d", B, N2);
  QD_CHECK_ARG(ne == 0 || (W_ && obs_), "qd_superop_rk4: W/obs null but ne=%d", ne);
  hipStream_t st = (hipStream_t)stream;
  const c128* L = (const c128*)L_;
  c128* v = (c128*)v_;
  const c128* W = (const c128*)W_;
  c128* obs = (c128*)obs_;
  c128* snap = (c128*)snap_;
  const int nsnap = save_every > 0 ? nsteps / save_every : 0;
  const int nrec = nsteps + 1;
  auto record = [&](int step) -> int {   // observables / snapshot of v [B][N2] after `step` steps
    const bool take = snap && save_every > 0 && step > 0 && (step % save_every == 0);
    if (ne || take) {
      hipLaunchKernelGGL(superop_obs_kernel, dim3(std::max(1, std::min(ne, 64)), B), dim3(SO_TPB), 0, st, v, N2, W,
                         ne, obs, step, nrec, take ? snap : nullptr, take ? step / save_every - 1 : 0, nsnap);
      QD_HIP(hipGetLastError());
    }
    return QD_OK;
  };
  int rc;
  if (ne && (rc = record(0))) return rc;
  // from 48 vectors the stages are MFMA GEMMs (one pass over L for the batch), below that GEMVs
  note_path(B >= 48 && N2 >= 64 ? "superop_gemm" : "superop_gemv");
  if (B >= 48 && N2 >= 64) {
    const int N2p = ceil_div(N2, 128) * 128;
    const int Bp = B <= 64 ? 64 : ceil_div(B, 128) * 128;
    constexpr int MAXS = 8;
    const size_t BN = (size_t)N2p * Bp;
    const bool padL = N2p != N2;
    void* w = nullptr;
    rc = workspace(WS_SUPEROP, (4 * BN + (size_t)MAXS * BN + (padL ? (size_t)N2p * N2p : 0)) * sizeof(c128), &w, st);
    if (rc) return rc;
    c128* X = (c128*)w;
    c128* x0 = X + BN;
    c128* x1 = x0 + BN;
    c128* acc = x1 + BN;
    c128* slabs = acc + BN;
    const c128* A = L;
    if (padL) {
      c128* Lp = slabs + (size_t)MAXS * BN;
      hipLaunchKernelGGL(superop_pad_l_kernel, dim3(8192), dim3(256), 0, st, L, N2, N2p, Lp);
      QD_HIP(hipGetLastError());
      A = Lp;
    }
    const int g2 = (int)std::min<size_t>((BN + 255) / 256, 8192);
    hipLaunchKernelGGL(superop_pack_kernel, dim3(g2), dim3(256), 0, st, v, B, N2, Bp, N2p, X, 0);
    QD_HIP(hipGetLastError());
    for (int s = 0; s < nsteps; ++s) {
      for (int stage = 0; stage < 4; ++stage) {
        const c128* xin = stage == 0 ? X : ((stage & 1) ? x0 : x1);   // stage 1: x0, 2: x1, 3: x0
        int S = 1;
        if ((rc = cgemm_splitk_slabs(A, xin, N2p, N2p, Bp, slabs, MAXS, &S, st))) return rc;
        hipLaunchKernelGGL(superop_gemm_rk4_kernel, dim3(g2), dim3(256), 0, st, (const c128*)slabs, S, BN, X, x0, x1,
                           acc, dt, stage);
        QD_HIP(hipGetLastError());
      }
      const bool take = snap && save_every > 0 && ((s + 1) % save_every == 0);
      if (ne || take || s + 1 == nsteps) {
        hipLaunchKernelGGL(superop_pack_kernel, dim3(g2), dim3(256), 0, st, v, B, N2, Bp, N2p, X, 1);
        QD_HIP(hipGetLastError());
        if ((rc = record(s + 1))) return rc;
      }
    }
    return QD_OK;
  }
  const size_t tot = (size_t)B * N2;
  void* w = nullptr;
  rc = workspace(WS_SUPEROP, 3 * tot * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* acc = (c128*)w;
  c128* xs[2] = {acc + tot, acc + 2 * tot};
  constexpr int GROUP = 8;
  for (int s = 0; s < nsteps; ++s) {
    for (int stage = 0; stage < 4; ++stage) {
      for (int b0 = 0; b0 < B; b0 += GROUP) {
        const int nb = std::min(GROUP, B - b0);
        const long off = (long)b0 * N2;
        const c128* xin = stage == 0 ? v + off : xs[(stage - 1) & 1] + off;
        if ((rc = launch_rows(nb, L, N2, xin, xs[stage & 1] + off, acc + off, v + off, N2, stage, dt, st))) return rc;
      }
    }
    if ((rc = record(s + 1))) return rc;
  }
  return QD_OK;
}

// Dense Liouville-space generator of a GLF operator set (see superop_from_glf_kernel), [N^2][N^2] into `out`.
extern "C" int qd_superop_from_glf(const qd_c128* P, const qd_c128* Q, const qd_c128* Lops, const qd_c128* Rops, int nc,
                                   int N, qd_c128* out, void* stream) {
  QD_CHECK_ARG(P && Q && out && (nc == 0 || (Lops && Rops)), "qd_superop_from_glf: null pointer");
  QD_CHECK_ARG(N >= 1 && N <= 512 && nc >= 0, "qd_superop_from_glf: bad sizes N=%d nc=%d", N, nc);
  hipLaunchKernelGGL(superop_from_glf_kernel, dim3(16384), dim3(256), 0, (hipStream_t)stream, (const c128*)P,
                     (const c128*)Q, (const c128*)Lops, (const c128*)Rops, nc, N, (c128*)out);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

// Dense Lindblad superoperator (oqs.liouvillian as a matrix on row-major vec(rho)), [N^2][N^2] into `out`.
extern "C" int qd_superop_lindblad(const qd_c128* H, const qd_c128* C, int nc, int N, qd_c128* out, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(H && out && (nc == 0 || C), "qd_superop_lindblad: null pointer");
  QD_CHECK_ARG(N >= 1 && N <= 512 && nc >= 0, "qd_superop_lindblad: bad sizes N=%d nc=%d", N, nc);
  hipStream_t st = (hipStream_t)stream;
  const size_t NN = (size_t)N * N;
  void* w = nullptr;
  int rc = workspace(WS_SUPEROP_OPS, (2 + (size_t)nc) * NN * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* P = (c128*)w;
  c128* Q = P + NN;
  c128* Rd = Q + NN;
  hipLaunchKernelGGL(lindblad_glf_ops_kernel, dim3((int)std::min<size_t>((NN + 255) / 256, 4096)), dim3(256), 0, st,
                     (const c128*)H, (const c128*)C, nc, N, P, Q, Rd);
  QD_HIP(hipGetLastError());
  return qd_superop_from_glf((const qd_c128*)P, (const qd_c128*)Q, C, (const qd_c128*)Rd, nc, N, out, stream);
}
