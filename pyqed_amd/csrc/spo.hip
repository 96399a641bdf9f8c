// spo.hip — split-operator wavepacket propagation (1D and 2D, multi-state).
//
// Replaces the Strang loops of pyqed/wpd.py:
//   SPO.run   (wpd.py:225-273, 1D single surface)   -> qd_spo1d_run
//   SPO2.run  (wpd.py:692-758, 2D diabatic, return_states=True, _KEO_linear
//              wpd.py:837-848)                       -> qd_spo2_run
//
// FFT: hand-written Stockham autosort (radix-4 stages + one radix-2 stage when
// log2 L is odd) on LDS, fp64 twiddles exp(-2 pi i k/L) from sincospi, L a power
// of two in [16, 1024].  Natural-order output, no bit reversal pass.
//
// 2D step layout (psi [nx][ny][ns], state index fastest, as the reference):
//   row kernel    (one row i per workgroup; contiguous 16-B loads):
//                   [IFFT_y] -> V/2 -> [snapshot] -> [V/2] -> [FFT_y]
//   column kernel (C columns per workgroup):
//                   FFT_x -> * exp_K / (nx ny) -> IFFT_x
// A run of n Strang steps V/2 K V/2 is: row(V/2, FFT_y), then n x {col, row},
// the last row kernel without the trailing V/2 + FFT_y.  Both V/2 are applied
// separately (no V/2 V/2 -> V merge) so every step is the reference's
// return_states=True arithmetic.  psi is read and written once per kernel;
// exp_V_half (ns^2 per point) once per row pass, exp_K once per column pass.
#include "qd_common.hpp"

#include <cstdlib>

namespace qd {
namespace {

constexpr int SPO_MAX_NS = 8;

__global__ void twiddle_kernel(int L, c128* tw) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < L; k += gridDim.x * blockDim.x) {
    double s, c;
    sincospi(-2.0 * (double)k / (double)L, &s, &c);
    tw[k] = cmk(c, s);
  }
}

// Stockham FFT of length L on LDS buffers a/b (one transform), T = L/4 threads,
// thread index t in [0, T).  All threads of the workgroup must call it (barriers).
// Returns the buffer holding the result.  INV: conjugated twiddles, no scaling.
template <int L, bool INV>
__device__ __forceinline__ c128* fft_lds(c128* a, c128* b, const c128* tw, int t, bool active) {
#pragma unroll
  for (int Ns = 1; Ns * 4 <= L; Ns *= 4) {
    if (active) {
      const int j = t;
      const int k = j % Ns;
      const int base = k * (L / (4 * Ns));
      c128 w1 = tw[base], w2 = tw[2 * base], w3 = tw[3 * base];
      if (INV) {
        w1 = cconj(w1);
        w2 = cconj(w2);
        w3 = cconj(w3);
      }
      const c128 v0 = a[j];
      const c128 v1 = cmul(a[j + L / 4], w1);
      const c128 v2 = cmul(a[j + L / 2], w2);
      const c128 v3 = cmul(a[j + 3 * L / 4], w3);
      const c128 a0 = cadd(v0, v2), a1 = csub(v0, v2), b0 = cadd(v1, v3), b1 = csub(v1, v3);
      const c128 ib1 = INV ? cmuli(b1) : cmulmi(b1);  // (+i or -i) * b1
      const int d = (j / Ns) * Ns * 4 + k;
      b[d] = cadd(a0, b0);
      b[d + Ns] = cadd(a1, ib1);
      b[d + 2 * Ns] = csub(a0, b0);
      b[d + 3 * Ns] = csub(a1, ib1);
    }
    __syncthreads();
    c128* tmp = a;
    a = b;
    b = tmp;
  }
  constexpr int lg = __builtin_ctz(L);
  if (lg & 1) {  // final radix-2 stage, Ns = L/2
    if (active) {
      constexpr int Ns = L / 2;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = t + h * (L / 4);
        const int k = j % Ns;
        c128 w = tw[k];
        if (INV) w = cconj(w);
        const c128 v0 = a[j], v1 = cmul(a[j + L / 2], w);
        const int d = (j / Ns) * Ns * 2 + k;
        b[d] = cadd(v0, v1);
        b[d + Ns] = csub(v0, v1);
      }
    }
    __syncthreads();
    c128* tmp = a;
    a = b;
    b = tmp;
  }
  return a;
}

// psi_point <- U psi_point for each grid point of one row held in LDS (buf[a][j]).
// out[a][j] = sum_b U[j][a][b] in[b][j] for the n points j of a row ([state][point] LDS layout, row
// stride `stride`).  Reads one LDS buffer and writes the other (no per-thread state arrays, which
// would be indexed at run time and land in scratch).
__device__ __forceinline__ void apply_point_op(const c128* in, c128* out, int stride, const c128* U /*[n][ns][ns]*/,
                                               int n, int ns) {
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const c128* u = U + (size_t)j * ns * ns;
    for (int a = 0; a < ns; ++a) {
      c128 s = cmk(0, 0);
      for (int b = 0; b < ns; ++b) s = cadd(s, cmul(u[a * ns + b], in[b * stride + j]));
      out[a * stride + j] = s;
    }
  }
}

enum RowFlags { ROW_INV = 1, ROW_VH1 = 2, ROW_SNAP = 4, ROW_VH2 = 8, ROW_FWD = 16, ROW_KY = 32, ROW_KZ = 64 };

// One row i of psi [nx][ny][ns]; FFTs along y (length L = ny) for each state.
// ROW_KY (Jacobi KEO, wpd.py:850-887): after FFT_y multiply by expKy[i][ky] (row i's k_y factor).
// `expVh` is the point operator of this pass (exp_V_half, or exp_V on merged passes).
template <int L>
__global__ __launch_bounds__(256) void spo2_row_kernel(c128* psi, const c128* expVh, const c128* twy, int ny, int ns,
                                                       int flags, c128* snap, const c128* expKy) {
  extern __shared__ c128 sm[];
  c128* tw = sm;            // L
  c128* A = sm + L;         // ns * L
  c128* Bf = A + ns * L;    // ns * L
  const int i = blockIdx.x;
  const size_t rowoff = (size_t)i * L * ns;
  for (int k = threadIdx.x; k < L; k += blockDim.x) tw[k] = twy[k];
  for (int e = threadIdx.x; e < L * ns; e += blockDim.x) A[(e % ns) * L + e / ns] = psi[rowoff + e];
  __syncthreads();
  const int T = L / 4;
  const int f = threadIdx.x / T, t = threadIdx.x % T;
  const bool active = f < ns;
  c128* cur = A;
  c128* oth = Bf;
  if (flags & ROW_INV) {
    c128* r = fft_lds<L, true>(A + (active ? f : 0) * L, Bf + (active ? f : 0) * L, tw, t, active);
    const bool inA = (r == A + (active ? f : 0) * L);
    cur = inA ? A : Bf;
    oth = inA ? Bf : A;
  }
  const c128* Ui = expVh + (size_t)i * L * ns * ns;
  if (flags & ROW_VH1) {
    apply_point_op(cur, oth, L, Ui, L, ns);
    c128* tmp = cur;
    cur = oth;
    oth = tmp;
    __syncthreads();
  }
  if (flags & ROW_SNAP) {
    for (int e = threadIdx.x; e < L * ns; e += blockDim.x) snap[rowoff + e] = cur[(e % ns) * L + e / ns];
    __syncthreads();
  }
  if (flags & ROW_VH2) {
    apply_point_op(cur, oth, L, Ui, L, ns);
    c128* tmp = cur;
    cur = oth;
    oth = tmp;
    __syncthreads();
  }
  if (flags & ROW_FWD) {
    c128* r = fft_lds<L, false>(cur + (active ? f : 0) * L, oth + (active ? f : 0) * L, tw, t, active);
    cur = (r == cur + (active ? f : 0) * L) ? cur : oth;
  }
  if (flags & ROW_KY) {
    const c128* ky = expKy + (size_t)i * L;
    for (int e = threadIdx.x; e < L * ns; e += blockDim.x) cur[e] = cmul(ky[e % L], cur[e]);
    __syncthreads();
  }
  for (int e = threadIdx.x; e < L * ns; e += blockDim.x) psi[rowoff + e] = cur[(e % ns) * L + e / ns];
}

// C columns j0..j0+C-1 of psi [nx][ny][ns]; FFT along x (length L = nx), multiply
// by expKT[j][i] (exp_K transposed and pre-scaled by 1/(nx ny)), inverse FFT.
template <int L, int C>
__global__ __launch_bounds__(256) void spo2_col_kernel(c128* psi, const c128* expKT, const c128* twx, int ny, int ns) {
  extern __shared__ c128 sm[];
  c128* tw = sm;                 // L
  c128* A = sm + L;              // C * ns * L   (layout [c][a][i])
  c128* Bf = A + C * ns * L;
  const int j0 = blockIdx.x * C;
  const int W = C * ns;  // transforms in this workgroup
  for (int k = threadIdx.x; k < L; k += blockDim.x) tw[k] = twx[k];
  for (int e = threadIdx.x; e < L * W; e += blockDim.x) {
    const int ca = e % W, i = e / W;
    A[ca * L + i] = psi[((size_t)i * ny + j0) * ns + ca];  // (j0 + c) * ns + a == j0*ns + ca
  }
  __syncthreads();
  const int T = L / 4;
  const int f = threadIdx.x / T, t = threadIdx.x % T;
  const bool active = f < W;
  const int fo = (active ? f : 0) * L;
  c128* r = fft_lds<L, false>(A + fo, Bf + fo, tw, t, active);
  c128* cur = (r == A + fo) ? A : Bf;
  c128* oth = (cur == A) ? Bf : A;
  for (int e = threadIdx.x; e < L * W; e += blockDim.x) {
    const int ca = e / L, i = e % L;
    const int c = ca / ns;
    cur[ca * L + i] = cmul(cur[ca * L + i], expKT[(size_t)(j0 + c) * L + i]);
  }
  __syncthreads();
  r = fft_lds<L, true>(cur + fo, oth + fo, tw, t, active);
  cur = (r == cur + fo) ? cur : oth;
  for (int e = threadIdx.x; e < L * W; e += blockDim.x) {
    const int ca = e % W, i = e / W;
    psi[((size_t)i * ny + j0) * ns + ca] = cur[ca * L + i];
  }
}

// ---------------------------------------------------------------- latency-shaped 2D passes (ns <= 2)
// At 256 x 256 x 2 a pass moves 8-16 KB per workgroup, so its time is the chain of dependent
// memory round trips, not bandwidth.  These variants issue EVERY global load of the pass (psi,
// the point operator, exp_Ky / exp_K, twiddles) before the first wait, keep the point-local work
// (V/2, snapshot, V/2, k_y phase) in registers, and touch LDS only for the FFT exchanges: one
// load round trip + one store drain per pass.  Same arithmetic, same order as the generic kernels.

// Row pass, thread j owns grid point j of row i (blockDim = max(L, 64)).
template <int L, int NS>
__global__ __launch_bounds__(L < 64 ? 64 : L) void spo2_row_fast_kernel(c128* psi, const c128* U, const c128* twy,
                                                                        int flags, c128* snap, const c128* expKy) {
  extern __shared__ c128 sm[];
  c128* tw = sm;          // L
  c128* A = sm + L;       // NS * L   ([state][point])
  c128* Bf = A + NS * L;  // NS * L
  const int i = blockIdx.x, j = threadIdx.x;
  const bool own = j < L;
  const size_t pt = (size_t)i * L + j;
  c128 p[NS], u[NS * NS], ky = cmk(1, 0);
  if (own) {
#pragma unroll
    for (int a = 0; a < NS; ++a) p[a] = psi[pt * NS + a];
    if (flags & (ROW_VH1 | ROW_VH2)) {
#pragma unroll
      for (int e = 0; e < NS * NS; ++e) u[e] = U[pt * NS * NS + e];
    }
    if (flags & ROW_KY) ky = expKy[pt];
    tw[j] = twy[j];
  }
  constexpr int T = L / 4;
  const int f = j / T, t = j % T;
  const bool active = f < NS;
  auto fft = [&](auto inv_tag) {
    constexpr bool INV = decltype(inv_tag)::value;
    if (own) {
#pragma unroll
      for (int a = 0; a < NS; ++a) A[a * L + j] = p[a];
    }
    __syncthreads();
    c128* r = fft_lds<L, INV>(A + (active ? f : 0) * L, Bf + (active ? f : 0) * L, tw, t, active);
    // fft_lds ends on a barrier; the result buffer is the same for every transform
    c128* res = (r == A + (active ? f : 0) * L) ? A : Bf;
    if (own) {
#pragma unroll
      for (int a = 0; a < NS; ++a) p[a] = res[a * L + j];
    }
    __syncthreads();  // the next FFT overwrites A
  };
  auto point_op = [&]() {
    c128 q[NS];
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      c128 s = cmk(0, 0);
#pragma unroll
      for (int b = 0; b < NS; ++b) s = cadd(s, cmul(u[a * NS + b], p[b]));
      q[a] = s;
    }
#pragma unroll
    for (int a = 0; a < NS; ++a) p[a] = q[a];
  };
  if (flags & ROW_INV) fft(std::true_type{});  // (fft's first barrier also publishes tw)
  if (flags & ROW_VH1) point_op();
  if ((flags & ROW_SNAP) && own) {
#pragma unroll
    for (int a = 0; a < NS; ++a) snap[pt * NS + a] = p[a];
  }
  if (flags & ROW_VH2) point_op();
  if (flags & ROW_FWD) fft(std::false_type{});
  if (flags & ROW_KY) {
#pragma unroll
    for (int a = 0; a < NS; ++a) p[a] = cmul(ky, p[a]);
  }
  if (own) {
#pragma unroll
    for (int a = 0; a < NS; ++a) psi[pt * NS + a] = p[a];
  }
}

// Column pass over C columns j0..j0+C-1 (W = C*NS transforms, blockDim = W*L/4): exp_K for the
// pass is loaded with psi, before the forward FFT.
template <int L, int C, int NS>
__global__ __launch_bounds__(C * NS * L / 4 < 64 ? 64 : C * NS * L / 4) void spo2_col_fast_kernel(
    c128* psi, const c128* expKT, const c128* twx, int ny) {
  constexpr int W = C * NS;
  constexpr int BD = W * L / 4 < 64 ? 64 : W * L / 4;
  constexpr int IT = (L * W + BD - 1) / BD;
  extern __shared__ c128 sm[];
  c128* tw = sm;           // L
  c128* A = sm + L;        // W * L  ([c][a][i])
  c128* Bf = A + W * L;
  const int j0 = blockIdx.x * C;
  const int tid = threadIdx.x;
  constexpr bool FULL = (L * W) % BD == 0;
  c128 v[IT], kf[IT];
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;  // load order: row i = e / W, transform ca = e % W (coalesced);
    v[n] = cmk(0, 0);            // multiply order: transform ca = e / L, row i = e % L
    kf[n] = cmk(0, 0);
    if (FULL || e < L * W) {
      v[n] = psi[((size_t)(e / W) * ny + j0) * NS + e % W];
      kf[n] = expKT[(size_t)(j0 + (e / L) / NS) * L + e % L];
    }
  }
  for (int k = tid; k < L; k += BD) tw[k] = twx[k];
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;
    if (FULL || e < L * W) A[(e % W) * L + e / W] = v[n];
  }
  __syncthreads();
  constexpr int T = L / 4;
  const int f = tid / T, t = tid % T;
  const bool active = f < W;
  const int fo = (active ? f : 0) * L;
  c128* r = fft_lds<L, false>(A + fo, Bf + fo, tw, t, active);
  c128* cur = (r == A + fo) ? A : Bf;
  c128* oth = (cur == A) ? Bf : A;
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;
    if (FULL || e < L * W) cur[e] = cmul(cur[e], kf[n]);
  }
  __syncthreads();
  r = fft_lds<L, true>(cur + fo, oth + fo, tw, t, active);
  cur = (r == cur + fo) ? cur : oth;
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;
    if (FULL || e < L * W) psi[((size_t)(e / W) * ny + j0) * NS + e % W] = cur[(e % W) * L + e / W];
  }
}

// Middle-axis pass of a 3D grid psi [nx][ny][nz][ns] viewed as [outer][L][inner]
// (inner = nz*ns): each workgroup transforms C consecutive inner indices of one
// outer index i along the L axis (chunks of C*16 B per row: coalesced).
template <int L, int C, bool INV>
__global__ __launch_bounds__(256) void spo_mid_kernel(c128* psi, const c128* tw_g, int inner) {
  __shared__ c128 tw[L];
  __shared__ c128 A[C * L], Bf[C * L];  // layout [c][j]; LDS sized to the C transforms of this block
  const int chunks = inner / C;
  const int i = blockIdx.x / chunks, c0 = (blockIdx.x % chunks) * C;
  c128* base = psi + (size_t)i * L * inner + c0;
  for (int k = threadIdx.x; k < L; k += blockDim.x) tw[k] = tw_g[k];
  for (int e = threadIdx.x; e < L * C; e += blockDim.x) {
    const int c = e % C, j = e / C;
    A[c * L + j] = base[(size_t)j * inner + c];
  }
  __syncthreads();
  const int T = L / 4;
  const int f = threadIdx.x / T, t = threadIdx.x % T;
  const bool active = f < C;
  const int fo = (active ? f : 0) * L;
  c128* r = fft_lds<L, INV>(A + fo, Bf + fo, tw, t, active);
  c128* cur = (r == A + fo) ? A : Bf;
  for (int e = threadIdx.x; e < L * C; e += blockDim.x) {
    const int c = e % C, j = e / C;
    base[(size_t)j * inner + c] = cur[c * L + j];
  }
}

// Latency-shaped middle-axis pass (same transforms and arithmetic as spo_mid_kernel): the block size is fixed at
// compile time (BD = C L / 4 threads, IT = 4 elements per thread), so every global load of the pass (the C
// columns of 16-B pieces and the twiddles) is issued before the first wait and every store after the transform:
// one load round trip + one store drain per pass instead of IT dependent load / LDS-store iterations.
template <int L, int C, bool INV>
__global__ __launch_bounds__(C * L / 4 < 64 ? 64 : C * L / 4) void spo_mid_fast_kernel(c128* psi, const c128* tw_g,
                                                                                       int inner) {
  constexpr int BD = C * L / 4 < 64 ? 64 : C * L / 4;
  constexpr int IT = (L * C + BD - 1) / BD;
  constexpr bool FULL = (L * C) % BD == 0;
  __shared__ c128 tw[L];
  __shared__ c128 A[C * L], Bf[C * L];  // layout [c][j]
  const int chunks = inner / C;
  const int i = blockIdx.x / chunks, c0 = (blockIdx.x % chunks) * C;
  c128* base = psi + (size_t)i * L * inner + c0;
  const int tid = threadIdx.x;
  c128 v[IT];
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;  // c = e % C fastest: C * 16 B contiguous per row j
    v[n] = (FULL || e < L * C) ? base[(size_t)(e / C) * inner + e % C] : cmk(0, 0);
  }
  static_assert(L <= BD, "one twiddle per thread");
  const c128 twv = tid < L ? tw_g[tid] : cmk(0, 0);
  if (tid < L) tw[tid] = twv;
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;
    if (FULL || e < L * C) A[(e % C) * L + e / C] = v[n];
  }
  __syncthreads();
  constexpr int T = L / 4;
  const int f = tid / T, t = tid % T;
  const bool active = f < C;
  const int fo = (active ? f : 0) * L;
  c128* r = fft_lds<L, INV>(A + fo, Bf + fo, tw, t, active);
  const c128* cur = (r == A + fo) ? A : Bf;
#pragma unroll
  for (int n = 0; n < IT; ++n) {
    const int e = tid + n * BD;
    if (FULL || e < L * C) base[(size_t)(e / C) * inner + e % C] = cur[(e % C) * L + e / C];
  }
}

// expKT[j][i] = expK[i][j] * scale
__global__ void transpose_scale_kernel(const c128* expK, int nx, int ny, double scale, c128* expKT) {
  const size_t tot = (size_t)nx * ny;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / ny), j = (int)(e % ny);
    expKT[(size_t)j * nx + i] = cscale(expK[e], scale);
  }
}

// ---------------------------------------------------------------- 1D persistent SPO
// SPO.run structure (wpd.py:250-270): V/2 ; for i in 1..nt//nout-1: nout x [K, V], snapshot ;
// then K, V/2.  One workgroup per wavepacket, all steps in LDS.
template <int L>
__global__ __launch_bounds__(256) void spo1d_kernel(c128* psi, const c128* expV, const c128* expVh, const c128* expK,
                                                    const c128* twg, int nt, int nout, c128* snap) {
  __shared__ c128 tw[L], A[L], Bf[L], eV[L], eK[L];
  const int b = blockIdx.x;
  c128* p = psi + (size_t)b * L;
  for (int k = threadIdx.x; k < L; k += blockDim.x) {
    tw[k] = twg[k];
    eV[k] = expV[k];
    eK[k] = cscale(expK[k], 1.0 / L);
    A[k] = cmul(expVh[k], p[k]);
  }
  __syncthreads();
  const int T = L / 4;
  const int t = threadIdx.x;
  const bool active = t < T;
  c128* cur = A;
  c128* oth = Bf;
  const int nblk = nt / nout;
  const int nsnap = nblk > 0 ? nblk - 1 : 0;
  auto kstep = [&]() {
    c128* r = fft_lds<L, false>(cur, oth, tw, t, active);
    if (r != cur) { oth = cur; cur = r; }
    for (int k = threadIdx.x; k < L; k += blockDim.x) cur[k] = cmul(cur[k], eK[k]);
    __syncthreads();
    r = fft_lds<L, true>(cur, oth, tw, t, active);
    if (r != cur) { oth = cur; cur = r; }
  };
  for (int blk = 1; blk < nblk; ++blk) {
    for (int s = 0; s < nout; ++s) {
      kstep();
      for (int k = threadIdx.x; k < L; k += blockDim.x) cur[k] = cmul(eV[k], cur[k]);
      __syncthreads();
    }
    if (snap)
      for (int k = threadIdx.x; k < L; k += blockDim.x) snap[((size_t)b * nsnap + (blk - 1)) * L + k] = cur[k];
  }
  kstep();
  for (int k = threadIdx.x; k < L; k += blockDim.x) p[k] = cmul(expVh[k], cur[k]);
}

// ---------------------------------------------------------------- point propagators (SPO build)
// exp(-i V tau) per grid point for tau = dt and dt/2 (wpd.py:585-623: eigh -> U e^{-i w tau} U^+).
// LAPACK's eigh reads the lower triangle and ignores Im of the diagonal; so does this: a = Re V00,
// d = Re V11, b = conj(V10).  For ns = 2 the exponential is closed form,
//   exp(-i H tau) = e^{-i m tau} [cos(r tau) I - i (sin(r tau)/r) (H - m I)],
//   m = (a + d)/2, delta = (a - d)/2, r = sqrt(delta^2 + |b|^2)   (sin(r tau)/r -> tau at r = 0),
// identical to the eigen form in exact arithmetic and independent of the eigenvector phases.
__device__ __forceinline__ void expv2(double a, double d, c128 b, double tau, c128* E) {
  const double m = 0.5 * (a + d), de = 0.5 * (a - d);
  const double r = sqrt(de * de + b.re * b.re + b.im * b.im);
  double sn, cs, ph_s, ph_c;
  sincos(r * tau, &sn, &cs);
  const double sr = r > 0.0 ? sn / r : tau;
  sincos(-m * tau, &ph_s, &ph_c);
  const c128 ph = cmk(ph_c, ph_s);
  E[0] = cmul(ph, cmk(cs, -sr * de));                 // c - i s delta
  E[3] = cmul(ph, cmk(cs, sr * de));                  // c + i s delta
  E[1] = cmul(ph, cmulmi(cscale(b, sr)));             // -i s b
  E[2] = cmul(ph, cmulmi(cscale(cconj(b), sr)));      // -i s b*
}

template <bool CPLX>
__global__ void spo_expv_kernel(const void* v_, long npts, int ns, double dt, c128* expV, c128* expVh) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < npts; e += (long)gridDim.x * blockDim.x) {
    if (ns == 1) {
      const double a = CPLX ? ((const c128*)v_)[e].re : ((const double*)v_)[e];
      double sn, cs;
      sincos(-a * dt, &sn, &cs);
      if (expV) expV[e] = cmk(cs, sn);
      sincos(-a * 0.5 * dt, &sn, &cs);
      expVh[e] = cmk(cs, sn);
      continue;
    }
    double a, d;
    c128 b;
    if (CPLX) {
      const c128* v = (const c128*)v_ + e * 4;
      a = v[0].re;
      d = v[3].re;
      b = cconj(v[2]);
    } else {
      const double* v = (const double*)v_ + e * 4;
      a = v[0];
      d = v[3];
      b = cmk(v[2], 0.0);
    }
    c128 E[4];
    if (expV) {
      expv2(a, d, b, dt, E);
#pragma unroll
      for (int q = 0; q < 4; ++q) expV[e * 4 + q] = E[q];
    }
    expv2(a, d, b, 0.5 * dt, E);
#pragma unroll
    for (int q = 0; q < 4; ++q) expVh[e * 4 + q] = E[q];
  }
}

// ---------------------------------------------------------------- 256-point passes in registers
// L = 256 = 16 x 16 (Cooley-Tukey, n = 16 n1 + n2, k = k1 + 16 k2):
//   X[k1 + 16 k2] = sum_n2 w16^(n2 k2) w256^(n2 k1) sum_n1 x[16 n1 + n2] w16^(n1 k1)
// ONE wave per transform set.  Lane (g, s) = (lane >> 2, lane & 3) holds the points
// p_a = 64 a + 16 s + g (a = 0..3) of its line, before and after every transform: an inverse FFT,
// point-local work and a forward FFT chain with no data movement.  Each 16-point DFT runs inside
// a quad (4 x 4: DFT4 in registers, three quad-DPP rotations, DFT4); the two 16-point steps
// exchange through LDS once.  Per pass: one global load round trip, two wave-local LDS
// transposes per FFT, no workgroup-wide barrier (the Stockham LDS FFT takes 4 barrier stages per
// transform plus the staging).  w = exp(-2 pi i / L) forward, its conjugate inverse; no scaling.
template <bool ZPOS>  // y[r] = sum_a x[a] z^(a r), z = +i (ZPOS) or -i
__device__ __forceinline__ void dft4(c128 (&x)[4]) {
  const c128 s02 = cadd(x[0], x[2]), d02 = csub(x[0], x[2]);
  const c128 s13 = cadd(x[1], x[3]), d13 = csub(x[1], x[3]);
  const c128 zd = ZPOS ? cmuli(d13) : cmulmi(d13);
  x[0] = cadd(s02, s13);
  x[1] = cadd(d02, zd);
  x[2] = csub(s02, s13);
  x[3] = csub(d02, zd);
}

struct Q16Tw {
  c128 a[4];  // w4^(a s)            (pre-rotation of the inputs, also the final w4^(s d))
  c128 b[4];  // w16^(s ((s - r) & 3))  (inner twiddle of the sent element r)
  c128 d[4];  // w256^(g (s + 4 d))  (inter-step twiddle of output k1 = s + 4 d)
};

__device__ __forceinline__ Q16Tw q16_twiddles(const c128* tw, int g, int s) {
  Q16Tw t;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    t.a[q] = tw[64 * ((q * s) & 3)];
    t.b[q] = tw[16 * ((s * ((s - q) & 3)) & 15)];
    t.d[q] = tw[(g * (s + 4 * q)) & 255];
  }
  return t;
}

__device__ __forceinline__ c128 twmul(c128 v, c128 w, bool inv) { return cmul(v, inv ? cconj(w) : w); }

// 16-point DFT of the quad: lane s holds v[a] = x[4 a + s]; on return lane s holds X[s + 4 d] in v[d].
template <bool INV>
__device__ __forceinline__ void dft16_quad(c128 (&v)[4], const Q16Tw& t) {
  // U_s[(s - r) & 3] = sum_a (v[a] w4^(a s)) w4^(-a r): pre-rotate, DFT4 with root w4^-1
#pragma unroll
  for (int a = 1; a < 4; ++a) v[a] = twmul(v[a], t.a[a], INV);
  dft4<!INV>(v);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = twmul(v[r], t.b[r], INV);
  // lane l receives element r of lane (l + r) & 3: R_r = U_b[l] w16^(b l), b = (l + r) & 3
  v[1] = dpp_qc<0x39>(v[1]);
  v[2] = dpp_qc<0x4E>(v[2]);
  v[3] = dpp_qc<0x93>(v[3]);
  // X[l + 4 d] = w4^(l d) sum_r w4^(r d) R_r
  dft4<INV>(v);
#pragma unroll
  for (int d = 1; d < 4; ++d) v[d] = twmul(v[d], t.a[d], INV);
}

// 256-point FFT of NS lines held in the wave's layout; S: NS x 16 x 17 c128 of LDS (this wave's).
template <bool INV, int NS>
__device__ __forceinline__ void fft256_wave(c128 (&x)[NS][4], const Q16Tw& t, c128* S, int g, int s) {
#pragma unroll
  for (int c = 0; c < NS; ++c) {
    dft16_quad<INV>(x[c], t);
#pragma unroll
    for (int d = 0; d < 4; ++d) S[c * 272 + (s + 4 * d) * 17 + g] = twmul(x[c][d], t.d[d], INV);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int c = 0; c < NS; ++c) {
#pragma unroll
    for (int a = 0; a < 4; ++a) x[c][a] = S[c * 272 + g * 17 + 4 * a + s];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int c = 0; c < NS; ++c) dft16_quad<INV>(x[c], t);
}

// Row pass of spo2_row_fast_kernel for L = 256: one workgroup per row, wave c = state c (its 256-point
// transforms run on 4 values per lane).  The point operators mix the states of a point, whose values
// sit in the same lane of every wave: they are exchanged through LDS (one workgroup barrier per point
// operator).  Same flags and arithmetic order of the point work as the LDS kernels:
// [IFFT_y] -> V/2 -> [snapshot] -> [V/2] -> [FFT_y] -> [k_y phase].
// Batches of wavefunctions (qd_spo2_run_batch): blockIdx.y = member w, psi / snap offset by w * wstride /
// w * sstride (the point operators are shared).
// KY: the Jacobi k_y factor is compiled in only where used (its 4 per-lane values would otherwise hold 16 VGPRs
// through the whole pass: 142 -> under 128 VGPRs, 3 -> 4 waves per SIMD for the linear case).
template <int NS, bool KY>
__global__ __launch_bounds__(64 * NS) void spo2_row_q16_kernel(c128* psi, const c128* U, const c128* twy, int flags,
                                                               c128* snap, const c128* expKy, size_t wstride = 0,
                                                               size_t sstride = 0) {
  __shared__ c128 S[NS * 272];
  __shared__ c128 Xs[NS * 256];   // point-operator exchange: [state][lane * 4 + a]
  const int i = blockIdx.x, c = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 2, s = lane & 3;
  psi += blockIdx.y * wstride;
  if (snap) snap += blockIdx.y * sstride;
  c128 x[1][4], u[4][NS], ky[4];
  const size_t row = (size_t)i * 256;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const size_t pt = row + 64 * a + 16 * s + g;
    x[0][a] = psi[pt * NS + c];
    if (flags & (ROW_VH1 | ROW_VH2)) {
#pragma unroll
      for (int b = 0; b < NS; ++b) u[a][b] = U[(pt * NS + c) * NS + b];   // row c of the point's operator
    }
    if constexpr (KY) ky[a] = expKy[pt];
  }
  const Q16Tw t = q16_twiddles(twy, g, s);
  c128* Sw = S + c * 272;
  auto point_op = [&]() {
    if (NS > 1) {
#pragma unroll
      for (int a = 0; a < 4; ++a) Xs[c * 256 + lane * 4 + a] = x[0][a];
      __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      c128 acc = cmk(0, 0);
#pragma unroll
      for (int b = 0; b < NS; ++b) acc = cadd(acc, cmul(u[a][b], NS > 1 ? Xs[b * 256 + lane * 4 + a] : x[0][a]));
      x[0][a] = acc;
    }
    if (NS > 1) __syncthreads();   // Xs is rewritten by the next operator
  };
  if (flags & ROW_INV) fft256_wave<true, 1>(x, t, Sw, g, s);
  if (flags & ROW_VH1) point_op();
  if (flags & ROW_SNAP) {
#pragma unroll
    for (int a = 0; a < 4; ++a) snap[(row + 64 * a + 16 * s + g) * NS + c] = x[0][a];
  }
  if (flags & ROW_VH2) point_op();
  if (flags & ROW_FWD) fft256_wave<false, 1>(x, t, Sw, g, s);
  if constexpr (KY) {
    if (flags & ROW_KY) {
#pragma unroll
      for (int a = 0; a < 4; ++a) x[0][a] = cmul(ky[a], x[0][a]);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) psi[(row + 64 * a + 16 * s + g) * NS + c] = x[0][a];
}

// Row pass for batches, one wave per (row i, member): the wave holds both states of its points (x[c][a] =
// psi[64 a + 16 s + g][c]), so the point operators are lane-local (no state exchange through LDS, no workgroup
// barrier but the one after the operator staging) and every lane loads 32 contiguous bytes per point.  The MB
// waves of a workgroup are MB members of one row and share the row's point operators, staged in LDS once.  The
// two states' 256-point transforms run one after the other through one 272-entry exchange buffer per wave (LDS
// per workgroup 16 KB + MB x 4.25 KB: four workgroups of MB = 4 per CU).  Same arithmetic and order as
// spo2_row_q16_kernel<2, false>, so the results are bit-identical.
template <int MB>
__global__ __launch_bounds__(64 * MB) void spo2_row_wave_kernel(c128* psi, const c128* U, const c128* twy, int flags,
                                                                c128* snap, int B, size_t wstride, size_t sstride) {
  __shared__ c128 Us[256 * 4];          // [point][row c][col b]
  __shared__ c128 S[MB * 272];          // per-wave FFT exchange
  const int i = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 2, s = lane & 3;
  const int member = blockIdx.y * MB + w;
  const bool live = member < B;          // uniform per wave; dead waves still join the staging barrier
  c128* ps = psi + (size_t)(live ? member : 0) * wstride;
  const size_t row = (size_t)i * 256;
  c128 x[2][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const size_t pt = row + 64 * a + 16 * s + g;
    x[0][a] = ps[pt * 2];
    x[1][a] = ps[pt * 2 + 1];
  }
  const bool vh = flags & (ROW_VH1 | ROW_VH2);
  if (vh) {
#pragma unroll
    for (int q = 0; q < 1024 / (64 * MB); ++q) {
      const int e = threadIdx.x + 64 * MB * q;
      Us[e] = U[row * 4 + e];
    }
  }
  const Q16Tw t = q16_twiddles(twy, g, s);
  c128* Sw = S + w * 272;
  auto line = [&](int c) -> c128 (&)[1][4] { return *reinterpret_cast<c128(*)[1][4]>(&x[c][0]); };
  if (vh) __syncthreads();
  if (!live) return;
  auto point_op = [&]() {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int pt = 64 * a + 16 * s + g;
      c128 y[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        c128 acc = cmk(0, 0);
#pragma unroll
        for (int b = 0; b < 2; ++b) acc = cadd(acc, cmul(Us[pt * 4 + c * 2 + b], x[b][a]));
        y[c] = acc;
      }
      x[0][a] = y[0];
      x[1][a] = y[1];
    }
  };
  if (flags & ROW_INV) {
    fft256_wave<true, 1>(line(0), t, Sw, g, s);
    fft256_wave<true, 1>(line(1), t, Sw, g, s);
  }
  if (flags & ROW_VH1) point_op();
  if (flags & ROW_SNAP) {
    c128* sn = snap + (size_t)member * sstride;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const size_t pt = row + 64 * a + 16 * s + g;
      sn[pt * 2] = x[0][a];
      sn[pt * 2 + 1] = x[1][a];
    }
  }
  if (flags & ROW_VH2) point_op();
  if (flags & ROW_FWD) {
    fft256_wave<false, 1>(line(0), t, Sw, g, s);
    fft256_wave<false, 1>(line(1), t, Sw, g, s);
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const size_t pt = row + 64 * a + 16 * s + g;
    ps[pt * 2] = x[0][a];
    ps[pt * 2 + 1] = x[1][a];
  }
}

// Column pass of spo2_col_fast_kernel for L = nx = 256: one 64-lane workgroup per (column j, state c)
// (no state mixing in this pass): FFT_x -> * exp_K / (nx ny) -> IFFT_x.  Blocks of one XCD (blockIdx.x
// % 8) take a contiguous run of columns, so the pieces that adjacent columns read from one row share
// that XCD's L2 lines.
template <int NS>
__global__ __launch_bounds__(64) void spo2_col_q16_kernel(c128* psi, const c128* expKT, const c128* twx, int ncols,
                                                          int pitch, size_t wstride = 0) {
  __shared__ c128 S[272];
  const int b = blockIdx.x, c = blockIdx.y;
  psi += blockIdx.z * wstride;
  const int j = (ncols % 8 == 0) ? (b % 8) * (ncols / 8) + b / 8 : b;
  const int lane = threadIdx.x, g = lane >> 2, s = lane & 3;
  c128 x[1][4], kf[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int p = 64 * a + 16 * s + g;
    x[0][a] = psi[((size_t)p * pitch + j) * NS + c];
    kf[a] = expKT[(size_t)j * 256 + p];
  }
  const Q16Tw t = q16_twiddles(twx, g, s);
  fft256_wave<false, 1>(x, t, S, g, s);
#pragma unroll
  for (int a = 0; a < 4; ++a) x[0][a] = cmul(x[0][a], kf[a]);
  fft256_wave<true, 1>(x, t, S, g, s);
#pragma unroll
  for (int a = 0; a < 4; ++a) psi[((size_t)(64 * a + 16 * s + g) * pitch + j) * NS + c] = x[0][a];
}

// Column pass for batches with NC adjacent columns per 64 NC-thread workgroup and one wave per column holding
// both states (x[c][a], c = state): the 256 x NC x 2 tile is read and written as NC x 32-B contiguous row pieces
// (256 B at NC = 8), and the waves' FFT exchange buffers live inside the tile (it is dead between the line reads
// and the write-back), so the workgroup's LDS is the tile alone (NC = 8: 68 KB, two workgroups per CU as the
// round-3 4-column kernel).  Same arithmetic per line as spo2_col_q16_kernel.  NS = 2, nx = ny = 256.
template <int NC>
__global__ __launch_bounds__(64 * NC) void spo2_col_tile8_kernel(c128* psi, const c128* expKT, const c128* twx,
                                                                 size_t wstride) {
  constexpr int TW = 2 * NC + 1;     // tile row stride: 2 NC lines + 1 pad
  __shared__ c128 T[256 * TW];       // [row][lines]; per-wave FFT exchange T + w * 272 in between
  psi += blockIdx.y * wstride;
  const int j0 = blockIdx.x * NC;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 2, s = lane & 3;
  const int j = j0 + w;
  {
    c128 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {    // element e = row * 2 NC + (column - j0) * 2 + state
      const int e = tid + 64 * NC * q, r = e / (2 * NC), cs = e % (2 * NC);
      v[q] = psi[((size_t)r * 256 + j0) * 2 + cs];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 64 * NC * q;
      T[(e / (2 * NC)) * TW + e % (2 * NC)] = v[q];
    }
  }
  c128 kf[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) kf[a] = expKT[(size_t)j * 256 + 64 * a + 16 * s + g];
  __syncthreads();
  c128 x[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int a = 0; a < 4; ++a) x[c][a] = T[(64 * a + 16 * s + g) * TW + 2 * w + c];
  const Q16Tw t = q16_twiddles(twx, g, s);
  __syncthreads();                   // every wave has its lines: the tile becomes the FFT exchange
  c128* Sw = T + w * 272;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    c128(&xl)[1][4] = *reinterpret_cast<c128(*)[1][4]>(&x[c][0]);
    fft256_wave<false, 1>(xl, t, Sw, g, s);
#pragma unroll
    for (int a = 0; a < 4; ++a) x[c][a] = cmul(x[c][a], kf[a]);
    fft256_wave<true, 1>(xl, t, Sw, g, s);
  }
  __syncthreads();                   // every wave is done with its exchange region
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int a = 0; a < 4; ++a) T[(64 * a + 16 * s + g) * TW + 2 * w + c] = x[c][a];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = tid + 64 * NC * q, r = e / (2 * NC), cs = e % (2 * NC);
    psi[((size_t)r * 256 + j0) * 2 + cs] = T[r * TW + cs];
  }
}

// ---------------------------------------------------------------- 64-point transforms on 16 lanes
// L = 64 = 4 x 16 (n = 4 m + q, k = k1 + 16 k2):
//   X[k1 + 16 k2] = sum_q w4^(q k2) [w64^(q k1) X_q[k1]],  X_q = 16-point DFT of x[4 m + q]
// A group of 16 lanes (lane l = 4 qq + s of the group) transforms one line held in LDS (any stride):
// quad qq runs the 16-point DFT of x[4 m + qq] (dft16_quad: lane s loads x[16 a + 4 s + qq]), scales output
// k1 = s + 4 d by w64^(qq k1), the 64 values are exchanged through the line's own storage (slot 4 k1 + q),
// and lane l finishes X[l + 16 k2] (k2 = 0..3) with one register DFT4.  Returns the result in v (natural order
// X[l + 16 k2] in v[k2]); the line's storage holds exchange values afterwards.  Twiddles t = q64_twiddles of the
// 64-entry table w64^k (they depend on the lane only).  INV: conjugated twiddles, no scaling.
__device__ __forceinline__ Q16Tw q64_twiddles(const c128* tw, int qq, int s) {
  Q16Tw t;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    t.a[q] = tw[16 * ((q * s) & 3)];
    t.b[q] = tw[4 * ((s * ((s - q) & 3)) & 15)];
    t.d[q] = tw[(qq * (s + 4 * q)) & 63];
  }
  return t;
}

// The transform from registers already in the input layout (v[a] = x[16 a + 4 s + qq]); `line` is exchange space.
template <bool INV>
__device__ __forceinline__ void fft64_regs(c128* line, int stride, const Q16Tw& t, int qq, int s, c128 (&v)[4]) {
  dft16_quad<INV>(v, t);
#pragma unroll
  for (int d = 0; d < 4; ++d) v[d] = twmul(v[d], t.d[d], INV);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int d = 0; d < 4; ++d) line[(4 * (s + 4 * d) + qq) * stride] = v[d];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int l = 4 * qq + s;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = line[(4 * l + q) * stride];
  dft4<INV>(v);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool INV>
__device__ __forceinline__ void fft64_group(c128* line, int stride, const Q16Tw& t, int qq, int s, c128 (&v)[4]) {
#pragma unroll
  for (int a = 0; a < 4; ++a) v[a] = line[(16 * a + 4 * s + qq) * stride];
  fft64_regs<INV>(line, stride, t, qq, s, v);
}

// Middle-axis pass at L = 64 with the register transform (same tiles and loads as spo_mid_fast_kernel<64, C>):
// the C columns (C x 16 B per row) are staged in LDS, each 16-lane group transforms one column line in place
// (fft64_group, wave barriers only), and the tile is stored back.
// KD: the whole separable axis propagator F^-1 diag(d) F on each line (forward transform, * d[k], inverse; d holds
// e_y / ny), natural order in and out (qd_spo3_run_axes on power-of-two 64-point axes)
template <int C, bool INV, bool KD = false>
__global__ __launch_bounds__(16 * C) void spo_mid64_kernel(c128* psi, const c128* tw_g, int inner,
                                                           const c128* dk = nullptr) {
  constexpr int BD = 16 * C, LS = 65;  // line stride (padded)
  __shared__ c128 A[C * LS];
  __shared__ c128 tw[64];
  const int chunks = inner / C;
  const int i = blockIdx.x / chunks, c0 = (blockIdx.x % chunks) * C;
  c128* base = psi + (size_t)i * 64 * inner + c0;
  const int tid = threadIdx.x, g = tid >> 4, lane16 = tid & 15, qq = lane16 >> 2, s = lane16 & 3;
  c128 v[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = tid + BD * n;
    v[n] = base[(size_t)(e / C) * inner + e % C];
  }
  if (tid < 64) tw[tid] = tw_g[tid];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = tid + BD * n;
    A[(e % C) * LS + e / C] = v[n];
  }
  __syncthreads();
  const Q16Tw t = q64_twiddles(tw, qq, s);
  c128* line = A + g * LS;
  fft64_group<INV>(line, 1, t, qq, s, v);
  if constexpr (KD) {
#pragma unroll
    for (int k = 0; k < 4; ++k) line[lane16 + 16 * k] = cmul(v[k], dk[lane16 + 16 * k]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    fft64_group<true>(line, 1, t, qq, s, v);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) line[lane16 + 16 * k] = v[k];
  __syncthreads();
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = tid + BD * n;
    base[(size_t)(e / C) * inner + e % C] = A[(e % C) * LS + e / C];
  }
}

// Column (x) pass at L = nx = 64 with the register transform (same tiles and loads as spo2_col_fast_kernel<64, C,
// NS>): W = C NS lines (column-major over states) staged in LDS, each 16-lane group runs FFT_x -> * exp_K /
// (nx ny nz) -> IFFT_x on one line in registers (natural order between the transforms).
template <int C, int NS>
__global__ __launch_bounds__(16 * C * NS) void spo_col64_kernel(c128* psi, const c128* expKT, const c128* tw_g,
                                                                int ny, int kstride = 64) {
  constexpr int W = C * NS, BD = 16 * W, LS = 65;
  __shared__ c128 A[W * LS];
  __shared__ c128 tw[64];
  const int j0 = blockIdx.x * C;
  const int tid = threadIdx.x, g = tid >> 4, lane16 = tid & 15, qq = lane16 >> 2, s = lane16 & 3;
  c128 v[4], kf[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = tid + BD * n;   // row i = e / W, line w = e % W (coalesced W x 16 B per row)
    v[n] = psi[((size_t)(e / W) * ny + j0) * NS + e % W];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) kf[k] = expKT[(size_t)(j0 + g / NS) * kstride + lane16 + 16 * k];   // 0: one factor
  if (tid < 64) tw[tid] = tw_g[tid];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = tid + BD * n;
    A[(e % W) * LS + e / W] = v[n];
  }
  __syncthreads();
  const Q16Tw t = q64_twiddles(tw, qq, s);
  c128* line = A + g * LS;
  fft64_group<false>(line, 1, t, qq, s, v);
#pragma unroll
  for (int k = 0; k < 4; ++k) line[lane16 + 16 * k] = cmul(v[k], kf[k]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  fft64_group<true>(line, 1, t, qq, s, v);
#pragma unroll
  for (int k = 0; k < 4; ++k) line[lane16 + 16 * k] = v[k];
  __syncthreads();
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int e = tid + BD * n;
    psi[((size_t)(e / W) * ny + j0) * NS + e % W] = A[(e % W) * LS + e / W];
  }
}

// Row pass along a 64-point contiguous axis (SPO3's z lines, psi [rows][64][NS]) with the register transform:
// one 16-lane group per row holding every state of its points, so the point operators are lane-local; 16 rows
// per 256-thread workgroup, each with NS x 64 entries of LDS exchange space.  The row's values come straight
// from global memory in the transform's input layout (lane l = 4 qq + s: points 16 a + 4 s + qq, NS x 16 B
// contiguous per point) and leave in natural order (points l + 16 k).  Same flags as spo2_row_kernel:
// [IFFT] -> V/2 -> [snapshot] -> [V/2] -> [FFT].
template <int NS>
__global__ __launch_bounds__(256) void spo_row64_kernel(c128* psi, const c128* U, const c128* tw_g, int flags,
                                                        c128* snap, const c128* dz = nullptr) {
  __shared__ c128 E[16 * NS * 64];      // per row: [state][64]
  __shared__ c128 tw[64];
  const int tid = threadIdx.x, grp = tid >> 4, lane16 = tid & 15, qq = lane16 >> 2, s = lane16 & 3;
  const size_t row = (size_t)blockIdx.x * 16 + grp;
  c128* pr = psi + row * 64 * NS;
  c128* ex = E + grp * NS * 64;
  c128 x[NS][4];
  const bool inv = flags & ROW_INV;
  // input layout: points 16 a + 4 s + qq (transform input) when the pass starts with the IFFT, else natural
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int p = inv ? 16 * a + 4 * s + qq : lane16 + 16 * a;
#pragma unroll
    for (int c = 0; c < NS; ++c) x[c][a] = pr[p * NS + c];
  }
  if (tid < 64) tw[tid] = tw_g[tid];
  __syncthreads();
  const Q16Tw t = q64_twiddles(tw, qq, s);
  if (inv) {
#pragma unroll
    for (int c = 0; c < NS; ++c) fft64_regs<true>(ex + c * 64, 1, t, qq, s, x[c]);
  }
  // from here the lane holds the points lane16 + 16 k
  if (flags & (ROW_VH1 | ROW_VH2 | ROW_SNAP)) {
    c128 u[4][NS * NS];
    if (flags & (ROW_VH1 | ROW_VH2)) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < NS * NS; ++e) u[k][e] = U[((row * 64) + lane16 + 16 * k) * NS * NS + e];
    }
    auto point_op = [&]() {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c128 q[NS];
#pragma unroll
        for (int a = 0; a < NS; ++a) {
          c128 acc = cmk(0, 0);
#pragma unroll
          for (int b = 0; b < NS; ++b) acc = cadd(acc, cmul(u[k][a * NS + b], x[b][k]));
          q[a] = acc;
        }
#pragma unroll
        for (int a = 0; a < NS; ++a) x[a][k] = q[a];
      }
    };
    if (flags & ROW_VH1) point_op();
    if (flags & ROW_SNAP) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < NS; ++c) snap[(row * 64 + lane16 + 16 * k) * NS + c] = x[c][k];
    }
    if (flags & ROW_VH2) point_op();
  }
  if (flags & ROW_FWD) {
    // natural -> transform input layout through the row's exchange space, then the forward transform
#pragma unroll
    for (int c = 0; c < NS; ++c) {
#pragma unroll
      for (int k = 0; k < 4; ++k) ex[c * 64 + lane16 + 16 * k] = x[c][k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c = 0; c < NS; ++c) fft64_group<false>(ex + c * 64, 1, t, qq, s, x[c]);
    if (flags & ROW_KZ) {   // * e_z / nz, inverse transform: the separable z propagator, natural order out
#pragma unroll
      for (int c = 0; c < NS; ++c) {
#pragma unroll
        for (int k = 0; k < 4; ++k) ex[c * 64 + lane16 + 16 * k] = cmul(x[c][k], dz[lane16 + 16 * k]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NS; ++c) fft64_group<true>(ex + c * 64, 1, t, qq, s, x[c]);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < NS; ++c) pr[(lane16 + 16 * k) * NS + c] = x[c][k];
}

bool pow2_in_range(int n) { return n >= 16 && n <= 1024 && (n & (n - 1)) == 0; }

// L dispatch helpers
#define QD_FFT_DISPATCH(L, CALL) \
  switch (L) {                   \
    case 16: CALL(16); break;    \
    case 32: CALL(32); break;    \
    case 64: CALL(64); break;    \
    case 128: CALL(128); break;  \
    case 256: CALL(256); break;  \
    case 512: CALL(512); break;  \
    case 1024: CALL(1024); break;\
    default: break;              \
  }

int twiddles(int L, hipStream_t st, c128* tw) {
  hipLaunchKernelGGL(twiddle_kernel, dim3((L + 255) / 256), dim3(256), 0, st, L, tw);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

// Launch the latency-shaped row pass (ns <= 2): `rows` rows of length L.
int row_fast(int L, int ns, int rows, int flags, c128* psi, const c128* U, const c128* tw, c128* snap,
             const c128* expKy, hipStream_t st) {
  if (L == 256) {
    const bool ky = (flags & ROW_KY) && expKy;
#define RQ16(NS, KYV) hipLaunchKernelGGL((spo2_row_q16_kernel<NS, KYV>), dim3(rows), dim3(64 * NS), 0, st, psi, U, tw, flags, snap, expKy)
    if (ns == 1) { if (ky) RQ16(1, true); else RQ16(1, false); }
    else { if (ky) RQ16(2, true); else RQ16(2, false); }
#undef RQ16
    QD_HIP(hipGetLastError());
    return QD_OK;
  }
  // L = 64: register transform, 16 lanes per row
  if (L == 64 && rows % 16 == 0 && !(flags & ROW_KY)) {
    if (ns == 1) hipLaunchKernelGGL(spo_row64_kernel<1>, dim3(rows / 16), dim3(256), 0, st, psi, U, tw, flags, snap);
    else hipLaunchKernelGGL(spo_row64_kernel<2>, dim3(rows / 16), dim3(256), 0, st, psi, U, tw, flags, snap);
    QD_HIP(hipGetLastError());
    return QD_OK;
  }
  const int bd = std::max(64, L);
  const size_t lds = (size_t)(L + 2 * ns * L) * sizeof(c128);
#define RF(LL)                                                                                                      \
  if (ns == 1) hipLaunchKernelGGL((spo2_row_fast_kernel<LL, 1>), dim3(rows), dim3(bd), lds, st, psi, U, tw, flags, \
                                  snap, expKy);                                                                     \
  else hipLaunchKernelGGL((spo2_row_fast_kernel<LL, 2>), dim3(rows), dim3(bd), lds, st, psi, U, tw, flags, snap,   \
                          expKy)
  QD_FFT_DISPATCH(L, RF)
#undef RF
  QD_HIP(hipGetLastError());
  return QD_OK;
}

// Latency-shaped column pass (ns <= 2, two columns per workgroup) over `cols` columns of length L;
// `pitch` = points per row of psi.
int col_fast(int L, int ns, int cols, c128* psi, const c128* expKT, const c128* tw, hipStream_t st, int pitch = -1) {
  if (pitch < 0) pitch = cols;
  if (L == 256) {
    if (ns == 1) hipLaunchKernelGGL(spo2_col_q16_kernel<1>, dim3(cols, 1), dim3(64), 0, st, psi, expKT, tw, cols, pitch);
    else hipLaunchKernelGGL(spo2_col_q16_kernel<2>, dim3(cols, 2), dim3(64), 0, st, psi, expKT, tw, cols, pitch);
    QD_HIP(hipGetLastError());
    return QD_OK;
  }
  const int W = 2 * ns;
  const int bd = std::max(64, W * L / 4);
  const size_t lds = (size_t)(L + 2 * W * L) * sizeof(c128);
#define CF(LL)                                                                                                   \
  if (ns == 1) hipLaunchKernelGGL((spo2_col_fast_kernel<LL, 2, 1>), dim3(cols / 2), dim3(bd), lds, st, psi,     \
                                  expKT, tw, pitch);                                                             \
  else hipLaunchKernelGGL((spo2_col_fast_kernel<LL, 2, 2>), dim3(cols / 2), dim3(bd), lds, st, psi, expKT, tw,  \
                          pitch)
  QD_FFT_DISPATCH(L, CF)
#undef CF
  QD_HIP(hipGetLastError());
  return QD_OK;
}

}  // namespace

// d[a][k] = fft(m_a)[k] / n (the axis factor e_a / n of a circulant axis propagator given by its first column)
__global__ void axis_factor_kernel(const c128* m0, const c128* m1, const c128* m2, int n, c128* d) {
  const c128* m = blockIdx.x == 0 ? m0 : blockIdx.x == 1 ? m1 : m2;
  const int k = threadIdx.x;
  if (k >= n) return;
  c128 acc = cmk(0.0, 0.0);
  for (int j = 0; j < n; ++j) {
    double sn, cs;
    sincospi(-2.0 * (double)((j * k) % n) / n, &sn, &cs);
    acc = cadd(acc, cmul(m[j], cmk(cs, sn)));
  }
  d[blockIdx.x * n + k] = cmk(acc.re / n, acc.im / n);
}

// SPO3 on a 64 x 64 x 64 grid with a separable kinetic propagator (qd_spo3_run_axes): three passes per step, each the
// whole axis propagator F^-1 diag(e_a / n) F on its lines with the 64-point register transforms -- z (contiguous,
// with the point operators: the previous step's closing half, the snapshot, this step's opening half), y (mid axis),
// x (columns) -- where the non-separable path needs four (the x pass multiplies the 3-D exp_K between the y and z
// transforms, so both are undone in passes of their own).
int spo3_sep64_run(c128* psi, const c128* Vh, const c128* const m[3], int ns, int nsteps, int nout, c128* snap,
                   hipStream_t st) {
  void* w = nullptr;
  int rc = workspace(WS_SPO, (size_t)4 * 64 * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* tw = (c128*)w;
  c128* d = tw + 64;
  if ((rc = twiddles(64, st, tw))) return rc;
  hipLaunchKernelGGL(axis_factor_kernel, dim3(3), dim3(64), 0, st, m[0], m[1], m[2], 64, d);
  QD_HIP(hipGetLastError());
  const int rows = 64 * 64, nyz = 64 * 64, inner = 64 * ns;
  const size_t grid_elems = (size_t)64 * 64 * 64 * ns;
  auto zpass = [&](int flags, c128* sp) -> int {
    if (ns == 1) hipLaunchKernelGGL(spo_row64_kernel<1>, dim3(rows / 16), dim3(256), 0, st, psi, Vh, tw, flags, sp, d + 128);
    else hipLaunchKernelGGL(spo_row64_kernel<2>, dim3(rows / 16), dim3(256), 0, st, psi, Vh, tw, flags, sp, d + 128);
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  auto ypass = [&]() -> int {
    if (ns == 1) hipLaunchKernelGGL((spo_mid64_kernel<4, false, true>), dim3(64 * (inner / 4)), dim3(64), 0, st, psi, tw, inner, d + 64);
    else hipLaunchKernelGGL((spo_mid64_kernel<8, false, true>), dim3(64 * (inner / 8)), dim3(128), 0, st, psi, tw, inner, d + 64);
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  auto xpass = [&]() -> int {
    if (ns == 1) hipLaunchKernelGGL((spo_col64_kernel<4, 1>), dim3(nyz / 4), dim3(64), 0, st, psi, (const c128*)d, tw, nyz, 0);
    else hipLaunchKernelGGL((spo_col64_kernel<4, 2>), dim3(nyz / 4), dim3(128), 0, st, psi, (const c128*)d, tw, nyz, 0);
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  for (int s = 0; s <= nsteps; ++s) {
    // step s's z pass closes step s - 1 (its snapshot) and opens step s; the pass after the last step only closes
    const bool take = snap && s > 0 && s % nout == 0;
    int flags = (s > 0 ? ROW_VH1 : 0) | (take ? ROW_SNAP : 0);
    if (s < nsteps) flags |= ROW_VH2 | ROW_FWD | ROW_KZ;
    if ((rc = zpass(flags, take ? snap + (size_t)(s / nout - 1) * grid_elems : nullptr))) return rc;
    if (s == nsteps) break;
    if ((rc = ypass())) return rc;
    if ((rc = xpass())) return rc;
  }
  return QD_OK;
}

// spo_gen.hip: every grid the specialised power-of-two kernels below do not cover
int spo_generic_run(c128* psi, const c128* expVh, const c128* expV, const c128* expK, const c128* expKy,
                    const int* dims, int D, int ns, int nsteps, int nout, c128* snap, hipStream_t st);
int spo1d_generic_run(c128* psi, const c128* expV, const c128* expVh, const c128* expK, int nx, int B, int nt,
                      int nout, c128* snap, hipStream_t st);
int spo_expm_run(const void* v, int v_complex, int herm, long npts, int ns, double dt, c128* expV, c128* expVh,
                 hipStream_t st);

}  // namespace qd

using namespace qd;

extern "C" int qd_spo2_run_ex(qd_c128* psi_, const qd_c128* expVh_, const qd_c128* expV_, const qd_c128* expK_,
                              const qd_c128* expKy_, int nx, int ny, int ns, int nsteps, int nout, qd_c128* snap_,
                              void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(psi_ && expVh_ && expK_, "qd_spo2_run_ex: null pointer");
  QD_CHECK_ARG(nx >= 1 && ny >= 1 && ns >= 1, "qd_spo2_run_ex: nx=%d ny=%d ns=%d", nx, ny, ns);
  QD_CHECK_ARG(nsteps >= 0 && nout >= 1, "qd_spo2_run_ex: nsteps=%d nout=%d", nsteps, nout);
  if (nsteps == 0 && !expV_) return QD_OK;
  {
    // the power-of-two LDS / register kernels below: L in [16, 1024], ns <= 8, one transform set per
    // workgroup; every other grid runs the any-size engine (spo_gen.hip)
    const size_t row_lds = (size_t)(ny + 2 * ns * ny) * sizeof(c128), col_lds = (size_t)(nx + 4 * ns * nx) * sizeof(c128);
    const bool special = pow2_in_range(nx) && pow2_in_range(ny) && ns <= SPO_MAX_NS && ns * (ny / 4) <= 256 &&
                         ns * (nx / 4) <= 256 && row_lds <= 160 * 1024 && col_lds <= 160 * 1024;
    note_path(special ? "spo2_pow2" : "spo_any");
    if (!special) {
      const int dims[2] = {nx, ny};
      return spo_generic_run((c128*)psi_, (const c128*)expVh_, (const c128*)expV_, (const c128*)expK_,
                             (const c128*)expKy_, dims, 2, ns, nsteps, nout, (c128*)snap_, (hipStream_t)stream);
    }
  }
  hipStream_t st = (hipStream_t)stream;
  c128* psi = (c128*)psi_;
  const c128* expVh = (const c128*)expVh_;
  c128* snap = (c128*)snap_;
  void* w = nullptr;
  const size_t nkt = (size_t)nx * ny;
  int rc = workspace(WS_SPO, (nkt + nx + ny) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* expKT = (c128*)w;
  c128* twx = expKT + nkt;
  c128* twy = twx + nx;
  if ((rc = twiddles(nx, st, twx))) return rc;
  if ((rc = twiddles(ny, st, twy))) return rc;
  hipLaunchKernelGGL(transpose_scale_kernel, dim3((int)std::min<size_t>((nkt + 255) / 256, 4096)), dim3(256), 0, st,
                     (const c128*)expK_, nx, ny, 1.0 / ((double)nx * ny), expKT);
  QD_HIP(hipGetLastError());

  // column tiling: C columns per workgroup so that C*ns transforms of nx/4 threads fit 256 threads
  int C = std::max(1, 256 / (ns * (nx / 4)));
  while (C > 1 && ny % C) C >>= 1;
  C = std::min(C, 2);  // keep >= ny/2 workgroups in flight
  QD_CHECK_ARG(ns * (nx / 4) <= 256, "qd_spo2_run_ex: ns*nx/4 = %d > 256 threads", ns * (nx / 4));
  const int row_threads = std::max(64, ((ns * (ny / 4) + 63) / 64) * 64);
  const size_t row_lds = (size_t)(ny + 2 * ns * ny) * sizeof(c128);
  const int col_threads = std::max(64, ((C * ns * (nx / 4) + 63) / 64) * 64);
  const size_t col_lds = (size_t)(nx + 2 * C * ns * nx) * sizeof(c128);
  QD_CHECK_ARG(row_lds <= 160 * 1024 && col_lds <= 160 * 1024, "qd_spo2_run_ex: LDS footprint too large");

  const c128* expV = (const c128*)expV_;
  const c128* expKy = (const c128*)expKy_;
  const int ky = expKy ? ROW_KY : 0;
  const bool fast = ns <= 2 && C == 2;
  auto row = [&](int flags, c128* sp, const c128* U) -> int {
    if (fast) return row_fast(ny, ns, nx, flags, psi, U, twy, sp, expKy, st);
#define ROWCALL(L) \
  hipLaunchKernelGGL(spo2_row_kernel<L>, dim3(nx), dim3(row_threads), row_lds, st, psi, U, twy, ny, ns, flags, sp, \
                     expKy)
    QD_FFT_DISPATCH(ny, ROWCALL)
#undef ROWCALL
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  auto col = [&]() -> int {
    if (fast) return col_fast(nx, ns, ny, psi, expKT, twx, st);
#define COLCALL(L)                                                                                                   \
  if (C == 2)                                                                                                        \
    hipLaunchKernelGGL((spo2_col_kernel<L, 2>), dim3(ny / 2), dim3(col_threads), col_lds, st, psi, expKT, twx, ny,   \
                       ns);                                                                                          \
  else                                                                                                               \
    hipLaunchKernelGGL((spo2_col_kernel<L, 1>), dim3(ny), dim3(col_threads), col_lds, st, psi, expKT, twx, ny, ns)
    QD_FFT_DISPATCH(nx, COLCALL)
#undef COLCALL
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  const size_t grid_elems = (size_t)nx * ny * ns;
  if ((rc = row(ROW_VH1 | ROW_FWD | ky, nullptr, expVh))) return rc;
  for (int s = 1; s <= nsteps; ++s) {
    if ((rc = col())) return rc;
    const bool take = snap && (s % nout == 0);
    c128* sp = take ? snap + (size_t)(s / nout - 1) * grid_elems : nullptr;
    int flags = ROW_INV | ROW_VH1 | (take ? ROW_SNAP : 0);
    if (expV) {  // merged: IFFT_y -> V -> [snapshot] -> FFT_y
      flags |= ROW_FWD | ky;
    } else if (s < nsteps) {  // Strang: IFFT_y -> V/2 -> [snapshot] -> V/2 -> FFT_y
      flags |= ROW_VH2 | ROW_FWD | ky;
    }
    if ((rc = row(flags, sp, expV ? expV : expVh))) return rc;
  }
  if (expV) {  // merged tail (wpd.py:752-755): K, then V/2
    if ((rc = col())) return rc;
    if ((rc = row(ROW_INV | ROW_VH1, nullptr, expVh))) return rc;
  }
  return QD_OK;
}

extern "C" int qd_spo2_run(qd_c128* psi_, const qd_c128* expVh_, const qd_c128* expK_, int nx, int ny, int ns,
                           int nsteps, int nout, qd_c128* snap_, void* stream) {
  return qd_spo2_run_ex(psi_, expVh_, nullptr, expK_, nullptr, nx, ny, ns, nsteps, nout, snap_, stream);
}

extern "C" int qd_spo2_run_batch(qd_c128* psi_, int B, const qd_c128* expVh_, const qd_c128* expK_, int nx, int ny,
                                 int ns, int nsteps, int nout, qd_c128* snap_, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(psi_ && expVh_ && expK_, "qd_spo2_run_batch: null pointer");
  QD_CHECK_ARG(B >= 1 && B <= 65535, "qd_spo2_run_batch: B=%d outside [1, 65535]", B);
  QD_CHECK_ARG(nsteps >= 0 && nout >= 1, "qd_spo2_run_batch: nsteps=%d nout=%d", nsteps, nout);
  const size_t grid_elems = (size_t)nx * ny * ns;
  const int nsave = nsteps / nout;
  if (!(nx == 256 && ny == 256 && ns <= 2)) {
    // other shapes: one member at a time on the single-wavefunction path
    for (int w = 0; w < B; ++w) {
      const int rc = qd_spo2_run_ex(psi_ + w * grid_elems, expVh_, nullptr, expK_, nullptr, nx, ny, ns, nsteps, nout,
                                    snap_ ? snap_ + (size_t)w * nsave * grid_elems : nullptr, stream);
      if (rc) return rc;
    }
    return QD_OK;
  }
  if (nsteps == 0) return QD_OK;
  hipStream_t st = (hipStream_t)stream;
  c128* psi = (c128*)psi_;
  const c128* U = (const c128*)expVh_;
  c128* snap = (c128*)snap_;
  void* w = nullptr;
  const size_t nkt = (size_t)nx * ny;
  int rc = workspace(WS_SPO, (nkt + nx + ny) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* expKT = (c128*)w;
  c128* twx = expKT + nkt;
  c128* twy = twx + nx;
  if ((rc = twiddles(nx, st, twx))) return rc;
  if ((rc = twiddles(ny, st, twy))) return rc;
  hipLaunchKernelGGL(transpose_scale_kernel, dim3((int)std::min<size_t>((nkt + 255) / 256, 4096)), dim3(256), 0, st,
                     (const c128*)expK_, nx, ny, 1.0 / ((double)nx * ny), expKT);
  QD_HIP(hipGetLastError());
  const size_t sstride = (size_t)nsave * grid_elems;
  // ns = 2: a wave per member, 4 members per workgroup sharing the staged point operators (64 wavepackets: 476k
  // wavepacket-steps/s against 428k for 2-member groups of the single-row kernel); the column pass in tiles of 8
  // columns (503k against 477k for 4)
  note_path("spo2_batch256");
  auto row = [&](int flags, c128* sp) {
    if (ns == 1)
      hipLaunchKernelGGL((spo2_row_q16_kernel<1, false>), dim3(nx, B), dim3(64), 0, st, psi, U, twy, flags, sp,
                         (const c128*)nullptr, grid_elems, sstride);
    else
      hipLaunchKernelGGL(spo2_row_wave_kernel<4>, dim3(nx, (B + 3) / 4), dim3(256), 0, st, psi, U, twy, flags, sp, B,
                         grid_elems, sstride);
  };
  auto col = [&]() {
    if (ns == 1)
      hipLaunchKernelGGL(spo2_col_q16_kernel<1>, dim3(ny, 1, B), dim3(64), 0, st, psi, (const c128*)expKT,
                         (const c128*)twx, ny, ny, grid_elems);
    else
      hipLaunchKernelGGL(spo2_col_tile8_kernel<8>, dim3(ny / 8, B), dim3(512), 0, st, psi, (const c128*)expKT,
                         (const c128*)twx, grid_elems);
  };
  // the Strang step sequence of qd_spo2_run_ex (both V/2 halves, wpd.py:723-730)
  row(ROW_VH1 | ROW_FWD, nullptr);
  QD_HIP(hipGetLastError());
  for (int s = 1; s <= nsteps; ++s) {
    col();
    QD_HIP(hipGetLastError());
    const bool take = snap && (s % nout == 0);
    c128* sp = take ? snap + (size_t)(s / nout - 1) * grid_elems : nullptr;
    row(ROW_INV | ROW_VH1 | (take ? ROW_SNAP : 0) | (s < nsteps ? ROW_VH2 | ROW_FWD : 0), sp);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}

extern "C" int qd_spo1d_run(qd_c128* psi_, const qd_c128* expV_, const qd_c128* expVh_, const qd_c128* expK_, int nx,
                            int B, int nt, int nout, qd_c128* snap_, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(psi_ && expV_ && expVh_ && expK_, "qd_spo1d_run: null pointer");
  QD_CHECK_ARG(nx >= 1 && B >= 1 && nt >= 0 && nout >= 1, "qd_spo1d_run: nx=%d B=%d nt=%d nout=%d", nx, B, nt, nout);
  note_path(pow2_in_range(nx) ? "spo1d_pow2" : "spo_any");
  if (!pow2_in_range(nx))
    return spo1d_generic_run((c128*)psi_, (const c128*)expV_, (const c128*)expVh_, (const c128*)expK_, nx, B, nt, nout,
                             (c128*)snap_, (hipStream_t)stream);
  hipStream_t st = (hipStream_t)stream;
  void* w = nullptr;
  int rc = workspace(WS_MISC, nx * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* tw = (c128*)w;
  if ((rc = twiddles(nx, st, tw))) return rc;
  const int threads = std::max(64, nx / 4);
#define CALL1D(L)                                                                                                   \
  hipLaunchKernelGGL(spo1d_kernel<L>, dim3(B), dim3(threads), 0, st, (c128*)psi_, (const c128*)expV_,               \
                     (const c128*)expVh_, (const c128*)expK_, (const c128*)tw, nt, nout, (c128*)snap_)
  QD_FFT_DISPATCH(nx, CALL1D)
#undef CALL1D
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_spo3_run(qd_c128* psi_, const qd_c128* expVh_, const qd_c128* expK_, int nx, int ny, int nz, int ns,
                           int nsteps, int nout, qd_c128* snap_, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(psi_ && expVh_ && expK_, "qd_spo3_run: null pointer");
  QD_CHECK_ARG(nx >= 1 && ny >= 1 && nz >= 1 && ns >= 1, "qd_spo3_run: nx=%d ny=%d nz=%d ns=%d", nx, ny, nz, ns);
  QD_CHECK_ARG(nsteps >= 0 && nout >= 1, "qd_spo3_run: nsteps=%d nout=%d", nsteps, nout);
  if (nsteps == 0) return QD_OK;
  {
    const size_t row_lds = (size_t)(nz + 2 * ns * nz) * sizeof(c128), col_lds = (size_t)(nx + 4 * ns * nx) * sizeof(c128);
    const bool special = pow2_in_range(nx) && pow2_in_range(ny) && pow2_in_range(nz) && nx <= 256 && ny <= 256 &&
                         nz <= 256 && ns <= SPO_MAX_NS && ns * (nz / 4) <= 256 && ns * (nx / 4) <= 256 &&
                         row_lds <= 160 * 1024 && col_lds <= 160 * 1024;
    note_path(special ? "spo3_pow2" : "spo_any");
    if (!special) {
      const int dims[3] = {nx, ny, nz};
      return spo_generic_run((c128*)psi_, (const c128*)expVh_, nullptr, (const c128*)expK_, nullptr, dims, 3, ns,
                             nsteps, nout, (c128*)snap_, (hipStream_t)stream);
    }
  }
  hipStream_t st = (hipStream_t)stream;
  c128* psi = (c128*)psi_;
  const c128* expVh = (const c128*)expVh_;
  c128* snap = (c128*)snap_;
  const int nyz = ny * nz;
  const size_t nk = (size_t)nx * nyz;
  void* w = nullptr;
  int rc = workspace(WS_SPO, (nk + nx + ny + nz) * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* expKT = (c128*)w;
  c128* twx = expKT + nk;
  c128* twy = twx + nx;
  c128* twz = twy + ny;
  if ((rc = twiddles(nx, st, twx))) return rc;
  if ((rc = twiddles(ny, st, twy))) return rc;
  if ((rc = twiddles(nz, st, twz))) return rc;
  hipLaunchKernelGGL(transpose_scale_kernel, dim3((int)std::min<size_t>((nk + 255) / 256, 4096)), dim3(256), 0, st,
                     (const c128*)expK_, nx, nyz, 1.0 / ((double)nx * ny * nz), expKT);
  QD_HIP(hipGetLastError());
  // z pass: rows = nx*ny, length nz (contiguous, fused V/2); x pass: columns = ny*nz
  const int row_threads = std::max(64, ((ns * (nz / 4) + 63) / 64) * 64);
  const size_t row_lds = (size_t)(nz + 2 * ns * nz) * sizeof(c128);
  const int col_threads = std::max(64, ((2 * ns * (nx / 4) + 63) / 64) * 64);
  const size_t col_lds = (size_t)(nx + 2 * 2 * ns * nx) * sizeof(c128);
  const int inner = nz * ns;
  const bool fast = ns <= 2;
  auto row = [&](int flags, c128* sp) -> int {
    if (fast) return row_fast(nz, ns, nx * ny, flags, psi, expVh, twz, sp, nullptr, st);
#define ROWCALL3(L) \
  hipLaunchKernelGGL(spo2_row_kernel<L>, dim3(nx * ny), dim3(row_threads), row_lds, st, psi, expVh, twz, nz, ns, flags, sp, \
                     (const c128*)nullptr)
    QD_FFT_DISPATCH(nz, ROWCALL3)
#undef ROWCALL3
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  // Mid pass: C consecutive inner indices (C * 16 B per row read) per block. C is the largest of
  // 16 / 8 / 4 that still gives >= 4 blocks per CU (on its own worth ~1% at 64^3 x 2: 512 -> 1024
  // blocks; C = 4 costs 13% at 128^3; tools/spo3_midc_sweep.sh).
  int midC = 4;
  for (int c : {16, 8}) {
    if (c * ny <= 1024 && inner % c == 0 && (size_t)nx * (inner / c) >= 1024) { midC = c; break; }
  }
  while (midC > 1 && inner % midC) midC >>= 1;  // inner = nz * ns >= 16 keeps midC >= 4
  // x pass: the latency-shaped two-column kernel (colC = 0), or the LDS-staged kernel over colC
  // columns x ns states per block (colC * ns * 16 B contiguous per row).
  // Default: at <= 64^3 x 2 points and midC >= 8 the LDS-staged kernel with the mid pass's row width
  // (colC * ns == midC, 128 B rows at 64^3 x 2: 41.1 -> 33.4 us per step); above that the
  // two-column kernel (128^3 x 2: 142 us either way, 146 us with colC * ns == midC).
  int colC = 0;
  // (nx <= 64: the LDS-staged x kernels are instantiated for 16 / 32 / 64-point columns)
  if (nk * ns <= (size_t)1 << 19 && midC >= 8 && midC % ns == 0 && nx <= 64) {  // 32^3 x 2 (midC = 4): 15.4 vs 16.6 us
    const int c = midC / ns;
    if ((c == 2 || c == 4 || c == 8) && nyz % c == 0 && c * ns * (nx / 4) <= 256) colC = c;
  }
  auto col = [&]() -> int {
    if (colC && fast && nx == 64) {
#define COL64(CC)                                                                                                    \
  if (ns == 1) hipLaunchKernelGGL((spo_col64_kernel<CC, 1>), dim3(nyz / CC), dim3(16 * CC), 0, st, psi, expKT, twx, nyz); \
  else hipLaunchKernelGGL((spo_col64_kernel<CC, 2>), dim3(nyz / CC), dim3(32 * CC), 0, st, psi, expKT, twx, nyz)
      if (colC == 2) { COL64(2); } else if (colC == 4) { COL64(4); } else { COL64(8); }
#undef COL64
      QD_HIP(hipGetLastError());
      return QD_OK;
    }
    if (colC && fast) {
      const int threads = std::max(64, colC * ns * (nx / 4));
      const size_t lds = (size_t)(nx + 2 * colC * ns * nx) * sizeof(c128);
#define COLFASTC(L)                                                                                                       if (colC == 2) { if (ns == 1) hipLaunchKernelGGL((spo2_col_fast_kernel<L, 2, 1>), dim3(nyz / 2), dim3(threads), lds, st, psi, expKT, twx, nyz);                    else hipLaunchKernelGGL((spo2_col_fast_kernel<L, 2, 2>), dim3(nyz / 2), dim3(threads), lds, st, psi, expKT, twx, nyz); }   else if (colC == 4) { if (ns == 1) hipLaunchKernelGGL((spo2_col_fast_kernel<L, 4, 1>), dim3(nyz / 4), dim3(threads), lds, st, psi, expKT, twx, nyz);                    else hipLaunchKernelGGL((spo2_col_fast_kernel<L, 4, 2>), dim3(nyz / 4), dim3(threads), lds, st, psi, expKT, twx, nyz); }   else { if (ns == 1) hipLaunchKernelGGL((spo2_col_fast_kernel<L, 8, 1>), dim3(nyz / 8), dim3(threads), lds, st, psi, expKT, twx, nyz);          else hipLaunchKernelGGL((spo2_col_fast_kernel<L, 8, 2>), dim3(nyz / 8), dim3(threads), lds, st, psi, expKT, twx, nyz); }
      switch (nx) {
        case 16: COLFASTC(16); break;
        case 32: COLFASTC(32); break;
        case 64: COLFASTC(64); break;
        default:   // colC is set only for nx <= 64
          set_error("qd_spo3_run: internal: column tile for nx = %d", nx);
          return QD_EINVAL;
      }
#undef COLFASTC
      QD_HIP(hipGetLastError());
      return QD_OK;
    }
    if (colC) {
      const int threads = std::max(64, colC * ns * (nx / 4));
      const size_t lds = (size_t)(nx + 2 * colC * ns * nx) * sizeof(c128);
#define COLCALLC(L)                                                                                                   \
  if (colC == 2) hipLaunchKernelGGL((spo2_col_kernel<L, 2>), dim3(nyz / 2), dim3(threads), lds, st, psi, expKT, twx, nyz, ns); \
  else if (colC == 4) hipLaunchKernelGGL((spo2_col_kernel<L, 4>), dim3(nyz / 4), dim3(threads), lds, st, psi, expKT, twx, nyz, ns); \
  else hipLaunchKernelGGL((spo2_col_kernel<L, 8>), dim3(nyz / 8), dim3(threads), lds, st, psi, expKT, twx, nyz, ns)
      QD_FFT_DISPATCH(nx, COLCALLC)
#undef COLCALLC
      QD_HIP(hipGetLastError());
      return QD_OK;
    }
    if (fast) return col_fast(nx, ns, nyz, psi, expKT, twx, st);
#define COLCALL3(L) \
  hipLaunchKernelGGL((spo2_col_kernel<L, 2>), dim3(nyz / 2), dim3(col_threads), col_lds, st, psi, expKT, twx, nyz, ns)
    QD_FFT_DISPATCH(nx, COLCALL3)
#undef COLCALL3
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  auto mid = [&](bool inv) -> int {
    const int grid = nx * (inner / midC);
    const int threads = std::max(64, midC * (ny / 4));
    if (ny == 64) {
#define MID64(C)                                                                                                  \
  if (inv) hipLaunchKernelGGL((spo_mid64_kernel<C, true>), dim3(grid), dim3(16 * C), 0, st, psi, twy, inner); \
  else hipLaunchKernelGGL((spo_mid64_kernel<C, false>), dim3(grid), dim3(16 * C), 0, st, psi, twy, inner)
      if (midC == 16) { MID64(16); } else if (midC == 8) { MID64(8); } else { MID64(4); }
#undef MID64
      QD_HIP(hipGetLastError());
      return QD_OK;
    }
    if (midC * ny / 4 <= 256 && ny <= 64) {
#define MIDF_C(L, C)                                                                                               \
  if (inv) hipLaunchKernelGGL((spo_mid_fast_kernel<L, C, true>), dim3(grid), dim3(threads), 0, st, psi, twy, inner); \
  else hipLaunchKernelGGL((spo_mid_fast_kernel<L, C, false>), dim3(grid), dim3(threads), 0, st, psi, twy, inner)
#define MIDF(L)                          \
  if (midC == 16) { MIDF_C(L, 16); }     \
  else if (midC == 8) { MIDF_C(L, 8); }  \
  else { MIDF_C(L, 4); }
      switch (ny) {
        case 16: MIDF(16); break;
        case 32: MIDF(32); break;
        default: MIDF(64); break;
      }
#undef MIDF
#undef MIDF_C
      QD_HIP(hipGetLastError());
      return QD_OK;
    }
#define MIDCALL_C(L, C)                                                                                      \
  if (inv) hipLaunchKernelGGL((spo_mid_kernel<L, C, true>), dim3(grid), dim3(threads), 0, st, psi, twy, inner); \
  else hipLaunchKernelGGL((spo_mid_kernel<L, C, false>), dim3(grid), dim3(threads), 0, st, psi, twy, inner)
#define MIDCALL(L)                   \
  if (midC == 16) { MIDCALL_C(L, 16); } \
  else if (midC == 8) { MIDCALL_C(L, 8); } \
  else { MIDCALL_C(L, 4); }
    switch (ny) {
      case 16: MIDCALL(16); break;
      case 32: MIDCALL(32); break;
      case 64: MIDCALL(64); break;
      case 128: if (midC >= 8) { MIDCALL_C(128, 8); } else { MIDCALL_C(128, 4); } break;
      case 256: { MIDCALL_C(256, 4); } break;
    }
#undef MIDCALL
#undef MIDCALL_C
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  const size_t grid_elems = nk * ns;
  if ((rc = row(ROW_VH1 | ROW_FWD, nullptr))) return rc;
  if ((rc = mid(false))) return rc;
  for (int s = 1; s <= nsteps; ++s) {
    if ((rc = col())) return rc;
    if ((rc = mid(true))) return rc;
    const bool take = snap && (s % nout == 0);
    c128* sp = take ? snap + (size_t)(s / nout - 1) * grid_elems : nullptr;
    int flags = ROW_INV | ROW_VH1 | (take ? ROW_SNAP : 0);
    if (s < nsteps) flags |= ROW_VH2 | ROW_FWD;
    if ((rc = row(flags, sp))) return rc;
    if (s < nsteps && (rc = mid(false))) return rc;
  }
  return QD_OK;
}

extern "C" int qd_spo_expv(const void* v, int v_complex, long npts, int ns, double dt, qd_c128* expV_,
                           qd_c128* expVh_, void* stream) {
  QD_CHECK_ARG(v && expVh_, "qd_spo_expv: null pointer");
  QD_CHECK_ARG(ns >= 1 && ns <= 1024, "qd_spo_expv: ns=%d outside [1, 1024]", ns);
  QD_CHECK_ARG(npts >= 0, "qd_spo_expv: npts=%ld", npts);
  if (npts == 0) return QD_OK;
  if (ns > 2)   // scaling-and-squaring Taylor exponential of the Hermitian matrix eigh reads (spo_gen.hip)
    return spo_expm_run(v, v_complex, 1, npts, ns, dt, (c128*)expV_, (c128*)expVh_, (hipStream_t)stream);
  const int grid = (int)std::min<long>((npts + 255) / 256, 8192);
  if (v_complex)
    hipLaunchKernelGGL(spo_expv_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, v, npts, ns, dt,
                       (c128*)expV_, (c128*)expVh_);
  else
    hipLaunchKernelGGL(spo_expv_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, v, npts, ns, dt,
                       (c128*)expV_, (c128*)expVh_);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_spo_expm(const qd_c128* v, int hermitian, long npts, int ns, double dt, qd_c128* expV_,
                           qd_c128* expVh_, void* stream) {
  QD_CHECK_ARG(v && expVh_, "qd_spo_expm: null pointer");
  QD_CHECK_ARG(ns >= 1 && ns <= 1024, "qd_spo_expm: ns=%d outside [1, 1024]", ns);
  QD_CHECK_ARG(npts >= 0, "qd_spo_expm: npts=%ld", npts);
  if (npts == 0) return QD_OK;
  return spo_expm_run(v, 1, hermitian ? 1 : 0, npts, ns, dt, (c128*)expV_, (c128*)expVh_, (hipStream_t)stream);
}
