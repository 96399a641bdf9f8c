// krylov.hip — the Arnoldi projections and the shifted Hessenberg solves of the multi-shift Krylov form of
// DEOMSolver.correlation_4op_3t (pyqed_amd/deom_krylov.py; reference heom/deom.py:1127-1209 diagonalises P instead).
//
// For every shift s: (-H_k - s I) y = beta e_1 with H_k the k x k upper Hessenberg Arnoldi matrix (leading dimension
// ldh, row k holding h_{k+1,k}).  One workgroup per shift runs Gaussian elimination with adjacent-row pivoting (the
// only rows that can pivot in a Hessenberg matrix), keeping the active row in LDS and storing the pivot rows (U) to
// scratch, then column-oriented back substitution; the FOM residual |h_{k+1,k} y_{k-1}| / beta comes out of the
// elimination's last pivot.  Replaces a host loop (O(S k^2) numpy steps per checkpoint) and a device loop of ~10
// small launches per row.
#include "qd_common.hpp"

namespace qd {
namespace {

__device__ __forceinline__ double cabs2(c128 a) { return a.re * a.re + a.im * a.im; }
__device__ __forceinline__ c128 cdiv(c128 a, c128 b) {
  const double d = b.re * b.re + b.im * b.im;
  return cmk((a.re * b.re + a.im * b.im) / d, (a.im * b.re - a.re * b.im) / d);
}

// dynamic LDS: cur[k], nxt[k] (nxt reused as the right-hand side during the back substitution)
__global__ __launch_bounds__(256) void hess_shift_kernel(const c128* __restrict__ H, int ldh, int k,
                                                         const c128* __restrict__ shifts, double beta, c128* Y,
                                                         double* res, c128* U) {
  extern __shared__ c128 sh[];
  c128* cur = sh;
  c128* nxt = sh + k;
  __shared__ c128 s_m, s_g;
  __shared__ int s_swap;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int b = blockIdx.x;
  const c128 sft = shifts[b];
  c128* Ub = U ? U + (size_t)b * k * k : nullptr;
  for (int l = tid; l < k; l += nt) {
    const c128 h = H[l];
    cur[l] = cmk(-h.re - (l == 0 ? sft.re : 0.0), -h.im - (l == 0 ? sft.im : 0.0));
  }
  c128 g = cmk(beta, 0.0);   // the active row's right-hand side (uniform across the workgroup)
  __syncthreads();
  for (int j = 0; j + 1 < k; ++j) {
    const c128* hr = H + (size_t)(j + 1) * ldh;
    for (int l = j + tid; l < k; l += nt) {
      const c128 h = hr[l];
      nxt[l] = cmk(-h.re - (l == j + 1 ? sft.re : 0.0), -h.im - (l == j + 1 ? sft.im : 0.0));
    }
    __syncthreads();
    if (tid == 0) {
      const bool swap = cabs2(nxt[j]) > cabs2(cur[j]);
      const c128 piv = swap ? nxt[j] : cur[j], oth = swap ? cur[j] : nxt[j];
      s_swap = swap;
      s_m = cdiv(oth, piv);
    }
    __syncthreads();
    const bool swap = s_swap;
    const c128 m = s_m;
    // pivot row -> U row j, active row <- other - m pivot (columns l > j)
    for (int l = j + tid; l < k; l += nt) {
      const c128 pv = swap ? nxt[l] : cur[l], ov = swap ? cur[l] : nxt[l];
      if (Ub) Ub[(size_t)j * k + l] = pv;
      if (l > j) cur[l] = csub(ov, cmul(m, pv));
    }
    // right-hand side: the pivot row's entry (g if the active row pivots, 0 for the fresh row), the other's
    const c128 gp = swap ? cmk(0.0, 0.0) : g, go = swap ? g : cmk(0.0, 0.0);
    if (Ub && tid == 0) nxt[j] = gp;   // nxt[0..j] is free from here on: the pivot rows' right-hand sides
    g = csub(go, cmul(m, gp));
    __syncthreads();
  }
  const c128 last = cur[k - 1];
  const c128 yk = cdiv(g, last);
  if (tid == 0 && res) {
    const c128 hk = H[(size_t)k * ldh + (k - 1)];
    res[b] = sqrt(cabs2(cmul(hk, yk))) / beta;
  }
  if (!Y) return;
  // back substitution, column by column: y_i = r_i / U_ii, then r_l -= U_li y_i for l < i
  if (tid == 0) {
    Ub[(size_t)(k - 1) * k + (k - 1)] = last;
    nxt[k - 1] = g;
  }
  __syncthreads();
  c128* Yb = Y + (size_t)b * k;
  for (int i = k - 1; i >= 0; --i) {
    const c128 yi = cdiv(nxt[i], Ub[(size_t)i * k + i]);
    if (tid == 0) Yb[i] = yi;
    for (int l = tid; l < i; l += nt) nxt[l] = csub(nxt[l], cmul(Ub[(size_t)l * k + i], yi));
    __syncthreads();
  }
}

// h[r] = sum_i conj(V[r][i]) w[i] for r < m, one workgroup per basis row (contiguous, coalesced), fixed-order
// reduction (deterministic); hsum (strided by ldh, or null) accumulates the same value (the Hessenberg column).
__global__ __launch_bounds__(256) void cgs_project_kernel(const c128* __restrict__ V, long ldv, int n,
                                                          const c128* __restrict__ w, c128* h, c128* hsum, long ldh) {
  __shared__ double red[2][256];
  const int r = blockIdx.x, tid = threadIdx.x;
  const c128* vr = V + (size_t)r * ldv;
  double sr = 0.0, si = 0.0;
  constexpr int U = 8;   // loads in flight per thread (the row is one dependent-latency chain otherwise)
  int i = tid;
  for (; i + 256 * (U - 1) < n; i += 256 * U) {
    c128 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = vr[i + 256 * u];
      b[u] = w[i + 256 * u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      sr += a[u].re * b[u].re + a[u].im * b[u].im;   // conj(a) b
      si += a[u].re * b[u].im - a[u].im * b[u].re;
    }
  }
  for (; i < n; i += 256) {
    const c128 a = vr[i], b = w[i];
    sr += a.re * b.re + a.im * b.im;
    si += a.re * b.im - a.im * b.re;
  }
  red[0][tid] = sr;
  red[1][tid] = si;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const c128 v = cmk(red[0][0], red[1][0]);
    h[r] = v;
    if (hsum) hsum[(size_t)r * ldh] = cadd(hsum[(size_t)r * ldh], v);
  }
}

// ||w||^2 in two fixed-order stages: per-workgroup partial sums, then one workgroup sums them, writes *hsub = nrm and
// (with the other workgroups of the scale launch) v = w / max(nrm, 1e-300)
constexpr int NRM_WG = 64;
__global__ __launch_bounds__(256) void cgs_norm_partial_kernel(const c128* __restrict__ w, int n, double* part) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int i = blockIdx.x * 256 + tid; i < n; i += NRM_WG * 256) {
    const c128 a = w[i];
    s += a.re * a.re + a.im * a.im;
  }
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void cgs_norm_scale_kernel(const c128* __restrict__ w, int n, const double* part,
                                                             c128* v, c128* hsub) {
  double s = 0.0;
  for (int q = 0; q < NRM_WG; ++q) s += part[q];   // same order in every workgroup
  const double nrm = sqrt(s);
  if (blockIdx.x == 0 && threadIdx.x == 0) *hsub = cmk(nrm, 0.0);
  const double inv = 1.0 / fmax(nrm, 1e-300);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const c128 a = w[i];
    v[i] = cmk(a.re * inv, a.im * inv);
  }
}

constexpr int DCGS_MAX_SLICES = 8;   // column slices of the projection pass (st holds 2 (j + 1) DCGS_MAX_SLICES)

// ---- delayed CGS2 Arnoldi step (two passes over the basis per step instead of CGS2's four) --------------------------
// State entering step j: V[0..j-1] final orthonormal, V[j] = u_j the candidate after ONE projection (unnormalised),
// z = P u_j, Hessenberg columns 0..j-2 final, column j-1 holding the first-pass coefficients.  One projection pass
// gives s = V_j^H u_j (the reorthogonalisation of u_j), t = V_j^H z, alpha = |u_j|^2, gamma = u_j^H z; then
//   rho = sqrt(alpha - |s|^2), v_j = (u_j - V_j s) / rho, column j-1 += s, h_{j,j-1} = rho,
//   P v_j = (z - V_j H_j s - v_j rho s_{j-1}) / rho   (Arnoldi relation P V_j = V_{j+1} Hbar_j),
//   first-pass coefficients of column j: a_r = (t_r - (H_j s)_r) / rho (r < j), a_j = ((gamma - s^H t)/rho - rho s_{j-1})/rho,
//   u_{j+1} = z / rho - V_j c - v_j d with c = H_j s / rho + a_{<j}, d = s_{j-1} + a_j
// and one update pass writes v_j and u_{j+1}.  Step 0 starts from V[0] = b (j = 0: no basis, rho = |b|).

// partial dot products over column slice g of S: st[(2r) S + g] = conj(V[r]) . V[j], st[(2r+1) S + g] = conj(V[r]) . z
// for r <= j (row j: alpha, gamma); S slices per row keep ~4 workgroups per CU busy at small j
__global__ __launch_bounds__(256) void dcgs_project_kernel(const c128* __restrict__ V, long ldv, int j, int n,
                                                           const c128* __restrict__ z, c128* st) {
  __shared__ double red[4][256];
  const int r = blockIdx.x, tid = threadIdx.x, g = blockIdx.y, S = gridDim.y;
  const int c0 = (int)((long)n * g / S), c1 = (int)((long)n * (g + 1) / S);
  const c128* vr = V + (size_t)r * ldv + c0;
  const c128* u = V + (size_t)j * ldv + c0;
  z += c0;
  n = c1 - c0;
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
  constexpr int U = 6;
  int i = tid;
  for (; i + 256 * (U - 1) < n; i += 256 * U) {
    c128 a[U], x[U], y[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      a[q] = vr[i + 256 * q];
      x[q] = u[i + 256 * q];
      y[q] = z[i + 256 * q];
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      a0 += a[q].re * x[q].re + a[q].im * x[q].im;
      a1 += a[q].re * x[q].im - a[q].im * x[q].re;
      b0 += a[q].re * y[q].re + a[q].im * y[q].im;
      b1 += a[q].re * y[q].im - a[q].im * y[q].re;
    }
  }
  for (; i < n; i += 256) {
    const c128 a = vr[i], x = u[i], y = z[i];
    a0 += a.re * x.re + a.im * x.im;
    a1 += a.re * x.im - a.im * x.re;
    b0 += a.re * y.re + a.im * y.im;
    b1 += a.re * y.im - a.im * y.re;
  }
  red[0][tid] = a0;
  red[1][tid] = a1;
  red[2][tid] = b0;
  red[3][tid] = b1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
#pragma unroll
      for (int c = 0; c < 4; ++c) red[c][tid] += red[c][tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    st[(size_t)(2 * r) * S + g] = cmk(red[0][0], red[1][0]);
    st[(size_t)(2 * r + 1) * S + g] = cmk(red[2][0], red[3][0]);
  }
}

// the S partial sums of entry e, in slice order (every reader gets the same value)
__device__ __forceinline__ c128 st_sum(const c128* st, int S, int e) {
  c128 a = st[(size_t)e * S];
  for (int g = 1; g < S; ++g) a = cadd(a, st[(size_t)e * S + g]);
  return a;
}

// one wave per Hessenberg row r < j (4 per workgroup); every workgroup recomputes |s|^2 and s^H t in the same order.
// cs[r] = c_r (r < j), cs[j] = d, cs[j+1] = (1/rho, 0), cs[j+2+r] = s_r; rho = 0 (exact breakdown) zeroes v_j,
// u_{j+1} and column j.
__global__ __launch_bounds__(256) void dcgs_coef_kernel(c128* H, long ldh, int j, const c128* __restrict__ st, int S,
                                                        c128* cs) {
  __shared__ double red[3][256];
  extern __shared__ c128 s_sh[];   // s summed over the slices, j entries (dynamic)
  const int tid = threadIdx.x;
  double ss = 0.0, p0 = 0.0, p1 = 0.0;
  for (int r = tid; r < j; r += 256) {
    const c128 s = st_sum(st, S, 2 * r), t = st_sum(st, S, 2 * r + 1);
    s_sh[r] = s;
    ss += s.re * s.re + s.im * s.im;
    p0 += s.re * t.re + s.im * t.im;   // conj(s) t
    p1 += s.re * t.im - s.im * t.re;
  }
  red[0][tid] = ss;
  red[1][tid] = p0;
  red[2][tid] = p1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
      red[2][tid] += red[2][tid + o];
    }
    __syncthreads();
  }
  const double rho2 = st_sum(st, S, 2 * j).re - red[0][0];
  const double rho = rho2 > 0.0 ? sqrt(rho2) : 0.0;
  const bool zero = !(rho > 1e-300);
  const double inv = zero ? 0.0 : 1.0 / rho;
  const c128 sl = j > 0 ? s_sh[j - 1] : cmk(0.0, 0.0);
  const int lane = tid & 63;
  const int r = blockIdx.x * 4 + (tid >> 6);
  if (r < j) {
    // (H_j s)_r over the final columns: column j-1 is its first-pass value plus s_r
    double h0 = 0.0, h1 = 0.0;
    c128* hr = H + (size_t)r * ldh;
    const c128 sr = s_sh[r];
    for (int c = (r > 0 ? r - 1 : 0) + lane; c < j; c += 64) {
      c128 h = hr[c];
      if (c == j - 1) h = cadd(h, sr);
      const c128 s = s_sh[c];
      h0 += h.re * s.re - h.im * s.im;
      h1 += h.re * s.im + h.im * s.re;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      h0 += __shfl_xor(h0, o);
      h1 += __shfl_xor(h1, o);
    }
    if (lane == 0) {
      const c128 hs = cmk(h0, h1);
      const c128 a = zero ? cmk(0.0, 0.0) : cscale(csub(st_sum(st, S, 2 * r + 1), hs), inv);
      hr[j - 1] = cadd(hr[j - 1], sr);
      hr[j] = a;
      cs[r] = zero ? cmk(0.0, 0.0) : cadd(cscale(hs, inv), a);
      cs[j + 2 + r] = sr;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    const c128 gam = st_sum(st, S, 2 * j + 1);
    const c128 sht = cmk(red[1][0], red[2][0]);
    const c128 aj = zero ? cmk(0.0, 0.0) : cscale(csub(cscale(csub(gam, sht), inv), cscale(sl, rho)), inv);
    if (j > 0) H[(size_t)j * ldh + (j - 1)] = cmk(rho, 0.0);
    H[(size_t)j * ldh + j] = aj;
    cs[j] = zero ? cmk(0.0, 0.0) : cadd(sl, aj);
    cs[j + 1] = cmk(inv, 0.0);
  }
}

// partial sums over a slice of the basis rows: part[g][i] = (sum_r V[r][i] s_r, sum_r V[r][i] c_r)
__global__ __launch_bounds__(256) void dcgs_update_partial_kernel(const c128* __restrict__ V, long ldv, int j, int n,
                                                                  const c128* __restrict__ cs, c128* part) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y, G = gridDim.y;
  const int r0 = (int)((long)j * g / G), r1 = (int)((long)j * (g + 1) / G);
  if (i >= n) return;
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
  constexpr int U = 8;
  int r = r0;
  for (; r + U <= r1; r += U) {
    c128 v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = V[(size_t)(r + q) * ldv + i];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const c128 s = cs[j + 2 + r + q], c = cs[r + q];
      a0 += v[q].re * s.re - v[q].im * s.im;
      a1 += v[q].re * s.im + v[q].im * s.re;
      b0 += v[q].re * c.re - v[q].im * c.im;
      b1 += v[q].re * c.im + v[q].im * c.re;
    }
  }
  for (; r < r1; ++r) {
    const c128 v = V[(size_t)r * ldv + i], s = cs[j + 2 + r], c = cs[r];
    a0 += v.re * s.re - v.im * s.im;
    a1 += v.re * s.im + v.im * s.re;
    b0 += v.re * c.re - v.im * c.im;
    b1 += v.re * c.im + v.im * c.re;
  }
  part[((size_t)g * n + i) * 2] = cmk(a0, a1);
  part[((size_t)g * n + i) * 2 + 1] = cmk(b0, b1);
}

// v_j = (u_j - V s) / rho into V[j], u_{j+1} = z / rho - V c - v_j d into V[j+1]
__global__ __launch_bounds__(256) void dcgs_update_final_kernel(c128* V, long ldv, int j, int n,
                                                                const c128* __restrict__ z,
                                                                const c128* __restrict__ cs,
                                                                const c128* __restrict__ part, int G) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  c128 p = cmk(0.0, 0.0), q = cmk(0.0, 0.0);
  for (int g = 0; g < G; ++g) {
    p = cadd(p, part[((size_t)g * n + i) * 2]);
    q = cadd(q, part[((size_t)g * n + i) * 2 + 1]);
  }
  const double inv = cs[j + 1].re;
  const c128 d = cs[j];
  const c128 v = cscale(csub(V[(size_t)j * ldv + i], p), inv);
  V[(size_t)j * ldv + i] = v;
  V[(size_t)(j + 1) * ldv + i] = csub(csub(cscale(z[i], inv), q), cmul(v, d));
}

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_arnoldi_dcgs2_step(qd_c128* V, long ldv, int j, int n, const qd_c128* z, qd_c128* H, long ldh,
                                     qd_c128* st, qd_c128* cs, void* stream) {
  WsScope wss_((hipStream_t)stream);
  QD_CHECK_ARG(V && z && H && st && cs, "qd_arnoldi_dcgs2_step: null pointer");
  QD_CHECK_ARG(j >= 0 && j <= 8192 && n >= 1 && ldv >= n && ldh >= j + 1,
               "qd_arnoldi_dcgs2_step: j=%d n=%d ldv=%ld ldh=%ld", j,
               n, ldv, ldh);
  hipStream_t st_ = (hipStream_t)stream;
  const int S = std::max(1, std::min(DCGS_MAX_SLICES, 1024 / (j + 1)));
  hipLaunchKernelGGL(dcgs_project_kernel, dim3(j + 1, S), dim3(256), 0, st_, (const c128*)V, ldv, j, n,
                     (const c128*)z, (c128*)st);
  QD_HIP(hipGetLastError());
  const size_t lds = (size_t)std::max(1, j) * sizeof(c128);
  if (lds > 48 * 1024) {
    static const bool lds_attr = [] {
      return hipFuncSetAttribute((const void*)dcgs_coef_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024 - 8 * 1024) == hipSuccess;
    }();
    (void)lds_attr;
  }
  hipLaunchKernelGGL(dcgs_coef_kernel, dim3(std::max(1, (j + 3) / 4)), dim3(256), lds, st_, (c128*)H, ldh, j,
                     (const c128*)st, S, (c128*)cs);
  QD_HIP(hipGetLastError());
  // row slices: enough workgroups to keep HBM busy (n / 256 columns of workgroups is ~100 at the bench hierarchy)
  const int G = std::max(1, std::min(16, j / 32));
  void* part = nullptr;
  if (int rc = workspace(WS_MISC, (size_t)G * n * 2 * sizeof(c128), &part, st_)) return rc;
  const int nb = (n + 255) / 256;
  hipLaunchKernelGGL(dcgs_update_partial_kernel, dim3(nb, G), dim3(256), 0, st_, (const c128*)V, ldv, j, n,
                     (const c128*)cs, (c128*)part);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(dcgs_update_final_kernel, dim3(nb), dim3(256), 0, st_, (c128*)V, ldv, j, n, (const c128*)z,
                     (const c128*)cs, (const c128*)part, G);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_cgs_project(const qd_c128* V, long ldv, int m, int n, const qd_c128* w, qd_c128* h, qd_c128* hsum,
                              long ldh, void* stream) {
  QD_CHECK_ARG(V && w && h, "qd_cgs_project: null pointer");
  QD_CHECK_ARG(m >= 1 && n >= 1 && ldv >= n, "qd_cgs_project: m=%d n=%d ldv=%ld", m, n, ldv);
  hipLaunchKernelGGL(cgs_project_kernel, dim3(m), dim3(256), 0, (hipStream_t)stream, (const c128*)V, ldv, n,
                     (const c128*)w, (c128*)h, (c128*)hsum, ldh);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_cgs_normalize(const qd_c128* w, int n, qd_c128* v, qd_c128* hsub, void* stream) {
  WsScope wss_((hipStream_t)stream);
  QD_CHECK_ARG(w && v && hsub && n >= 1, "qd_cgs_normalize: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  void* part = nullptr;
  if (int rc = workspace(WS_MISC, NRM_WG * sizeof(double), &part, st)) return rc;
  hipLaunchKernelGGL(cgs_norm_partial_kernel, dim3(NRM_WG), dim3(256), 0, st, (const c128*)w, n, (double*)part);
  QD_HIP(hipGetLastError());
  hipLaunchKernelGGL(cgs_norm_scale_kernel, dim3(std::min(256, (n + 255) / 256)), dim3(256), 0, st, (const c128*)w, n,
                     (const double*)part, (c128*)v, (c128*)hsub);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_shifted_hessenberg_solve(const qd_c128* H, int ldh, int k, const qd_c128* shifts, int S,
                                           double beta, qd_c128* Y, double* res, void* stream) {
  WsScope wss_((hipStream_t)stream);
  QD_CHECK_ARG(H && shifts && (Y || res), "qd_shifted_hessenberg_solve: null pointer");
  QD_CHECK_ARG(k >= 1 && ldh >= k && S >= 1 && k <= 4096, "qd_shifted_hessenberg_solve: k=%d ldh=%d S=%d", k, ldh, S);
  hipStream_t st = (hipStream_t)stream;
  void* w = nullptr;
  if (Y) {
    const int rc = workspace(WS_MISC, (size_t)S * k * k * sizeof(c128), &w, st);
    if (rc) return rc;
  }
  const size_t lds = (size_t)2 * k * sizeof(c128);   // <= 128 KB at k = 4096
  if (lds > 64 * 1024) {
    static const bool lds_attr = [] {
      // the 160 KiB of a CU less the kernel's static LDS (the attribute is refused above that)
      return hipFuncSetAttribute((const void*)hess_shift_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024 - 1024) == hipSuccess;
    }();
    (void)lds_attr;
  }
  hipLaunchKernelGGL(hess_shift_kernel, dim3(S), dim3(256), lds, st, (const c128*)H, ldh, k, (const c128*)shifts, beta,
                     (c128*)Y, res, (c128*)w);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
