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

}  // namespace
}  // namespace qd

using namespace qd;

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
