// krylov.hip — the shifted Hessenberg solves of the multi-shift Krylov form of DEOMSolver.correlation_4op_3t
// (pyqed_amd/deom_krylov.py; reference heom/deom.py:1127-1209 diagonalises P instead).
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

}  // namespace
}  // namespace qd

using namespace qd;

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
  const size_t lds = (size_t)2 * k * sizeof(c128);
  hipLaunchKernelGGL(hess_shift_kernel, dim3(S), dim3(256), lds, st, (const c128*)H, ldh, k, (const c128*)shifts, beta,
                     (c128*)Y, res, (c128*)w);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
