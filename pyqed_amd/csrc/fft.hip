// fft.hip — physical-unit Fourier transforms of pyqed/fft.py on the GPU.
//
//   qd_fft_axis : FFT / inverse FFT along one axis of a contiguous array viewed as
//                 [outer][n][inner], fused with fftshift, a scale factor and the
//                 phase exp(-/+ i freq x0) of pyqed.fft.fft / ifft (fft.py:11-102)
//                 and fft2 (fft.py:104-126).  Any n (numpy.fft takes every length):
//                 powers of two in [16, 1024] run one Stockham LDS kernel with the
//                 epilogue fused; every other n runs the any-size engine of the SPO
//                 grids (spo_gen.hip fft_lines: mixed radix 2/3/4/5/p <= 61 in LDS,
//                 Bluestein, four-step for long smooth lengths, direct DFT for the
//                 rest) on a copy, then one shift / scale / phase pass back.
//   qd_dft2     : DFT at arbitrary momenta (fft.py:128-160 dft / dft2).
#include "qd_common.hpp"

#include <cstdlib>

namespace qd {
namespace {

template <int L, bool INV>
__device__ __forceinline__ c128* stockham(c128* a, c128* b, const c128* tw, int t) {
#pragma unroll
  for (int Ns = 1; Ns * 4 <= L; Ns *= 4) {
    if (t < L / 4) {
      const int j = t, k = j % Ns, base = k * (L / (4 * Ns));
      c128 w1 = tw[base], w2 = tw[2 * base], w3 = tw[3 * base];
      if (INV) { w1 = cconj(w1); w2 = cconj(w2); w3 = cconj(w3); }
      const c128 v0 = a[j], v1 = cmul(a[j + L / 4], w1), v2 = cmul(a[j + L / 2], w2), v3 = cmul(a[j + 3 * L / 4], w3);
      const c128 a0 = cadd(v0, v2), a1 = csub(v0, v2), b0 = cadd(v1, v3), b1 = csub(v1, v3);
      const c128 ib1 = INV ? cmuli(b1) : cmulmi(b1);
      const int d = (j / Ns) * Ns * 4 + k;
      b[d] = cadd(a0, b0);
      b[d + Ns] = cadd(a1, ib1);
      b[d + 2 * Ns] = csub(a0, b0);
      b[d + 3 * Ns] = csub(a1, ib1);
    }
    __syncthreads();
    c128* tmp = a; a = b; b = tmp;
  }
  constexpr int lg = __builtin_ctz(L);
  if (lg & 1) {
    if (t < L / 4) {
      constexpr int Ns = L / 2;
      for (int h = 0; h < 2; ++h) {
        const int j = t + h * (L / 4), k = j % Ns;
        c128 w = tw[k];
        if (INV) w = cconj(w);
        const c128 v0 = a[j], v1 = cmul(a[j + L / 2], w);
        const int d = (j / Ns) * Ns * 2 + k;
        b[d] = cadd(v0, v1);
        b[d + Ns] = csub(v0, v1);
      }
    }
    __syncthreads();
    c128* tmp = a; a = b; b = tmp;
  }
  return a;
}

// post-processing of one transformed row X (natural order) into data
__device__ __forceinline__ void fft_store(const c128* X, c128* base, long stride, int n, int shift, double scale,
                                          const double* freq, double x0, int sign) {
  for (int kp = threadIdx.x; kp < n; kp += blockDim.x) {
    const int k = shift ? ((kp - n / 2) % n + n) % n : kp;
    c128 v = cscale(X[k], scale);
    if (freq) {
      double s, c;
      sincos(sign * freq[kp] * x0, &s, &c);
      v = cmul(v, cmk(c, s));
    }
    base[(long)kp * stride] = v;
  }
}

template <int L>
__global__ void fft_pow2_kernel(c128* data, int inner, int inverse, int shift, double scale, const double* freq,
                                double x0, const c128* twg) {
  __shared__ c128 tw[L], A[L], B[L];
  const long b = blockIdx.x;
  const long o = b / inner, i = b % inner;
  c128* base = data + o * (long)L * inner + i;
  for (int k = threadIdx.x; k < L; k += blockDim.x) {
    tw[k] = twg[k];
    A[k] = base[(long)k * inner];
  }
  __syncthreads();
  c128* X = inverse ? stockham<L, true>(A, B, tw, threadIdx.x) : stockham<L, false>(A, B, tw, threadIdx.x);
  fft_store(X, base, inner, L, shift, scale, freq, x0, inverse ? 1 : -1);
}

// out[o][kp][i] = scale X[o][pos(k)][i] exp(sign i freq[kp] x0), k = fftshift source of kp; pos = the slot of X[k]
// in fft_lines' output (four-step order when l2 != 0)
__global__ void fft_post_kernel(const c128* __restrict__ X, c128* __restrict__ out, long O, int n, long I, int shift,
                                double scale, const double* __restrict__ freq, double x0, int sign, int l2) {
  const long tot = O * n * I;
  const int l1 = l2 ? n / l2 : 1;
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < tot; f += (long)gridDim.x * blockDim.x) {
    const long o = f / ((long)n * I), r = f - o * n * I;
    const int kp = (int)(r / I);
    const long i = r - (long)kp * I;
    const int k = shift ? ((kp - n / 2) % n + n) % n : kp;
    const int pos = l2 ? (k % l1) * l2 + k / l1 : k;
    c128 v = cscale(X[((size_t)o * n + pos) * I + i], scale);
    if (freq) {
      double sn, c;
      sincos(sign * freq[kp] * x0, &sn, &c);
      v = cmul(v, cmk(c, sn));
    }
    out[f] = v;
  }
}

__global__ void twiddles_kernel(int L, c128* tw) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < L; k += gridDim.x * blockDim.x) {
    double s, c;
    sincospi(-2.0 * (double)k / (double)L, &s, &c);
    tw[k] = cmk(c, s);
  }
}

// out[i][j] = sum_{a,b} f[a][b] exp(-i (kx_i x_b + ky_j y_a)) * w    (ny == 1 / y == 0 gives 1D dft)
__global__ void dft2_kernel(const double* x, int nx, const double* y, int ny, const c128* f, const double* kx, int nkx,
                            const double* ky, int nky, double w, c128* out) {
  const int tot = nkx * nky;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
    const int i = e / nky, j = e % nky;
    c128 acc = cmk(0, 0);
    for (int a = 0; a < ny; ++a)
      for (int bb = 0; bb < nx; ++bb) {
        double s, c;
        sincos(-(kx[i] * x[bb] + ky[j] * y[a]), &s, &c);
        acc = cadd(acc, cmul(f[(long)a * nx + bb], cmk(c, s)));
      }
    out[e] = cscale(acc, w);
  }
}

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_fft_axis(qd_c128* data, int outer, int n, int inner, int inverse, int shift, double scale,
                           const double* freq, double x0, void* stream) {
  WsScope wss_((hipStream_t)stream);  // call-scoped scratch (qd_runtime.hip)
  QD_CHECK_ARG(data, "qd_fft_axis: null pointer");
  QD_CHECK_ARG(outer >= 1 && inner >= 1 && n >= 1, "qd_fft_axis: bad sizes");
  QD_CHECK_ARG((long)outer * n * inner < (1L << 31), "qd_fft_axis: array too large (%ld elements)",
               (long)outer * n * inner);
  hipStream_t st = (hipStream_t)stream;
  const int batch = outer * inner;
  const bool pow2 = n >= 16 && n <= 1024 && (n & (n - 1)) == 0;
  note_path(pow2 ? "fft_pow2" : "fft_any");
  if (pow2) {
    void* w = nullptr;
    int rc = workspace(WS_MISC, n * sizeof(c128), &w, st);
    if (rc) return rc;
    hipLaunchKernelGGL(twiddles_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, (c128*)w);
    QD_HIP(hipGetLastError());
    const int threads = std::max(64, n / 4);
#define FCALL(L)                                                                                                   \
  hipLaunchKernelGGL(fft_pow2_kernel<L>, dim3(batch), dim3(threads), 0, st, (c128*)data, inner, inverse, shift,    \
                     scale, freq, x0, (const c128*)w)
    switch (n) {
      case 16: FCALL(16); break;
      case 32: FCALL(32); break;
      case 64: FCALL(64); break;
      case 128: FCALL(128); break;
      case 256: FCALL(256); break;
      case 512: FCALL(512); break;
      case 1024: FCALL(1024); break;
    }
#undef FCALL
    QD_HIP(hipGetLastError());
    return QD_OK;
  }
  // any other length: transform a copy with the any-size engine, then shift / scale / phase back into data
  const long tot = (long)outer * n * inner;
  void* w = nullptr;
  int rc = workspace(WS_MISC, (size_t)tot * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* X = (c128*)w;
  QD_TRY(copy_device(X, data, (size_t)tot * sizeof(c128), st));
  int l2 = 0;
  if ((rc = fft_lines(X, outer, n, inner, inverse != 0, st, &l2))) return rc;
  const int grid = (int)std::max<long>(1, std::min<long>((tot + 255) / 256, 16384));
  hipLaunchKernelGGL(fft_post_kernel, dim3(grid), dim3(256), 0, st, (const c128*)X, (c128*)data, (long)outer, n,
                     (long)inner, shift, scale, freq, x0, inverse ? 1 : -1, l2);
  QD_HIP(hipGetLastError());
  return QD_OK;
}

extern "C" int qd_dft2(const double* x, int nx, const double* y, int ny, const qd_c128* f, const double* kx, int nkx,
                       const double* ky, int nky, double weight, qd_c128* out, void* stream) {
  QD_CHECK_ARG(x && y && f && kx && ky && out, "qd_dft2: null pointer");
  QD_CHECK_ARG(nx >= 1 && ny >= 1 && nkx >= 1 && nky >= 1, "qd_dft2: bad sizes");
  const int tot = nkx * nky;
  hipLaunchKernelGGL(dft2_kernel, dim3(std::min(16384, (tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, nx, y,
                     ny, (const c128*)f, kx, nkx, ky, nky, weight, (c128*)out);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
