// fft.hip — physical-unit Fourier transforms of pyqed/fft.py on the GPU.
//
//   qd_fft_axis : FFT / inverse FFT along one axis of a contiguous array viewed as
//                 [outer][n][inner], fused with fftshift, a scale factor and the
//                 phase exp(-/+ i freq x0) of pyqed.fft.fft / ifft (fft.py:11-102)
//                 and fft2 (fft.py:104-126).  n a power of two <= 1024 uses the
//                 Stockham LDS FFT of spo.hip's family; any other n <= 4096 uses a
//                 direct DFT with integer-reduced fp64 twiddles (exact periodicity).
//   qd_dft2     : DFT at arbitrary momenta (fft.py:128-160 dft / dft2).
#include "qd_common.hpp"

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

// direct DFT for arbitrary n: X[k] = sum_j x[j] w^{(j k) mod n}, w = exp(-/+ 2 pi i / n)
__global__ void dft_kernel(c128* data, int n, int inner, int inverse, int shift, double scale, const double* freq,
                           double x0) {
  extern __shared__ c128 sm[];
  c128* x = sm;       // n
  c128* X = sm + n;   // n
  c128* tw = X + n;   // n
  const long b = blockIdx.x;
  const long o = b / inner, i = b % inner;
  c128* base = data + o * (long)n * inner + i;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    x[k] = base[(long)k * inner];
    double s, c;
    sincospi((inverse ? 2.0 : -2.0) * (double)k / (double)n, &s, &c);
    tw[k] = cmk(c, s);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    c128 acc = cmk(0, 0);
    long idx = 0;
    for (int j = 0; j < n; ++j) {
      acc = cadd(acc, cmul(x[j], tw[idx]));
      idx += k;
      if (idx >= n) idx -= n;
    }
    X[k] = acc;
  }
  __syncthreads();
  fft_store(X, base, inner, n, shift, scale, freq, x0, inverse ? 1 : -1);
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
  QD_CHECK_ARG((long)outer * inner < (1L << 31), "qd_fft_axis: batch too large");
  hipStream_t st = (hipStream_t)stream;
  const int batch = outer * inner;
  const bool pow2 = n >= 16 && n <= 1024 && (n & (n - 1)) == 0;
  QD_CHECK_ARG(pow2 || n <= 3200, "qd_fft_axis: n=%d: powers of two up to 1024 or any n up to 3200", n);
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
  } else {
    hipLaunchKernelGGL(dft_kernel, dim3(batch), dim3(256), 3 * n * sizeof(c128), st, (c128*)data, n, inner, inverse,
                       shift, scale, freq, x0);
  }
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
