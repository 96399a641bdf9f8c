// sos.hip — sum-over-states 2D photon-echo spectrum on a (omega3, omega1) grid.
//
// Replaces the vectorised NumPy loops of pyqed/signal/sos.py:
//   GSB (sos.py:624-678), SE (:731-785), ESA (:498-557), _photon_echo (:845-879),
//   photon_echo (:962-1052, omega1 = -pump).
// Output S[i][j]: i = probe (omega3) index, j = pump index — the reference's
// meshgrid('xy') layout.  One thread per grid point; the sums run over the
// g/e/f index lists in the reference's loop order (b, c, d).
#include "qd_common.hpp"

namespace qd {
namespace {

__device__ __forceinline__ c128 cinv(c128 z) {
  const double d = z.re * z.re + z.im * z.im;
  return cmk(z.re / d, -z.im / d);
}

// G_xy(w) = 1 / (w - (E_x - E_y) + i (g_x + g_y)/2)
__device__ __forceinline__ c128 green(double w, const c128* E, const double* g, int x, int y) {
  const c128 dE = csub(E[x], E[y]);
  return cinv(cmk(w - dE.re, -dE.im + 0.5 * (g[x] + g[y])));
}

__global__ void photon_echo_kernel(const c128* E, const c128* dip, const double* gam, int N, const int* gi, int ng,
                                   const int* ei, int nee, const int* fi, int nf, const double* pump, int n1,
                                   const double* probe, int n3, double t2, c128* S) {
  const int tot = n1 * n3;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
    const int i = e / n1, j = e % n1;
    const double w1 = -pump[j], w3 = probe[i];
    const int a = 0;
    c128 gsb = cmk(0, 0), se = cmk(0, 0), esa = cmk(0, 0);
    for (int bi = 0; bi < nee; ++bi) {
      const int b = ei[bi];
      const c128 Gab = green(w1, E, gam, a, b);
      // GSB: c = a = 0, d in e
      for (int di = 0; di < nee; ++di) {
        const int d = ei[di], c = 0;
        const c128 amp = cmul(cmul(dip[a * N + b], dip[b * N + c]), cmul(dip[c * N + d], dip[d * N + a]));
        gsb = cadd(gsb, cmul(amp, cmul(green(w3, E, gam, d, c), Gab)));
      }
      for (int ci = 0; ci < nee; ++ci) {
        const int c = ei[ci];
        // U_cb = -i exp(-i (E_c - E_b) t2 - (g_c + g_b)/2 t2)
        const c128 dE = csub(E[c], E[b]);
        const double re = dE.im * t2 - 0.5 * (gam[c] + gam[b]) * t2;
        const double ph = -dE.re * t2;
        double sn, cs;
        sincos(ph, &sn, &cs);
        const double mag = exp(re);
        const c128 U = cmulmi(cmk(mag * cs, mag * sn));
        const c128 UG = cmul(U, Gab);
        for (int di = 0; di < ng; ++di) {  // SE
          const int d = gi[di];
          const c128 amp = cmul(cmul(dip[a * N + b], dip[c * N + a]), cmul(dip[d * N + c], dip[b * N + d]));
          se = cadd(se, cmul(amp, cmul(green(w3, E, gam, c, d), UG)));
        }
        for (int di = 0; di < nf; ++di) {  // ESA
          const int d = fi[di];
          const c128 amp = cmul(cmul(dip[b * N + a], dip[c * N + a]), cmul(dip[d * N + c], dip[b * N + d]));
          esa = cadd(esa, cmul(amp, cmul(green(w3, E, gam, d, b), UG)));
        }
      }
    }
    S[e] = csub(cadd(gsb, se), esa);
  }
}

}  // namespace
}  // namespace qd

using namespace qd;

extern "C" int qd_photon_echo(const qd_c128* E, const qd_c128* dip, const double* gamma, int N, const int32_t* g_idx,
                              int ng, const int32_t* e_idx, int ne, const int32_t* f_idx, int nf, const double* pump,
                              int n1, const double* probe, int n3, double t2, qd_c128* S, void* stream) {
  QD_CHECK_ARG(E && dip && gamma && g_idx && e_idx && f_idx && pump && probe && S, "qd_photon_echo: null pointer");
  QD_CHECK_ARG(N >= 1 && n1 >= 1 && n3 >= 1 && ng >= 0 && ne >= 0 && nf >= 0, "qd_photon_echo: bad sizes");
  const int tot = n1 * n3;
  hipLaunchKernelGGL(photon_echo_kernel, dim3(std::min(16384, (tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const c128*)E, (const c128*)dip, gamma, N, g_idx, ng, e_idx, ne, f_idx, nf, pump, n1, probe, n3,
                     t2, (c128*)S);
  QD_HIP(hipGetLastError());
  return QD_OK;
}
