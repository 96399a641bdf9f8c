// spo_gen.hip — split-operator propagation on ANY grid (every size the reference's SPO classes accept).
//
// The reference transforms with scipy.fftpack / numpy.fft (pocketfft), which take every length
// (wpd.py:225-273 SPO, :692-758 SPO2, :1349-1411 SPO3).  spo.hip's register / Stockham kernels cover
// powers of two in [16, 1024]; this file serves every other grid with the same pass structure:
//
//   axis plan per grid axis of length L (plan_axis):
//     MIXED      mixed-radix Stockham autosort in LDS: radix 8, 4, 2, 3, 5 butterflies in closed form, any
//                other prime p <= 61 as a direct p-point DFT stage; natural-order output, fp64 twiddles
//                exp(-2 pi i m / L) from sincospi, L <= 5120 (two LDS lines of L complex values)
//     BLUESTEIN  lengths with a prime factor > 61: chirp-z, X_k = c_k sum_n (x_n c_n) conj(c_{k-n}),
//                c_n = exp(-pi i n^2 / L) (n^2 mod 2L exact in integers), the convolution as an M-point
//                mixed-radix FFT pair in LDS, M = the smallest 2^a 3^b 5^c >= 2L - 1 (M <= 5120)
//     DIRECT     everything longer: O(L^2) DFT straight from HBM / L2, twiddle index (n k) mod L exact
//
//   one fused LDS pass per axis (spo_axis_kernel): a tile of G outer rows x C consecutive inner columns
//   (C * 16 B contiguous per line element, the whole [L][ns] row when C == ns) is loaded once, then
//     [IFFT] -> [U1 point op] -> [snapshot] -> [U2 point op] -> [FFT] -> [k_y phase] -> [FFT * K * IFFT]
//   run on it in LDS and it is stored once.  Point operators (exp(-i V dt/2) per grid point, any ns)
//   need every state of a point, i.e. the last (contiguous) axis with C == ns; KMUL (exp_K / N) is the
//   outermost axis's FFT -> multiply -> IFFT.  The step sequence is spo.hip's (qd_spo2_run_ex /
//   qd_spo3_run): both V/2 halves of every Strang step applied, as the reference's return_states=True
//   arithmetic (wpd.py:723-730), or the merged V structure (wpd.py:736-755).
//   A pass that does not fit the LDS budget (DIRECT axes, ns * M too large for a fused row) runs
//   unfused: axis transforms, a point-operator kernel (thread per (point, state), any ns) and a
//   k-space multiply, with one grid-sized scratch buffer.
//
//   2D grids alternate two layouts between the passes (Exec::xpose): the row pass reads [x][y][s] rows and writes
//   [y][x][s], the kinetic pass reads those x lines contiguously (exp_K / N transposed to match) and writes [x][y][s]
//   back, so every pass loads whole contiguous lines and only the stores are strided (fire-and-forget, off the
//   dependent chain): 200^2 x 2 24.3 -> 22.5 us per step, 1000^2 x 2 143 -> 134 (profiles/r04/spo/spo_xpose_ab.txt).
//   3D grids can rotate their layouts the same way (QD_SPO_XPOSE3=1) but lose at 96^3 and above (see Exec).
//
//   SPO (1D, wpd.py:225-273): one persistent workgroup per wavepacket, all steps in LDS when the line
//   fits; otherwise one launch sequence per step.
#include "qd_common.hpp"

#include <cstdlib>
#include <functional>
#include <vector>

namespace qd {
namespace spog {

constexpr int MAX_ST = 32;
constexpr size_t LDS_MAX = 163840;            // one workgroup may hold all 160 KiB on gfx950
constexpr size_t LDS_SOFT = 65536;            // tile target: two or more workgroups per CU
constexpr int GEN_MAXP = 61;                  // largest prime run as a direct radix stage
constexpr int MAX_LDS_M = (int)(LDS_MAX / (2 * sizeof(c128)));   // 5120

enum Kind { MIXED = 0, BLUESTEIN = 1, DIRECT = 2 };

// Division by a launch-invariant divisor d >= 1 as a multiply-high (Granlund-Montgomery / Hacker's Delight 10-8,
// exact for every 32-bit x): l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, t = umulhi(x, m),
// x / d = (t + ((x - t) >> 1)) >> (l - 1); d = 1 is x itself.  The element loops of the LDS passes divide their
// flat index by runtime lengths several times per element; a 32-bit udiv is ~25 VALU instructions, this is 5.
struct FDiv {
  unsigned d, m, s;
};
inline FDiv make_fdiv(unsigned d) {
  FDiv r{d, 0u, 0u};
  if (d > 1) {
    unsigned l = 0;
    while ((1ull << l) < d) ++l;
    r.m = (unsigned)((((unsigned long long)1 << 32) * ((1ull << l) - d)) / d + 1);
    r.s = l - 1;
  }
  return r;
}
__host__ __device__ __forceinline__ unsigned fdiv(unsigned x, FDiv D) {
  if (D.d == 1) return x;
  const unsigned t = (unsigned)(((unsigned long long)x * D.m) >> 32);
  return (t + ((x - t) >> 1)) >> D.s;
}

struct Fft {           // device-side plan of one axis, passed by value
  int L, M, kind, nst;
  int R[MAX_ST];
  int Ns[MAX_ST];
  FDiv dnb[MAX_ST];    // M / R[s]
  FDiv dns[MAX_ST];    // Ns[s]
  FDiv dM;             // M
  const c128* tw;      // exp(-2 pi i m / M), m < M (DIRECT: M = L)
  const c128* chirp;   // BLUESTEIN: exp(-pi i n^2 / L), n < L
  const c128* bhat;    // BLUESTEIN: (1/M) FFT_M(b), b_m = conj(c_|m|) wrapped
};

enum Flags { F_INV = 1, F_PT1 = 2, F_SNAP = 4, F_PT2 = 8, F_FWD = 16, F_KY = 32, F_KMUL = 64,
             F_XOUT = 128,    // store into another layout: element (o, e, i) of [O][L][I], o = hi nlo + lo, to
                              // out[hi sh + lo sl + e se + i] (2D: [L][O][I])
             F_KROW = 256 };  // KMUL on whole rows (C == I == ns): factor K[o][e] of the [O][L] table

struct AxisArgs {
  c128* psi;           // tile source
  c128* out;           // tile destination (psi: in place; F_XOUT: the other layout's buffer)
  long sh, sl, se;     // F_XOUT strides of hi, lo, e
  FDiv dlo;            // F_XOUT: division by nlo
  int O, L, I, C, G, flags, ns;
  FDiv dLC, dC, dLns, dns;   // L C, C, L ns, ns
  int twl;             // 1: twiddles staged in LDS (M more c128 of dynamic LDS)
  const c128* U1;      // [points][ns][ns] (F_PT1)
  const c128* U2;      // (F_PT2)
  c128* snap;          // (F_SNAP) same layout as psi
  const c128* K;       // (F_KMUL) exp_K / N over the grid points, [L][I / ns]
  const c128* Ky;      // (F_KY) [O][L]
};

// ---------------------------------------------------------------- device FFT
// One Stockham stage over nl lines of length M: butterfly j of a line reads src[j + r M/R] (r < R) times
// tw^(r k M/(Ns R)), k = j mod Ns, and writes the R-point DFT to dst[(j / Ns) Ns R + k + q Ns].
template <bool INV, int R0>   // R0 = 2, 3, 4, 5, 8: closed-form butterflies; 0: any prime R <= GEN_MAXP
__device__ __forceinline__ void stage(const c128* __restrict__ src, c128* __restrict__ dst, int nl, int M, int Rr,
                                      int Ns, FDiv dnb, FDiv dns, const c128* __restrict__ tw) {
  const int R = R0 ? R0 : Rr;
  const int nb = M / R;
  const int tot = nl * nb;
  const int tstep = M / (Ns * R);
  for (int f = threadIdx.x; f < tot; f += blockDim.x) {
    const int l = (int)fdiv((unsigned)f, dnb), j = f - l * nb;
    const c128* s = src + (size_t)l * M;
    c128* d = dst + (size_t)l * M;
    const int jq = (int)fdiv((unsigned)j, dns);
    const int k = j - jq * Ns;
    const int db = jq * Ns * R + k;
    auto ld = [&](int r) {
      const c128 x = s[j + r * nb];
      if (r == 0 || k == 0) return x;
      c128 w = tw[r * k * tstep];
      if (INV) w = cconj(w);
      return cmul(x, w);
    };
    if constexpr (R0 == 8) {   // DFT8 = DFT4 of the even and of the odd inputs, combined with w8^k
      const c128 x0 = ld(0), x1 = ld(1), x2 = ld(2), x3 = ld(3), x4 = ld(4), x5 = ld(5), x6 = ld(6), x7 = ld(7);
      auto mj = [](c128 v) { return INV ? cmuli(v) : cmulmi(v); };   // times -+ i
      const c128 a0 = cadd(x0, x4), a1 = csub(x0, x4), a2 = cadd(x2, x6), a3 = mj(csub(x2, x6));
      const c128 b0 = cadd(x1, x5), b1 = csub(x1, x5), b2 = cadd(x3, x7), b3 = mj(csub(x3, x7));
      const c128 e0 = cadd(a0, a2), e2 = csub(a0, a2), e1 = cadd(a1, a3), e3 = csub(a1, a3);
      c128 o0 = cadd(b0, b2), o2 = csub(b0, b2), o1 = cadd(b1, b3), o3 = csub(b1, b3);
      const double h = 0.70710678118654752440;   // 1 / sqrt(2)
      // o1 w8, o2 w8^2 = -+ i, o3 w8^3 with w8 = (1 -+ i) / sqrt(2)
      o1 = INV ? cmk((o1.re - o1.im) * h, (o1.re + o1.im) * h) : cmk((o1.re + o1.im) * h, (o1.im - o1.re) * h);
      o2 = mj(o2);
      o3 = INV ? cmk(-(o3.re + o3.im) * h, (o3.re - o3.im) * h) : cmk((o3.im - o3.re) * h, -(o3.re + o3.im) * h);
      d[db] = cadd(e0, o0);
      d[db + Ns] = cadd(e1, o1);
      d[db + 2 * Ns] = cadd(e2, o2);
      d[db + 3 * Ns] = cadd(e3, o3);
      d[db + 4 * Ns] = csub(e0, o0);
      d[db + 5 * Ns] = csub(e1, o1);
      d[db + 6 * Ns] = csub(e2, o2);
      d[db + 7 * Ns] = csub(e3, o3);
    } else if constexpr (R0 == 4) {
      const c128 x0 = ld(0), x1 = ld(1), x2 = ld(2), x3 = ld(3);
      const c128 a0 = cadd(x0, x2), a1 = csub(x0, x2), b0 = cadd(x1, x3), b1 = csub(x1, x3);
      const c128 ib1 = INV ? cmuli(b1) : cmulmi(b1);
      d[db] = cadd(a0, b0);
      d[db + Ns] = cadd(a1, ib1);
      d[db + 2 * Ns] = csub(a0, b0);
      d[db + 3 * Ns] = csub(a1, ib1);
    } else if constexpr (R0 == 2) {
      const c128 x0 = ld(0), x1 = ld(1);
      d[db] = cadd(x0, x1);
      d[db + Ns] = csub(x0, x1);
    } else if constexpr (R0 == 3) {
      const double c = -0.5, sn = 0.86602540378443864676;   // cos, sin(2 pi / 3)
      const c128 x0 = ld(0), x1 = ld(1), x2 = ld(2);
      const c128 t = cadd(x1, x2), u = csub(x1, x2);
      const c128 a = cadd(x0, cscale(t, c));
      const c128 b = INV ? cmuli(cscale(u, sn)) : cmulmi(cscale(u, sn));   // -+ i s (x1 - x2)
      d[db] = cadd(x0, t);
      d[db + Ns] = cadd(a, b);
      d[db + 2 * Ns] = csub(a, b);
    } else if constexpr (R0 == 5) {
      const double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;   // cos(2 pi/5), cos(4 pi/5)
      const double s1 = 0.95105651629515357212, s2 = 0.58778525229247312917;    // sin(2 pi/5), sin(4 pi/5)
      const c128 x0 = ld(0), x1 = ld(1), x2 = ld(2), x3 = ld(3), x4 = ld(4);
      const c128 t1 = cadd(x1, x4), t2 = cadd(x2, x3), t3 = csub(x1, x4), t4 = csub(x2, x3);
      const c128 a1 = cadd(x0, cadd(cscale(t1, c1), cscale(t2, c2)));
      const c128 a2 = cadd(x0, cadd(cscale(t1, c2), cscale(t2, c1)));
      const c128 b1r = cadd(cscale(t3, s1), cscale(t4, s2));
      const c128 b2r = csub(cscale(t3, s2), cscale(t4, s1));
      const c128 b1 = INV ? cmuli(b1r) : cmulmi(b1r), b2 = INV ? cmuli(b2r) : cmulmi(b2r);
      d[db] = cadd(x0, cadd(t1, t2));
      d[db + Ns] = cadd(a1, b1);
      d[db + 4 * Ns] = csub(a1, b1);
      d[db + 2 * Ns] = cadd(a2, b2);
      d[db + 3 * Ns] = csub(a2, b2);
    } else {  // any prime R <= GEN_MAXP: y_q = sum_r x_r w_R^(r q), w_R^m = tw[m M/R]
      for (int q = 0; q < R; ++q) {
        c128 acc = cmk(0.0, 0.0);
        int e = 0;  // r q mod R
        for (int r = 0; r < R; ++r) {
          c128 w = tw[e * nb];
          if (INV) w = cconj(w);
          acc = cadd(acc, cmul(ld(r), w));
          e += q;
          if (e >= R) e -= R;
        }
        d[db + q * Ns] = acc;
      }
    }
  }
}
template <bool INV>
__device__ __forceinline__ void stockham(const Fft& p, const c128* tw, c128*& cur, c128*& oth, int nl, int M) {
  for (int s = 0; s < p.nst; ++s) {
    const int R = p.R[s], Ns = p.Ns[s];
    const FDiv dnb = p.dnb[s], dns = p.dns[s];   // copies: a reference would put the plan in scratch
    switch (R) {   // wave-uniform: one branch-free element loop per radix
      case 8: stage<INV, 8>(cur, oth, nl, M, 8, Ns, dnb, dns, tw); break;
      case 4: stage<INV, 4>(cur, oth, nl, M, 4, Ns, dnb, dns, tw); break;
      case 2: stage<INV, 2>(cur, oth, nl, M, 2, Ns, dnb, dns, tw); break;
      case 3: stage<INV, 3>(cur, oth, nl, M, 3, Ns, dnb, dns, tw); break;
      case 5: stage<INV, 5>(cur, oth, nl, M, 5, Ns, dnb, dns, tw); break;
      default: stage<INV, 0>(cur, oth, nl, M, R, Ns, dnb, dns, tw); break;
    }
    __syncthreads();
    c128* t = cur;
    cur = oth;
    oth = t;
  }
}

// Length-L DFT (INV: conjugate kernel, no scaling) of nl lines held in the first L slots of each M-slot
// line of cur.  Result in cur (first L slots).
template <bool INV>
__device__ __forceinline__ void lds_fft(const Fft& p, const c128* tw, c128*& cur, c128*& oth, int nl) {
  const int M = p.M, L = p.L;
  if (p.kind == BLUESTEIN) {
    const int tot = nl * M;
    for (int f = threadIdx.x; f < tot; f += blockDim.x) {
      const int n = f - (int)fdiv((unsigned)f, p.dM) * M;
      c128 v = cmk(0.0, 0.0);
      if (n < L) {
        c128 ch = p.chirp[n];
        if (INV) ch = cconj(ch);
        v = cmul(cur[f], ch);
      }
      cur[f] = v;
    }
    __syncthreads();
    stockham<false>(p, tw, cur, oth, nl, M);
    for (int f = threadIdx.x; f < tot; f += blockDim.x) {
      c128 b = p.bhat[f - (int)fdiv((unsigned)f, p.dM) * M];
      if (INV) b = cconj(b);
      cur[f] = cmul(cur[f], b);
    }
    __syncthreads();
    stockham<true>(p, tw, cur, oth, nl, M);
    for (int f = threadIdx.x; f < tot; f += blockDim.x) {
      const int n = f - (int)fdiv((unsigned)f, p.dM) * M;
      if (n < L) {
        c128 ch = p.chirp[n];
        if (INV) ch = cconj(ch);
        cur[f] = cmul(cur[f], ch);
      }
    }
    __syncthreads();
  } else {
    stockham<INV>(p, tw, cur, oth, nl, M);
  }
}

// ---------------------------------------------------------------- fused axis pass
#ifdef QD_PHASE_TIMING
// diagnostics build: per-pass phase wall clock summed over blocks (thread 0's view after each barrier)
// [0] load, [1] inverse FFT, [2] point ops / snapshot / k_y, [3] forward FFT / kinetic step, [4] store, [5] blocks
__device__ unsigned long long g_spo_tim[2][6];
#define SPO_MARK(k)                                   \
  if (threadIdx.x == 0) {                             \
    const unsigned long long now_ = wall_clock64();   \
    atomicAdd(&g_spo_tim[a.flags & F_KMUL ? 1 : 0][k], now_ - tl_); \
    tl_ = now_;                                       \
  }
#else
#define SPO_MARK(k)
#endif
__global__ __launch_bounds__(256) void spo_axis_kernel(Fft p, AxisArgs a) {
  extern __shared__ c128 sm[];
#ifdef QD_PHASE_TIMING
  unsigned long long tl_ = wall_clock64();
  if (threadIdx.x == 0) atomicAdd(&g_spo_tim[a.flags & F_KMUL ? 1 : 0][5], 1ull);
#endif
  const int M = p.M, L = a.L, C = a.C, G = a.G, I = a.I;
  const int nl = G * C;
  c128* cur = sm;
  c128* oth = sm + (size_t)nl * M;
  // twiddles: staged in LDS behind the two line buffers when the host reserved room (a.twl), else read from HBM/L2
  const c128* tw = p.tw;
  if (a.twl) {
    c128* stw = oth + (size_t)nl * M;
    for (int m = threadIdx.x; m < M; m += blockDim.x) stw[m] = p.tw[m];
    tw = stw;
  }
  const int o0 = blockIdx.x * G, i0 = blockIdx.y * C;
  const int gv = min(G, a.O - o0), cv = min(C, I - i0);
  const int tot = G * L * C;
  const int ns = a.ns;
  const int pts = I / ns;
  for (int f = threadIdx.x; f < tot; f += blockDim.x) {
    const int g = (int)fdiv((unsigned)f, a.dLC), r = f - g * (L * C), e = (int)fdiv((unsigned)r, a.dC), c = r - e * C;
    cur[(g * C + c) * M + e] =
        (g < gv && c < cv) ? a.psi[((size_t)(o0 + g) * L + e) * I + i0 + c] : cmk(0.0, 0.0);
  }
  __syncthreads();
  SPO_MARK(0)
  if (a.flags & F_INV) lds_fft<true>(p, tw, cur, oth, nl);
  SPO_MARK(1)
  auto point_op = [&](const c128* U) {   // C == I == ns: line g * ns + s holds state s of row g
    const int n = G * L * ns;
    const int row0 = o0;
    for (int f = threadIdx.x; f < n; f += blockDim.x) {
      const int g = (int)fdiv((unsigned)f, a.dLns), r = f - g * (L * ns), e = (int)fdiv((unsigned)r, a.dns),
                s = r - e * ns;
      if (g >= gv) continue;
      const c128* u = U + (((size_t)(row0 + g) * L + e) * ns + s) * ns;
      c128 acc = cmk(0.0, 0.0);
      for (int b = 0; b < ns; ++b) acc = cadd(acc, cmul(u[b], cur[(g * ns + b) * M + e]));
      oth[(g * ns + s) * M + e] = acc;
    }
    __syncthreads();
    c128* t = cur;
    cur = oth;
    oth = t;
  };
  if (a.flags & F_PT1) point_op(a.U1);
  if (a.flags & F_SNAP) {
    for (int f = threadIdx.x; f < tot; f += blockDim.x) {
      const int g = (int)fdiv((unsigned)f, a.dLC), r = f - g * (L * C), e = (int)fdiv((unsigned)r, a.dC), c = r - e * C;
      if (g < gv && c < cv) a.snap[((size_t)(o0 + g) * L + e) * I + i0 + c] = cur[(g * C + c) * M + e];
    }
  }
  if (a.flags & F_PT2) point_op(a.U2);
  SPO_MARK(2)
  if (a.flags & F_FWD) lds_fft<false>(p, tw, cur, oth, nl);
  if (a.flags & F_KY) {
    for (int f = threadIdx.x; f < tot; f += blockDim.x) {
      const int g = (int)fdiv((unsigned)f, a.dLC), r = f - g * (L * C), e = (int)fdiv((unsigned)r, a.dC), c = r - e * C;
      if (g < gv) cur[(g * C + c) * M + e] = cmul(a.Ky[(size_t)(o0 + g) * L + e], cur[(g * C + c) * M + e]);
    }
    __syncthreads();
  }
  if (a.flags & F_KMUL) {   // outermost axis (O == 1): FFT -> * exp_K / N -> IFFT
    lds_fft<false>(p, tw, cur, oth, nl);
    for (int f = threadIdx.x; f < tot; f += blockDim.x) {
      const int r = f - (int)fdiv((unsigned)f, a.dLC) * (L * C), e = (int)fdiv((unsigned)r, a.dC), c = r - e * C;
        if (a.flags & F_KROW) {
        const int g = (int)fdiv((unsigned)f, a.dLC);
        if (g < gv) cur[(g * C + c) * M + e] = cmul(cur[(g * C + c) * M + e], a.K[(size_t)(o0 + g) * L + e]);
      } else if (c < cv) {
        cur[c * M + e] = cmul(cur[c * M + e], a.K[(size_t)e * pts + (int)fdiv((unsigned)(i0 + c), a.dns)]);
      }
    }
    __syncthreads();
    lds_fft<true>(p, tw, cur, oth, nl);
  }
  SPO_MARK(3)
  for (int f = threadIdx.x; f < tot; f += blockDim.x) {
    const int g = (int)fdiv((unsigned)f, a.dLC), r = f - g * (L * C), e = (int)fdiv((unsigned)r, a.dC), c = r - e * C;
    if (g < gv && c < cv) {
      size_t o;
      if (a.flags & F_XOUT) {
        const unsigned og = (unsigned)(o0 + g), hi = fdiv(og, a.dlo), lo = og - hi * a.dlo.d;
        o = (size_t)hi * a.sh + (size_t)lo * a.sl + (size_t)e * a.se + i0 + c;
      } else {
        o = ((size_t)(o0 + g) * L + e) * I + i0 + c;
      }
      a.out[o] = cur[(g * C + c) * M + e];
    }
  }
#ifdef QD_PHASE_TIMING
  __syncthreads();
#endif
  SPO_MARK(4)
}

// ---------------------------------------------------------------- unfused kernels
// Direct DFT along one axis, out of place: dst[o][k][i] = sum_n src[o][n][i] w^(n k) (w = exp(-+2 pi i / L)).
// Block (x, y): outputs k in [256 x, 256 x + 256) of lines y, y + gridDim.y, ...; input staged 256 points at a
// time in LDS, per-output accumulators in LDS (flat loops: any blockDim).
template <bool INV>
__global__ __launch_bounds__(256) void dft_axis_kernel(const c128* __restrict__ src, c128* __restrict__ dst, long O,
                                                       int L, long I, const c128* __restrict__ tw) {
  __shared__ c128 xs[256];
  __shared__ c128 acc[256];
  const long nlines = O * I;
  const int k0 = blockIdx.x * 256;
  const int nk = min(256, L - k0);
  for (long line = blockIdx.y; line < nlines; line += gridDim.y) {
    const long o = line / I, i = line - o * I;
    const c128* s = src + (size_t)o * L * I + i;
    for (int t = threadIdx.x; t < 256; t += blockDim.x) acc[t] = cmk(0.0, 0.0);
    for (int n0 = 0; n0 < L; n0 += 256) {
      const int cnt = min(256, L - n0);
      __syncthreads();
      for (int t = threadIdx.x; t < cnt; t += blockDim.x) xs[t] = s[(size_t)(n0 + t) * I];
      __syncthreads();
      for (int kk = threadIdx.x; kk < nk; kk += blockDim.x) {
        const long k = k0 + kk;
        long e = ((long)n0 * k) % L;
        c128 a = acc[kk];
        for (int t = 0; t < cnt; ++t) {
          c128 w = tw[e];
          if (INV) w = cconj(w);
          a = cadd(a, cmul(xs[t], w));
          e += k;
          if (e >= L) e -= L;
        }
        acc[kk] = a;
      }
    }
    __syncthreads();
    for (int kk = threadIdx.x; kk < nk; kk += blockDim.x) dst[(size_t)o * L * I + (size_t)(k0 + kk) * I + i] = acc[kk];
    __syncthreads();
  }
}

// dst[p][s] = sum_b U[p][s][b] src[p][b], one thread per (point, state), any ns
__global__ void pointop_kernel(const c128* __restrict__ src, c128* __restrict__ dst, const c128* __restrict__ U,
                               long npts, int ns) {
  const long n = npts * ns;
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < n; f += (long)gridDim.x * blockDim.x) {
    const long pt = f / ns;
    const c128* u = U + (size_t)f * ns;
    const c128* x = src + (size_t)pt * ns;
    c128 acc = cmk(0.0, 0.0);
    for (int b = 0; b < ns; ++b) acc = cadd(acc, cmul(u[b], x[b]));
    dst[f] = acc;
  }
}

// psi[p][s] *= K[p / rep_div % rep_mod ...]: psi element f multiplies K[(f / ns) / kdiv] (kdiv = 1: K per
// point; used for exp_K / N on the whole grid and the Jacobi k_y phase per (row, k_y))
__global__ void kmul_kernel(c128* psi, const c128* __restrict__ K, long n, int ns) {
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < n; f += (long)gridDim.x * blockDim.x)
    psi[f] = cmul(psi[f], K[f / ns]);
}

// dst[z][y][x] = s src[x][y][z] (src [n0][n1][n2]): the kinetic table of the 3D rotated passes
// dst[j][i] = s src[i][j] (src [r][c]): the kinetic table of the xpose passes
__global__ void scale_transpose_kernel(const c128* __restrict__ src, c128* __restrict__ dst, int r, int c, double s) {
  const long n = (long)r * c;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / c), j = (int)(e % c);
    dst[(size_t)j * r + i] = cscale(src[e], s);
  }
}
__global__ void scale_copy_kernel(const c128* __restrict__ src, c128* __restrict__ dst, long n, double s) {
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < n; f += (long)gridDim.x * blockDim.x)
    dst[f] = cscale(src[f], s);
}

// psi[f] *= K[f % L] (one factor per line position, every line of the batch)
__global__ void bcast_mul_kernel(c128* psi, const c128* __restrict__ K, long n, int L) {
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < n; f += (long)gridDim.x * blockDim.x)
    psi[f] = cmul(psi[f], K[f % L]);
}

// Four-step twiddle of a line viewed as [L1][L2]: element (k1, n2) *= w_L^(+-n2 k1) (index (n2 k1) mod L exact)
__global__ void fourstep_twiddle_kernel(c128* psi, long n, int L1, int L2, const c128* __restrict__ twL, int inv) {
  const long L = (long)L1 * L2;
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < n; f += (long)gridDim.x * blockDim.x) {
    const long r = f % L;
    const long k1 = r / L2, n2 = r - k1 * L2;
    c128 w = twL[(n2 * k1) % L];
    if (inv) w = cconj(w);
    psi[f] = cmul(psi[f], w);
  }
}

// exp_K in the four-step's k order: Kp[k1 L2 + k2] = scale * K[k1 + L1 k2]
__global__ void fourstep_kperm_kernel(const c128* __restrict__ K, c128* Kp, int L1, int L2, double scale) {
  const long L = (long)L1 * L2;
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < L; r += (long)gridDim.x * blockDim.x) {
    const long k1 = r / L2, k2 = r - k1 * L2;
    Kp[r] = cscale(K[k1 + (long)L1 * k2], scale);
  }
}

// Four-step twiddle of lines viewed as [L1][L2] inside a [O][L][I] grid: element (o, k1, n2, i) *= w_L^(+-n2 k1)
__global__ void fourstep_twiddle_inner_kernel(c128* psi, long n, int L1, int L2, long I, const c128* __restrict__ twL,
                                              int inv) {
  const long L = (long)L1 * L2;
  for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < n; f += (long)gridDim.x * blockDim.x) {
    const long r = (f / I) % L;
    const long k1 = r / L2, n2 = r - k1 * L2;
    c128 w = twL[(n2 * k1) % L];
    if (inv) w = cconj(w);
    psi[f] = cmul(psi[f], w);
  }
}

// ---------------------------------------------------------------- plan tables
__global__ void twiddle_table_kernel(int M, c128* tw) {
  for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < M; m += gridDim.x * blockDim.x) {
    double s, c;
    sincospi(-2.0 * (double)m / (double)M, &s, &c);
    tw[m] = cmk(c, s);
  }
}

// c_n = exp(-pi i n^2 / L) with n^2 mod 2L exact; b_m = conj(c_|m|) wrapped into M slots
__global__ void chirp_kernel(int L, int M, c128* chirp, c128* b) {
  for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < M; m += gridDim.x * blockDim.x) {
    const int n = m < L ? m : (M - m < L ? M - m : -1);
    c128 v = cmk(0.0, 0.0);
    if (n >= 0) {
      const long q = ((long)n * n) % (2L * L);
      double s, c;
      sincospi(-(double)q / (double)L, &s, &c);
      if (m < L) chirp[m] = cmk(c, s);
      v = cmk(c, -s);
    }
    b[m] = v;
  }
}

// bhat[k] = (1/M) sum_m b[m] exp(-2 pi i m k / M) (direct, exact index (m k) mod M)
__global__ void bhat_kernel(int M, const c128* __restrict__ b, const c128* __restrict__ tw, c128* bhat) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < M; k += gridDim.x * blockDim.x) {
    c128 acc = cmk(0.0, 0.0);
    long e = 0;
    for (int m = 0; m < M; ++m) {
      acc = cadd(acc, cmul(b[m], tw[e]));
      e += k;
      if (e >= M) e -= M;
    }
    bhat[k] = cscale(acc, 1.0 / M);
  }
}

// ---------------------------------------------------------------- 1D persistent SPO
// SPO.run (wpd.py:250-270): V/2; for blk in 1..nt//nout-1: nout x [K, V], snapshot; K; V/2.
// One workgroup per wavepacket, the line resident in LDS for the whole run.
__global__ __launch_bounds__(256) void spo1d_gen_kernel(Fft p, c128* psi, const c128* eV, const c128* eVh,
                                                        const c128* eK, int nt, int nout, c128* snap, int twl) {
  extern __shared__ c128 sm[];
  const int L = p.L, M = p.M;
  c128* cur = sm;
  c128* oth = sm + M;
  const c128* tw = p.tw;
  if (twl) {
    c128* stw = sm + 2 * M;
    for (int m = threadIdx.x; m < M; m += blockDim.x) stw[m] = p.tw[m];
    tw = stw;
  }
  const int b = blockIdx.x;
  c128* x = psi + (size_t)b * L;
  const double inv = 1.0 / L;
  for (int k = threadIdx.x; k < L; k += blockDim.x) cur[k] = cmul(eVh[k], x[k]);
  __syncthreads();
  const int nblk = nt / nout;
  const int nsnap = nblk > 0 ? nblk - 1 : 0;
  auto kstep = [&]() {
    lds_fft<false>(p, tw, cur, oth, 1);
    for (int k = threadIdx.x; k < L; k += blockDim.x) cur[k] = cmul(cur[k], cscale(eK[k], inv));
    __syncthreads();
    lds_fft<true>(p, tw, cur, oth, 1);
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
  for (int k = threadIdx.x; k < L; k += blockDim.x) x[k] = cmul(eVh[k], cur[k]);
}

// ---------------------------------------------------------------- point propagators, any ns
// exp(-i V tau) per grid point for the SPO build (wpd.py:585-623 SPO2, :1290-1330 SPO3: eigh -> U e^{-iw tau} U^+;
// wpd.py:960-985 SPO2NH: eig -> U_R e^{-iw tau} U_R^-1).  Both are the matrix exponential; here it is evaluated
// directly, by scaling and squaring a degree-18 Taylor polynomial (||X|| <= 1/2 after scaling: truncation
// < 1e-22), so no eigenvectors are needed on the device.  exp(-i V dt) = exp(-i V dt/2)^2 (one more product).
// herm: the Hermitian matrix LAPACK's eigh sees (lower triangle, real diagonal); otherwise the full matrix.
// One workgroup per grid point (grid-stride), lane e = i ns + j owns element (i, j).  GLB = false: the four ns x ns
// matrices live in LDS (ns <= 50: 160 KB at ns = 50); GLB = true (50 < ns <= 1024): in a per-workgroup slice of a
// global scratch buffer (64 ns^2 bytes, L2-resident up to ns ~ 90), with the same code -- the workgroup barrier
// orders its global stores and loads as it does LDS ones.
template <bool CPLX, bool GLB>
__global__ __launch_bounds__(1024) void spo_expm_kernel(const void* v_, int herm, long npts, int ns, double dt,
                                                        c128* expV, c128* expVh, c128* work) {
  extern __shared__ c128 sm[];
  const int ns2 = ns * ns;
  c128* X = GLB ? work + (size_t)blockIdx.x * 4 * ns2 : sm;
  c128* T = X + ns2;
  c128* S = T + ns2;
  c128* W = S + ns2;
  __shared__ int sh_s;
  const int t0 = threadIdx.x, nt = blockDim.x;
  auto vat = [&](long p, int r, int c) {
    const size_t o = (size_t)p * ns2 + (size_t)r * ns + c;
    return CPLX ? ((const c128*)v_)[o] : cmk(((const double*)v_)[o], 0.0);
  };
  auto matmul = [&](const c128* A, const c128* B, c128* C, double scale) {   // C = scale A B (C distinct from A, B)
    __syncthreads();
    for (int e = t0; e < ns2; e += nt) {
      const int i = e / ns, j = e - i * ns;
      c128 acc = cmk(0.0, 0.0);
      for (int l = 0; l < ns; ++l) acc = cadd(acc, cmul(A[i * ns + l], B[l * ns + j]));
      C[e] = cscale(acc, scale);
    }
    __syncthreads();
  };
  for (long p = blockIdx.x; p < npts; p += gridDim.x) {
    // ||V tau||_inf (max row sum), tau = dt / 2; H (the matrix eigh / eig would see) staged in X
    const double tau = 0.5 * dt;
    for (int e = t0; e < ns2; e += nt) {
      const int i = e / ns, j = e - i * ns;
      c128 h;
      if (herm) {
        if (i == j) h = cmk(vat(p, i, i).re, 0.0);
        else h = i > j ? vat(p, i, j) : cconj(vat(p, j, i));
      } else {
        h = vat(p, i, j);
      }
      X[e] = h;
      W[e] = cmk(sqrt(h.re * h.re + h.im * h.im), 0.0);
    }
    __syncthreads();
    for (int e = t0; e < ns; e += nt) {
      double r = 0.0;
      for (int l = 0; l < ns; ++l) r += W[e * ns + l].re;
      T[e] = cmk(r, 0.0);
    }
    __syncthreads();
    if (t0 == 0) {
      double nrm = 0.0;
      for (int l = 0; l < ns; ++l) nrm = fmax(nrm, T[l].re);
      nrm *= fabs(tau);
      int sq = 0;
      if (!(nrm <= 1.7976931348623157e308)) {
        sq = -1;   // inf / NaN in V: no exponential (the host raises LinAlgError first, as eigh does)
      } else {
        while (nrm > 0.5 && sq < 1100) {   // a finite norm needs at most ~1025 halvings: the loop always ends
          nrm *= 0.5;
          ++sq;
        }
      }
      sh_s = sq;
    }
    __syncthreads();
    const int sq = sh_s;
    if (sq < 0) {
      const c128 nan = cmk(__builtin_nan(""), __builtin_nan(""));
      for (int e = t0; e < ns2; e += nt) {
        expVh[(size_t)p * ns2 + e] = nan;
        if (expV) expV[(size_t)p * ns2 + e] = nan;
      }
      __syncthreads();
      continue;
    }
    const double sc = ldexp(tau, -sq);   // tau / 2^sq without an integer shift (sq may exceed 63)
    // X = -i V tau / 2^sq ; S = I + X ; T = X
    for (int e = t0; e < ns2; e += nt) {
      const int i = e / ns, j = e - i * ns;
      const c128 x = cmulmi(cscale(X[e], sc));
      X[e] = x;
      T[e] = x;
      S[e] = cadd(x, cmk(i == j ? 1.0 : 0.0, 0.0));
    }
    for (int k = 2; k <= 18; ++k) {
      matmul(T, X, W, 1.0 / k);   // W = T X / k
      for (int e = t0; e < ns2; e += nt) {
        T[e] = W[e];
        S[e] = cadd(S[e], W[e]);
      }
    }
    for (int q = 0; q < sq; ++q) {
      matmul(S, S, W, 1.0);
      for (int e = t0; e < ns2; e += nt) S[e] = W[e];
    }
    __syncthreads();
    for (int e = t0; e < ns2; e += nt) expVh[(size_t)p * ns2 + e] = S[e];
    if (expV) {
      matmul(S, S, W, 1.0);
      for (int e = t0; e < ns2; e += nt) expV[(size_t)p * ns2 + e] = W[e];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- host planning
bool all_factors_small(int n, int maxp) {
  for (int p = 2; (long)p * p <= n; ++p)
    while (n % p == 0) {
      if (p > maxp) return false;
      n /= p;
    }
  return n <= maxp;
}

int next_smooth(int n) {  // smallest 2^a 3^b 5^c >= n
  for (int m = n;; ++m) {
    int r = m;
    for (int p : {2, 3, 5})
      while (r % p == 0) r /= p;
    if (r == 1) return m;
  }
}

void factor_stages(int M, Fft& f) {
  f.nst = 0;
  int ns = 1, n = M;
  f.dM = make_fdiv((unsigned)M);
  auto push = [&](int r) {
    if (f.nst < MAX_ST) {
      f.R[f.nst] = r;
      f.Ns[f.nst] = ns;
      f.dnb[f.nst] = make_fdiv((unsigned)(M / r));
      f.dns[f.nst] = make_fdiv((unsigned)ns);
    }
    ++f.nst;
    ns *= r;
    n /= r;
  };
  // radix 8 first (one LDS stage and barrier instead of a radix-4 and a radix-2 one: 200 = 8 5 5 in three stages
  // instead of four)
  {
    // 8s as long as no single 2 would be left over unpaired with a 4 (16 = 8 2 would take as many stages as 4 4)
    int twos = 0;
    for (int m = n; m % 2 == 0; m /= 2) ++twos;
    for (int k = 0; k < twos / 3 && twos % 3 != 1; ++k) push(8);
    if (twos % 3 == 1 && twos >= 4) {   // 2^(3j+1): 8^(j-1) 4 4 is as short as 8^j 2 and has no radix-2 stage
      for (int k = 0; k < (twos - 4) / 3; ++k) push(8);
    }
  }
  while (n % 4 == 0) push(4);
  while (n % 2 == 0) push(2);
  while (n % 3 == 0) push(3);
  while (n % 5 == 0) push(5);
  int p = 7;
  while (n > 1) {
    while (n % p == 0) push(p);
    p += 2;
  }
}

// Kind and table sizes of an axis of length L (count of c128 table slots in *tab).
void plan_kind(int L, int* kind, int* M, size_t* tab) {
  if (L <= MAX_LDS_M && all_factors_small(L, GEN_MAXP)) {
    *kind = MIXED;
    *M = L;
    *tab = L;
    return;
  }
  const int m = next_smooth(2 * L - 1);
  if (L >= 2 && m <= MAX_LDS_M) {
    *kind = BLUESTEIN;
    *M = m;
    *tab = (size_t)3 * m + L;   // tw[M], chirp[L], b[M], bhat[M]
    return;
  }
  *kind = DIRECT;
  *M = L;
  *tab = L;
}

int plan_axis(int L, c128* tab, Fft& f, hipStream_t st) {
  int kind, M;
  size_t n;
  plan_kind(L, &kind, &M, &n);
  f.L = L;
  f.M = M;
  f.kind = kind;
  f.tw = tab;
  f.chirp = f.bhat = nullptr;
  f.nst = 0;
  hipLaunchKernelGGL(twiddle_table_kernel, dim3((M + 255) / 256), dim3(256), 0, st, M, tab);
  QD_HIP(hipGetLastError());
  f.dM = make_fdiv((unsigned)M);
  if (kind != DIRECT) factor_stages(M, f);
  if (f.nst > MAX_ST) {
    set_error("spo: FFT plan of length %d needs %d stages (max %d)", M, f.nst, MAX_ST);
    return QD_EINVAL;
  }
  if (kind == BLUESTEIN) {
    c128* chirp = tab + M;
    c128* b = chirp + L;
    c128* bhat = b + M;
    hipLaunchKernelGGL(chirp_kernel, dim3((M + 255) / 256), dim3(256), 0, st, L, M, chirp, b);
    hipLaunchKernelGGL(bhat_kernel, dim3((M + 255) / 256), dim3(256), 0, st, M, (const c128*)b, (const c128*)tab, bhat);
    QD_HIP(hipGetLastError());
    f.chirp = chirp;
    f.bhat = bhat;
  }
  return QD_OK;
}

size_t plan_slots(int L) {
  int k, M;
  size_t n;
  plan_kind(L, &k, &M, &n);
  return n;
}

inline int grid_for(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

// ---------------------------------------------------------------- executor
struct Exec {
  int D = 0;
  int n[3] = {1, 1, 1};
  int ns = 1;
  long npts = 0;
  Fft f[3];
  hipStream_t st = nullptr;
  c128* psi = nullptr;
  c128* tmp = nullptr;     // grid-sized scratch (unfused passes)
  const c128* Ks = nullptr;   // exp_K / N
  const c128* KsT = nullptr;  // exp_K / N in the kinetic pass's input layout (xpose): [n1][n0]
  const c128* Ky = nullptr;   // Jacobi k_y phase [n0][n1] (D == 2)
  bool xpose = false;         // 2D: alternating layouts (file header); psi [n0][n1][ns] <-> tmp [n1][n0][ns]
  int kin_g = 1;              // xpose: rows per tile of the kinetic pass

  long outer(int d) const { long o = 1; for (int k = 0; k < d; ++k) o *= n[k]; return o; }
  long inner(int d) const { long i = ns; for (int k = d + 1; k < D; ++k) i *= n[k]; return i; }

  int launch_axis(int d, int flags, int C, int G, const c128* U1, const c128* U2, c128* snap) {
    return launch_tile(f[d], outer(d), inner(d), flags, C, G, U1, U2, snap, psi, psi, Ks);
  }
  struct Store {   // F_XOUT map (see Flags)
    long nlo, sh, sl, se;
  };
  // one spo_axis_kernel pass with plan p over the [O][p.L][I] grid at src, stored to dst ([p.L][O][I] with F_XOUT)
  int launch_tile(const Fft& p, long O, long I, int flags, int C, int G, const c128* U1, const c128* U2, c128* snap,
                  c128* src, c128* dst, const c128* K, Store sm = {1, 0, 0, 0}) {
    const int L = p.L;
    AxisArgs a;
    a.psi = src;
    a.out = dst;
    a.sh = sm.sh;
    a.sl = sm.sl;
    a.se = sm.se;
    a.dlo = make_fdiv((unsigned)sm.nlo);
    a.O = (int)O;
    a.L = L;
    a.I = (int)I;
    a.C = C;
    a.dLC = make_fdiv((unsigned)(L * C));
    a.dC = make_fdiv((unsigned)C);
    a.dLns = make_fdiv((unsigned)(L * ns));
    a.dns = make_fdiv((unsigned)ns);
    a.G = G;
    a.flags = flags;
    a.ns = ns;
    a.U1 = U1;
    a.U2 = U2;
    a.snap = snap;
    a.K = K;
    a.Ky = Ky;
    size_t lds = (size_t)2 * G * C * p.M * sizeof(c128);
    a.twl = lds + (size_t)p.M * sizeof(c128) <= LDS_MAX;
    if (a.twl) lds += (size_t)p.M * sizeof(c128);
    // (round 4 tried staging the pass's operators in LDS with the tile: 500^2 x 2 50.3 vs 43.8 us per step, the larger
    // tile lowering the workgroups per CU; profiles/r04/spo/spo_any_aux_*.txt)
    (void)hipFuncSetAttribute((const void*)spo_axis_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
    hipLaunchKernelGGL(spo_axis_kernel, dim3((a.O + G - 1) / G, (a.I + C - 1) / C), dim3(256), lds, st, p, a);
    QD_HIP(hipGetLastError());
    return QD_OK;
  }

  // rows per tile of a whole-row pass (C == I) over O rows of length L: stack short rows (< 256 elements per
  // tile) while >= 256 tiles remain
  int stack_rows(long O, int L, int c, int M) const {
    const size_t line = (size_t)2 * M * sizeof(c128);
    int g = 1;
    while (g < O && (long)g * c * L < 256 && O / (2 * g) >= 256 && (size_t)(2 * g) * c * line <= LDS_SOFT) g *= 2;
    return (int)std::min<long>(g, O);
  }
  // xpose passes (D == 2): the row pass over psi ([n0][n1][ns] rows), stored transposed into tmp when xout; the
  // kinetic pass over tmp's x lines ([n1][n0][ns]) with exp_K / N transposed, stored transposed back into psi
  int row_pass(int flags, const c128* U1, const c128* U2, c128* snap, bool xout) {
    const int G = stack_rows(n[0], n[1], ns, f[1].M);
    return launch_tile(f[1], n[0], ns, flags | (xout ? F_XOUT : 0), ns, G, U1, U2, snap, psi, xout ? tmp : psi, Ks,
                       Store{n[0], 0, ns, (long)n[0] * ns});
  }
  int kin_pass() {
    return launch_tile(f[0], n[1], ns, F_KMUL | F_KROW | F_XOUT, ns, kin_g, nullptr, nullptr, nullptr, tmp, psi, KsT,
                       Store{n[1], 0, ns, (long)n[1] * ns});
  }

  // lines-per-tile choice for an LDS pass over axis d; C == I (whole rows) required for point ops
  bool tile(int d, bool rows, int* C, int* G) const {
    const long I = inner(d), O = outer(d);
    const size_t line = (size_t)2 * f[d].M * sizeof(c128);
    int c;
    if (rows) {
      c = (int)I;
    } else {   // 8 consecutive columns (128-B rows) when that still leaves >= 256 tiles, else fewer
      c = (int)std::min<long>(I, 8);
      while (c > 1 && ((size_t)c * line > LDS_SOFT || ((I + c - 1) / c) * O < 256)) c >>= 1;
    }
    if ((size_t)c * line > LDS_MAX) return false;
    int g = 1;
    if (c == I) g = stack_rows(O, n[d], c, f[d].M);   // whole rows
    *C = c;
    *G = g;
    return true;
  }

  int transform(int d, bool inv) {
    if (f[d].kind != DIRECT) {
      int C, G;
      if (tile(d, false, &C, &G)) return launch_axis(d, inv ? F_INV : F_FWD, C, G, nullptr, nullptr, nullptr);
    }
    // direct DFT from HBM into the scratch grid, then back
    const long O = outer(d), I = inner(d);
    const int L = n[d];
    const long lines = O * I;
    const dim3 grid((L + 255) / 256, (unsigned)std::min<long>(lines, 65535));
    if (inv)
      hipLaunchKernelGGL(dft_axis_kernel<true>, grid, dim3(256), 0, st, (const c128*)psi, tmp, O, L, I, f[d].tw);
    else
      hipLaunchKernelGGL(dft_axis_kernel<false>, grid, dim3(256), 0, st, (const c128*)psi, tmp, O, L, I, f[d].tw);
    QD_HIP(hipGetLastError());
    QD_TRY(copy_device(psi, tmp, (size_t)npts * ns * sizeof(c128), st));
    return QD_OK;
  }

  int pointop(const c128* U) {
    hipLaunchKernelGGL(pointop_kernel, dim3(grid_for(npts * ns)), dim3(256), 0, st, (const c128*)psi, tmp, U, npts, ns);
    QD_HIP(hipGetLastError());
    QD_TRY(copy_device(psi, tmp, (size_t)npts * ns * sizeof(c128), st));
    return QD_OK;
  }

  int kmul(const c128* K) {
    hipLaunchKernelGGL(kmul_kernel, dim3(grid_for(npts * ns)), dim3(256), 0, st, psi, K, npts * ns, ns);
    QD_HIP(hipGetLastError());
    return QD_OK;
  }

  // One pass over axis d with the ops of `flags` (F_PT*, F_SNAP, F_KY: last axis; F_KMUL: axis 0).
  int pass(int d, int flags, const c128* U1, const c128* U2, c128* snap) {
    const bool pt = flags & (F_PT1 | F_PT2 | F_SNAP | F_KY);
    if (f[d].kind != DIRECT) {
      int C, G;
      if (tile(d, pt, &C, &G)) return launch_axis(d, flags, C, G, U1, U2, snap);
    }
    int rc;
    if ((flags & F_INV) && (rc = transform(d, true))) return rc;
    if ((flags & F_PT1) && (rc = pointop(U1))) return rc;
    if (flags & F_SNAP)
      QD_TRY(copy_device(snap, psi, (size_t)npts * ns * sizeof(c128), st));
    if ((flags & F_PT2) && (rc = pointop(U2))) return rc;
    if ((flags & F_FWD) && (rc = transform(d, false))) return rc;
    if ((flags & F_KY) && (rc = kmul(Ky))) return rc;
    if (flags & F_KMUL) {
      if ((rc = transform(d, false))) return rc;
      if ((rc = kmul(Ks))) return rc;
      if ((rc = transform(d, true))) return rc;
    }
    return QD_OK;
  }
};

// Strang / merged step sequence of qd_spo2_run_ex / qd_spo3_run on a D-dimensional grid (D = 2, 3).
int run_nd(Exec& x, const c128* Uh, const c128* Ufull, int nsteps, int nout, c128* snap, bool ky) {
  const int D = x.D, last = D - 1;
  const int kyf = ky ? F_KY : 0;
  const size_t grid_elems = (size_t)x.npts * x.ns;
  int rc;
  if (x.xpose) {   // D == 2, nsteps >= 1: the same pass sequence with the row pass storing into the other layout
    if ((rc = x.row_pass(F_PT1 | F_FWD | kyf, Uh, nullptr, nullptr, true))) return rc;
    for (int s = 1; s <= nsteps; ++s) {
      if ((rc = x.kin_pass())) return rc;
      const bool take = snap && (s % nout == 0);
      c128* sp = take ? snap + (size_t)(s / nout - 1) * grid_elems : nullptr;
      int flags = F_INV | F_PT1 | (take ? F_SNAP : 0);
      if (Ufull) flags |= F_FWD | kyf;
      else if (s < nsteps) flags |= F_PT2 | F_FWD | kyf;
      if ((rc = x.row_pass(flags, Ufull ? Ufull : Uh, Uh, sp, (flags & F_FWD) != 0))) return rc;
    }
    if (Ufull) {
      if ((rc = x.kin_pass())) return rc;
      if ((rc = x.row_pass(F_INV | F_PT1, Uh, nullptr, nullptr, false))) return rc;
    }
    return QD_OK;
  }
  if ((rc = x.pass(last, F_PT1 | F_FWD | kyf, Uh, nullptr, nullptr))) return rc;
  for (int d = last - 1; d >= 1; --d)
    if ((rc = x.pass(d, F_FWD, nullptr, nullptr, nullptr))) return rc;
  for (int s = 1; s <= nsteps; ++s) {
    if ((rc = x.pass(0, F_KMUL, nullptr, nullptr, nullptr))) return rc;
    for (int d = 1; d < last; ++d)
      if ((rc = x.pass(d, F_INV, nullptr, nullptr, nullptr))) return rc;
    const bool take = snap && (s % nout == 0);
    c128* sp = take ? snap + (size_t)(s / nout - 1) * grid_elems : nullptr;
    int flags = F_INV | F_PT1 | (take ? F_SNAP : 0);
    if (Ufull) flags |= F_FWD | kyf;
    else if (s < nsteps) flags |= F_PT2 | F_FWD | kyf;
    if ((rc = x.pass(last, flags, Ufull ? Ufull : Uh, Uh, sp))) return rc;
    if (flags & F_FWD)
      for (int d = last - 1; d >= 1; --d)
        if ((rc = x.pass(d, F_FWD, nullptr, nullptr, nullptr))) return rc;
  }
  if (Ufull) {   // merged tail (wpd.py:752-755): K, then V/2
    if ((rc = x.pass(0, F_KMUL, nullptr, nullptr, nullptr))) return rc;
    for (int d = 1; d < last; ++d)
      if ((rc = x.pass(d, F_INV, nullptr, nullptr, nullptr))) return rc;
    if ((rc = x.pass(last, F_INV | F_PT1, Uh, nullptr, nullptr))) return rc;
  }
  return QD_OK;
}

}  // namespace spog

// Unnormalised DFT along the middle axis of the [O][L][I] grid x, in place (inv: the conjugate kernel), for pyqed.fft's
// any-length transforms (fft.hip).  Lengths the LDS plans take (mixed radix <= 5120, Bluestein with M <= 5120) run one
// spo_axis_kernel pass; longer lengths that split as L1 L2 with both factors LDS-plannable run the four-step FFT and
// leave X[k1 + L1 k2] at slot L2 k1 + k2 (*l2 = L2; *l2 = 0: natural order); anything else a direct DFT.
int fft_lines(c128* x, long O, int L, long I, bool inv, hipStream_t st, int* l2) {
  using namespace spog;
  *l2 = 0;
  const long total = O * L * I;
  int kind, M;
  size_t nslots;
  plan_kind(L, &kind, &M, &nslots);
  int L1 = 0;
  if (kind == DIRECT) {
    for (int a = 2; (long)a * a <= L; ++a) {
      if (L % a) continue;
      int k1, k2, m1, m2;
      size_t s1, s2;
      plan_kind(a, &k1, &m1, &s1);
      plan_kind(L / a, &k2, &m2, &s2);
      if (k1 != DIRECT && k2 != DIRECT) L1 = a;   // the most balanced plannable split
    }
  }
  Exec e;
  e.st = st;
  e.psi = x;
  e.ns = (int)I;
  int rc;
  if (L1) {
    const int L2 = L / L1;
    void* w = nullptr;
    if ((rc = workspace(WS_MISC, (plan_slots(L1) + plan_slots(L2) + (size_t)L) * sizeof(c128), &w, st))) return rc;
    c128* tab = (c128*)w;
    c128* twL = tab + plan_slots(L1) + plan_slots(L2);
    e.D = 3;
    e.n[0] = (int)O;
    e.n[1] = L1;
    e.n[2] = L2;
    e.npts = O * L;
    if ((rc = plan_axis(L1, tab, e.f[1], st))) return rc;
    if ((rc = plan_axis(L2, tab + plan_slots(L1), e.f[2], st))) return rc;
    hipLaunchKernelGGL(twiddle_table_kernel, dim3((L + 255) / 256), dim3(256), 0, st, L, twL);
    QD_HIP(hipGetLastError());
    if ((rc = e.transform(1, inv))) return rc;
    hipLaunchKernelGGL(fourstep_twiddle_inner_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, total, L1, L2, I,
                       (const c128*)twL, inv ? 1 : 0);
    QD_HIP(hipGetLastError());
    if ((rc = e.transform(2, inv))) return rc;
    *l2 = L2;
    return QD_OK;
  }
  void* w = nullptr;
  const size_t tmp = kind == DIRECT ? (size_t)total : 0;
  if ((rc = workspace(WS_MISC, (nslots + tmp) * sizeof(c128), &w, st))) return rc;
  e.D = 2;
  e.n[0] = (int)O;
  e.n[1] = L;
  e.npts = O * L;
  e.tmp = (c128*)w + nslots;
  if ((rc = plan_axis(L, (c128*)w, e.f[1], st))) return rc;
  return e.transform(1, inv);
}

// Generic SPO2 / SPO3 run (any grid, any ns).  dims = {nx, ny} or {nx, ny, nz}; expK [dims] unscaled;
// expKy [nx][ny] (2D Jacobi) or null; expV (merged V structure) or null.
int spo_generic_run(c128* psi, const c128* expVh, const c128* expV, const c128* expK, const c128* expKy,
                    const int* dims, int D, int ns, int nsteps, int nout, c128* snap, hipStream_t st) {
  using namespace spog;
  WsScope wss_(st);
  Exec x;
  x.D = D;
  x.ns = ns;
  x.st = st;
  x.psi = psi;
  x.npts = 1;
  for (int d = 0; d < D; ++d) {
    x.n[d] = dims[d];
    x.npts *= dims[d];
  }
  size_t slots = (size_t)x.npts * ns + 2 * x.npts;   // tmp grid + exp_K / N (+ transposed)
  for (int d = 0; d < D; ++d) slots += plan_slots(dims[d]);
  void* w = nullptr;
  int rc = workspace(WS_SPO, slots * sizeof(c128), &w, st);
  if (rc) return rc;
  x.tmp = (c128*)w;
  c128* ks = x.tmp + (size_t)x.npts * ns;
  c128* tab = ks + x.npts;
  for (int d = 0; d < D; ++d) {
    if ((rc = plan_axis(dims[d], tab, x.f[d], st))) return rc;
    tab += plan_slots(dims[d]);
  }
  hipLaunchKernelGGL(scale_copy_kernel, dim3(grid_for(x.npts)), dim3(256), 0, st, expK, ks, x.npts,
                     1.0 / (double)x.npts);
  QD_HIP(hipGetLastError());
  x.Ks = ks;
  x.Ky = expKy;
  // alternating layouts (2D, every axis an LDS plan whose whole-row tile fits).  (Round 4 measured the same rotation
  // for 3D grids: 60^3 x 2 55.4 -> 54.4 us per step, but 96^3 126.5 -> 143.4 and 100^3 140.7 -> 161.7, the scattered
  // 32-B stores at large strides costing more than the strided loads removed; profiles/r04/spo/spo_xpose_ab.txt.)
  {
    bool fit = nsteps >= 1 && D == 2;
    for (int d = 0; d < D && fit; ++d)   // every axis a whole-row LDS pass (C == ns)
      fit = x.f[d].kind != DIRECT && (size_t)2 * ns * x.f[d].M * sizeof(c128) <= LDS_MAX;
    x.xpose = fit;
    for (int d = 0; d < D; ++d)
      note_path(x.f[d].kind == DIRECT ? "spo_axis_direct" : x.f[d].kind == BLUESTEIN ? "spo_axis_bluestein"
                                                                                      : "spo_axis_mixed");
    note_path(x.xpose ? "spo_layout_alternating" : "spo_layout_in_place");
    if (x.xpose) {
      c128* kt = tab;   // behind the plan tables
      hipLaunchKernelGGL(scale_transpose_kernel, dim3(grid_for(x.npts)), dim3(256), 0, st, expK, kt, dims[0], dims[1],
                         1.0 / (double)x.npts);
      QD_HIP(hipGetLastError());
      x.KsT = kt;
      x.kin_g = x.stack_rows(x.npts / dims[0], dims[0], ns, x.f[0].M);
    }
  }
#ifdef QD_PHASE_TIMING
  {
    unsigned long long z[2][6] = {};
    QD_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_spo_tim), z, sizeof(z), 0, hipMemcpyHostToDevice, st));
    rc = run_nd(x, expVh, expV, nsteps, nout, snap, expKy != nullptr);
    QD_HIP(hipStreamSynchronize(st));
    QD_HIP(hipMemcpyFromSymbol(z, HIP_SYMBOL(g_spo_tim), sizeof(z)));
    const char* nm[5] = {"load", "inv_fft", "point_ops", "fwd_fft_or_kin", "store"};
    for (int k = 0; k < 2; ++k) {
      if (!z[k][5]) continue;
      fprintf(stderr, "[spo_axis phase timing] %s pass, us per block:", k ? "kinetic" : "row");
      for (int q = 0; q < 5; ++q) fprintf(stderr, " %s %.3f", nm[q], (double)z[k][q] / z[k][5] / 100.0);
      fprintf(stderr, " (%llu blocks)\n", z[k][5]);
    }
    return rc;
  }
#else
  return run_nd(x, expVh, expV, nsteps, nout, snap, expKy != nullptr);
#endif
}

// exp(-i V dt/2), exp(-i V dt) per point for any ns <= SPO_EXPM_MAX_NS (spo_expm_kernel): LDS-resident matrices up to
// ns = 50, a global scratch slice per workgroup above (grid bounded by a 512 MB slab).
int spo_expm_run(const void* v, int v_complex, int herm, long npts, int ns, double dt, c128* expV, c128* expVh,
                 hipStream_t st) {
  using namespace spog;
  if (npts == 0) return QD_OK;
  const int threads = std::min(1024, std::max(64, ((ns * ns + 63) / 64) * 64));
  if (ns <= 50) {
    const size_t lds = (size_t)4 * ns * ns * sizeof(c128);
    (void)hipFuncSetAttribute((const void*)spo_expm_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(LDS_MAX - 64));
    (void)hipFuncSetAttribute((const void*)spo_expm_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(LDS_MAX - 64));
    const int grid = (int)std::min<long>(npts, 16384);
    if (v_complex)
      hipLaunchKernelGGL((spo_expm_kernel<true, false>), dim3(grid), dim3(threads), lds, st, v, herm, npts, ns, dt,
                         expV, expVh, nullptr);
    else
      hipLaunchKernelGGL((spo_expm_kernel<false, false>), dim3(grid), dim3(threads), lds, st, v, herm, npts, ns, dt,
                         expV, expVh, nullptr);
    note_path("spo_expm_lds");
  } else {
    const size_t per = (size_t)4 * ns * ns * sizeof(c128);
    const int grid = (int)std::max<long>(1, std::min<long>({npts, 1024, (long)((512ull << 20) / per)}));
    WsScope wss_(st);
    void* work = nullptr;
    const int rc = workspace(WS_SPO, per * grid, &work, st);
    if (rc) return rc;
    if (v_complex)
      hipLaunchKernelGGL((spo_expm_kernel<true, true>), dim3(grid), dim3(threads), 0, st, v, herm, npts, ns, dt, expV,
                         expVh, (c128*)work);
    else
      hipLaunchKernelGGL((spo_expm_kernel<false, true>), dim3(grid), dim3(threads), 0, st, v, herm, npts, ns, dt,
                         expV, expVh, (c128*)work);
    note_path("spo_expm_global");
  }
  QD_HIP(hipGetLastError());
  return QD_OK;
}

// Generic 1D SPO.run (any nx), B wavepackets [B][nx].
int spo1d_generic_run(c128* psi, const c128* expV, const c128* expVh, const c128* expK, int nx, int B, int nt,
                      int nout, c128* snap, hipStream_t st) {
  using namespace spog;
  WsScope wss_(st);
  const long n = (long)nx * B;
  const size_t slots = plan_slots(nx) + (size_t)2 * n + nx;
  void* w = nullptr;
  int rc = workspace(WS_MISC, slots * sizeof(c128), &w, st);
  if (rc) return rc;
  c128* tab = (c128*)w;
  c128* tmp = tab + plan_slots(nx);
  c128* ks = tmp + 2 * n;
  Fft f;
  if ((rc = plan_axis(nx, tab, f, st))) return rc;
  note_path(f.kind == DIRECT ? "spo1d_long" : f.kind == BLUESTEIN ? "spo1d_bluestein" : "spo1d_mixed");
  if (f.kind != DIRECT) {
    const int twl = (size_t)3 * f.M * sizeof(c128) <= LDS_MAX;
    const size_t lds = (size_t)(2 + twl) * f.M * sizeof(c128);
    (void)hipFuncSetAttribute((const void*)spo1d_gen_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
    hipLaunchKernelGGL(spo1d_gen_kernel, dim3(B), dim3(256), lds, st, f, psi, expV, expVh, expK, nt, nout, snap, twl);
    QD_HIP(hipGetLastError());
    return QD_OK;
  }
  // Lines beyond the LDS plans.  Smooth lengths L = L1 L2 with both factors LDS-plannable run the four-step FFT:
  // the line viewed as [L1][L2] (n = L2 n1 + n2), FFT_L1 over n1 (stride L2), twiddle w_L^(n2 k1), FFT_L2 over n2
  // (contiguous) leaves X[k1 + L1 k2] at L2 k1 + k2; the kinetic factor is applied in that order (exp_K permuted once)
  // and the inverse runs the same passes backwards, so no transpose is ever made.  Other lengths: direct DFT.
  int L1 = 0;
  {
    int best = 0;
    for (int a = 2; (long)a * a <= nx; ++a) {
      if (nx % a) continue;
      const int b2 = nx / a;
      if (a <= MAX_LDS_M && b2 <= MAX_LDS_M && all_factors_small(a, GEN_MAXP) && all_factors_small(b2, GEN_MAXP))
        best = a;   // the largest divisor <= sqrt(L): the most balanced split
    }
    L1 = best;
    note_path(L1 ? "spo1d_fourstep" : "spo1d_direct");
  }
  const long total = n;
  auto vmul = [&](const c128* V) -> int {   // psi[b][k] *= V[k]
    hipLaunchKernelGGL(bcast_mul_kernel, dim3(grid_for(total)), dim3(256), 0, st, psi, V, total, nx);
    QD_HIP(hipGetLastError());
    return QD_OK;
  };
  std::function<int()> kstep;
  Exec x;
  c128* tab2 = nullptr;
  if (L1 > 0) {
    const int L2 = nx / L1;
    void* w2 = nullptr;
    if ((rc = workspace(WS_MISC, (plan_slots(L1) + plan_slots(L2)) * sizeof(c128), &w2, st))) return rc;
    tab2 = (c128*)w2;
    x.D = 3;
    x.n[0] = B;
    x.n[1] = L1;
    x.n[2] = L2;
    x.ns = 1;
    x.npts = total;
    x.st = st;
    x.psi = psi;
    x.tmp = tmp;
    if ((rc = plan_axis(L1, tab2, x.f[1], st))) return rc;
    if ((rc = plan_axis(L2, tab2 + plan_slots(L1), x.f[2], st))) return rc;
    hipLaunchKernelGGL(fourstep_kperm_kernel, dim3(grid_for(nx)), dim3(256), 0, st, expK, ks, L1, L2, 1.0 / nx);
    QD_HIP(hipGetLastError());
    kstep = [&, L2]() -> int {
      int r;
      if ((r = x.pass(1, F_FWD, nullptr, nullptr, nullptr))) return r;
      hipLaunchKernelGGL(fourstep_twiddle_kernel, dim3(grid_for(total)), dim3(256), 0, st, psi, total, L1, L2, f.tw, 0);
      if ((r = x.pass(2, F_FWD, nullptr, nullptr, nullptr))) return r;
      hipLaunchKernelGGL(bcast_mul_kernel, dim3(grid_for(total)), dim3(256), 0, st, psi, (const c128*)ks, total, nx);
      if ((r = x.pass(2, F_INV, nullptr, nullptr, nullptr))) return r;
      hipLaunchKernelGGL(fourstep_twiddle_kernel, dim3(grid_for(total)), dim3(256), 0, st, psi, total, L1, L2, f.tw, 1);
      if ((r = x.pass(1, F_INV, nullptr, nullptr, nullptr))) return r;
      QD_HIP(hipGetLastError());
      return QD_OK;
    };
  } else {   // direct DFT lines, one launch sequence per step on the [B][nx] grid
    hipLaunchKernelGGL(scale_copy_kernel, dim3(grid_for(nx)), dim3(256), 0, st, expK, ks, (long)nx, 1.0 / nx);
    QD_HIP(hipGetLastError());
    const dim3 grid((nx + 255) / 256, (unsigned)std::min<long>(B, 65535));
    kstep = [&, grid]() -> int {
      hipLaunchKernelGGL(dft_axis_kernel<false>, grid, dim3(256), 0, st, (const c128*)psi, tmp, (long)B, nx, 1L, f.tw);
      hipLaunchKernelGGL(bcast_mul_kernel, dim3(grid_for(total)), dim3(256), 0, st, tmp, (const c128*)ks, total, nx);
      hipLaunchKernelGGL(dft_axis_kernel<true>, grid, dim3(256), 0, st, (const c128*)tmp, psi, (long)B, nx, 1L, f.tw);
      QD_HIP(hipGetLastError());
      return QD_OK;
    };
  }
  if ((rc = vmul(expVh))) return rc;
  const int nblk = nt / nout;
  const int nsnap = nblk > 0 ? nblk - 1 : 0;
  for (int blk = 1; blk < nblk; ++blk) {
    for (int s = 0; s < nout; ++s) {
      if ((rc = kstep())) return rc;
      if ((rc = vmul(expV))) return rc;
    }
    if (snap)
      for (int b = 0; b < B; ++b)
        QD_TRY(copy_device(snap + ((size_t)b * nsnap + (blk - 1)) * nx, psi + (size_t)b * nx, nx * sizeof(c128), st));
  }
  if ((rc = kstep())) return rc;
  return vmul(expVh);
}

}  // namespace qd
