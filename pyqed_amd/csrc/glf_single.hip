// glf_single.hip — a few density matrices (one trajectory: LindbladSolver.run, oqs.py:1596-1696) as ONE persistent
// launch.
//
// The batch kernels give one CU per density matrix, and the split path (glf.hip) spreads one matrix over many
// workgroups but pays eight dependent launches per RK4 step, each a chain of operand-load / slab / ticket round trips
// (~10 us per launch, 12.3k steps/s at N = 128).  Here every 16 x 16 output tile of every matrix is a workgroup
// (T = Np / 16, T^2 workgroups per matrix, B T^2 <= 256) that lives for the whole run:
//   - its slices of the constant operators (P rows, Q columns, L_c rows, R_c columns of the GLF form
//     d rho/dt = P rho + rho Q + sum_c L_c rho R_c) are loaded ONCE into registers in the MFMA fragment layout;
//   - its tile of rho stays in registers (threads 0..255, one element each);
//   - the 8 waves split K = Np into 8 chunks (KS k-steps of 4 each) and the partial tiles are summed in LDS in the
//     fixed wave order (deterministic);
//   - split roles (round 5, while 2 B T^2 <= 256): a second workgroup per tile computes and publishes the Y_c tile,
//     so the tile's k workgroup runs P r + r Q while the row's Y_c tiles are made (N = 128, one matrix: 35.5k ->
//     39.6k steps/s, profiles/r05/lindblad/glf_single_split_roles.txt); otherwise one workgroup does both in turn;
//   - at N_p = 128 the Y workgroup also makes the tile's P r (see PRY below);
//   - per RK4 stage two hand-offs inside the launch: Y_c(bm, bn) = L_c[bm, :] r[:, bn] is published, then
//     k(bm, bn) = P[bm, :] r[:, bn] + r[bm, :] Q[:, bn] + sum_c Y_c[bm, :] R_c[:, bn] needs the Y_c row block bm;
//     the Horner update s' = rho + dt / (4 - m) k (glf.hip header) is published as the next stage input, whose row
//     block bm and column block bn the next stage reads.
// Hand-off form (cdna_hip_programming.md Guideline 16, R2: the data is the flag): every handed-off double carries the
// parity of its epoch in its lowest mantissa bit, stored with 16-B write-through (sc1) buffer stores (no drain, no
// barrier, no flag word); each consuming wave re-loads with 16-B sc1 buffer loads until every granule of its chunk
// holds the expected parity (granules observed untorn on gfx950, MI355X_MICROARCH.md "Valid forms").  Stage outputs
// and Y_c alternate between two buffers, so a buffer's previous contents (two stages back) carry the other parity,
// and the host presets each buffer to the parity its first epoch does not have.  The tag perturbs a handed-off value
// by at most one unit in its last place; it enters the result only through dt k(r), never the state rho the
// workgroup keeps in registers.  Against the epoch-flag form (drain, barrier, flag, poll, barrier, load): N = 128, one
// matrix 39.9k -> 43.5k steps/s, N = 64 50k -> 70k, N = 32 61k -> 92k (profiles/r05/lindblad/glf_single_r2.txt).
// Buffer reuse: stage outputs and Y_c alternate between two buffers.  A workgroup overwrites r_{g-1} (buffer
// (g+1) & 1) at the end of stage g only after it has loaded stage g's Y_c of every workgroup of its row and stage g's
// input from every workgroup of its row and column, i.e. after every reader of its r_{g-1} tile (the workgroups of
// its row and column) finished loading in stage g - 1 (their stage-g values depend on what they loaded); likewise
// Y_{g-2} and the P r tile (buffer g & 1) are overwritten in stage g after every reader of them (the row; the tile's k
// workgroup) produced stage g - 1's output, loaded at the start of stage g.  Every spin is bounded; a timeout sets
// *status (the host re-runs the batch on the split path).
// Observables: each workgroup sums Tr(E rho) over its tile after every step into a partial slot, and one small
// kernel adds the T^2 partials in fixed order after the launch.
#include "glf_kernel.hpp"
#include "handoff.hpp"

namespace qd {
namespace {

constexpr int SG_WG = 512;
constexpr unsigned SG_SPIN_LIMIT = 1u << 22;    // sweeps (one round trip each, s_sleep between): ~2 s

struct SingleParams {
  const c128* P;       // [Np][Np] padded GLF operators (glf_run's operator workspace)
  const c128* Q;
  const c128* Lop;     // [nc][Np][Np]
  const c128* Rop;     // [nc][Np][Np]
  const c128* eT;      // [ne][Np][Np] E_m^T
  c128* rho;           // [B][Np][Np] state (in / out)
  c128* rbuf;          // [2][B][Np][Np] stage outputs
  c128* ybuf;          // [2][nc][B][Np][Np] Y_c, then [2][B][Np][Np] P r tiles (split roles)
  c128* obs_part;      // [B][total_steps + 1][ne][T^2]
  c128* snap;          // [B][nsave][N][N] or null
  int* status;
  unsigned long long* tim;   // QD_PHASE_TIMING builds: [grid][8] wall-clock ticks per phase (thread 0's view)
  int N, ne, nsteps, step0, total_steps, save_every, nsave;
  int split;           // 1: a second workgroup per tile computes the Y_c tiles (grid = 2 B T^2)
  int B;               // matrices (the Hermitian launch)
  double dt;
};

#ifdef QD_PHASE_TIMING
#define SG_MARK(k)                                 \
  if (tid == 0) {                                  \
    const unsigned long long now_ = wall_clock64(); \
    tacc[k] += now_ - tlast;                       \
    tlast = now_;                                  \
  }
#else
#define SG_MARK(k)
#endif

// the epoch parity t in the lowest mantissa bit of both halves (at most one unit in the last place)
__device__ __forceinline__ c128 sg_tag(c128 v, unsigned t) {
  const unsigned long long a = __builtin_bit_cast(unsigned long long, v.re);
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v.im);
  return cmk(__builtin_bit_cast(double, (a & ~1ull) | t), __builtin_bit_cast(double, (b & ~1ull) | t));
}
__device__ __forceinline__ bool sg_has(c128 v, unsigned t) {
  const unsigned a = (unsigned)__builtin_bit_cast(unsigned long long, v.re);
  const unsigned b = (unsigned)__builtin_bit_cast(unsigned long long, v.im);
  return (((a ^ t) | (b ^ t)) & 1u) == 0;
}
// One wave loads its NL handed-off granules (byte offsets off(q)) with sc1 loads and re-loads the ones without parity
// t until all have it, s_sleep(1) between passes.  FS: s_sleep units (64 clocks) before the first pass -- a pass
// issued before the producers' stores can have landed only adds traffic (profiles/r05/lindblad/glf_single_r2.txt).
// False after SG_SPIN_LIMIT sweeps or when another workgroup reported a timeout (*status).
template <int FS, int NL, typename Off>
__device__ __forceinline__ bool sg_sweep(c128 (&v)[NL], __amdgpu_buffer_rsrc_t rs, Off off, unsigned t, int* status,
                                         int lane) {
  if constexpr (FS > 0) __builtin_amdgcn_s_sleep(FS > 8 ? 8 : FS);   // the first pass after the data can land
  if constexpr (FS > 8) __builtin_amdgcn_s_sleep(FS - 8);
#pragma unroll
  for (int q = 0; q < NL; ++q) v[q] = ld16_sc1(rs, off(q));
  for (unsigned spins = 0;;) {
    bool okq[NL], ok = true;
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      okq[q] = sg_has(v[q], t);
      ok &= okq[q];
    }
    if (__all(ok)) return true;
    ++spins;
    if (spins > SG_SPIN_LIMIT ||
        ((spins & 255) == 0 && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      if (lane == 0) __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");   // the granules change under us: re-load, never reuse the value
#pragma unroll
    for (int q = 0; q < NL; ++q)
      if (!okq[q]) v[q] = ld16_sc1(rs, off(q));
  }
}

// Split roles at N_p = 128: before a sweep a wave sleeps num/8 of its previous stage's wait for the same data (Y
// workgroups' stage input 6/8, k workgroups' stage input 4/8 and Y_c rows 4/8; capped at 20 us), so the passes that
// could only find stale data -- traffic in the way of the k workgroups' loads -- are skipped; self-tuning, it settles
// below the data's arrival (a factor f overshoots for good once f RT / (1 - f) exceeds the wait: 7/8 was slower).
// N = 128 one matrix 43.3k -> 47.3k, two 73k -> 80k (profiles/r05/lindblad/glf_single_adaptive_delay.txt)
constexpr int SG_ADAPT_Y = 6, SG_ADAPT_K = 4, SG_ADAPT_KY = 4;
__device__ __forceinline__ unsigned long long sg_delay_ticks(unsigned long long prev, int num) {
  const unsigned long long d = prev * (unsigned)num / 8u;
  return d < 2000u ? d : 2000u;
}
__device__ __forceinline__ void sg_delay_until(unsigned long long t) {
  while (wall_clock64() < t) __builtin_amdgcn_s_sleep(2);
}

// one complex k-step of a 16 x 16 tile: acc += a b (a: A fragment, b: B fragment of v_mfma_f64_16x16x4_f64)
__device__ __forceinline__ void sg_mac(d4& re, d4& im, c128 a, c128 b) {
  re = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.re, re, 0, 0, 0);
  im = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.im, im, 0, 0, 0);
  re = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.im, b.im, re, 0, 0, 0);
  im = __builtin_amdgcn_mfma_f64_16x16x4f64(a.im, b.re, im, 0, 0, 0);
}

// A 16 x 16 complex accumulator.  M3 = false: 4 real MFMAs per complex k-step (re += ar br - ai bi, im += ar bi + ai br).
// M3 = true: the 3-product form, P1 += ar br, P2 += ai bi, P3 += (ar + ai)(br + bi), re = P1 - P2, im = P3 - P1 - P2
// (3 MFMAs per k-step; the two operand sums are VALU adds beside the MFMAs; one accumulator set more).
template <bool M3>
struct SgAcc {
  d4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0}, a2 = {0, 0, 0, 0};
  __device__ __forceinline__ void mac(c128 a, c128 b) {
    if constexpr (M3) {
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re, b.re, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.im, b.im, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.re + a.im, b.re + b.im, a2, 0, 0, 0);
    } else {
      sg_mac(a0, a1, a, b);
    }
  }
  __device__ __forceinline__ void result(d4& re, d4& im) const {
    if constexpr (M3) {
      re = a0 - a1;
      im = a2 - a0 - a1;
    } else {
      re = a0;
      im = a1;
    }
  }
};

// KS: k-steps of 4 per wave (Np = 32 KS), NC collapse operators / GLF pairs, M3: SgAcc form, SPLIT: p.split (a
// workgroup holds only its role's operator fragments)
template <int KS, int NC, bool M3, bool SPLIT>
__global__ __launch_bounds__(SG_WG) void glf_single_kernel(SingleParams p) {
  constexpr int T = 2 * KS, Np = 32 * KS, NN = Np * Np;
  // partial tiles of the reductions, by stage parity: a wave writes stage g + 2's partials only after the barrier of
  // stage g + 1, which every wave reaches after reading stage g's (there is no other barrier between stages)
  __shared__ c128 red[2][8][256];
  __shared__ int sAbort[2];   // a wave's timed-out sweep in stage g sets sAbort[g & 1]; read after the next barrier
  // split: workgroups [0, B T^2) are the tiles' k workgroups, [B T^2, 2 B T^2) their Y workgroups
  const int nk = SPLIT ? (int)gridDim.x / 2 : (int)gridDim.x;
  const bool yrole = SPLIT && (int)blockIdx.x >= nk;
  const int w = yrole ? (int)blockIdx.x - nk : (int)blockIdx.x;
  const int b = w / (T * T), tile = w - b * (T * T), bm = tile / T, bn = tile - bm * T;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
  const int kb = wave * 4 * KS;
  // split roles at N_p = 128: the Y workgroup also makes the tile's P r (from the column it reads anyway), so the k
  // workgroup ingests the row of r and the row of Y_c only -- per-CU load bandwidth, not the MFMAs, bounds the stage
  // there (N = 128, one matrix: 42.2k -> 43.5k steps/s; at N_p = 32 / 64 the extra hand-off costs more than it saves,
  // profiles/r05/lindblad/glf_single_r2.txt)
  constexpr bool PRY = SPLIT && KS == 4;
  // adaptive sweep delays (SG_ADAPT_*) at N_p = 128 with split roles; at N_p = 32 / 64 they measured 0-2 % slower
  // than the static first-pass delays FS (glf_single_adaptive_delay.txt)
  constexpr bool ADAPT = PRY;
  // delay before a sweep's first pass (s_sleep units), per shape class: none where one matrix's tiles hand off at
  // N_p = 128 or many N_p = 32 matrices run joint, else 8 or 16 (N = 128 four matrices 112k -> 121k, N = 64 sixteen
  // 746k -> 794k, N = 32 thirty-two 2.42M -> 2.60M; profiles/r05/lindblad/glf_single_first_sweep.txt)
  constexpr int FS = (KS == 4 && SPLIT) || (KS == 1 && !SPLIT) ? 0 : (KS == 2 && SPLIT) ? 8 : 16;
  // constant operator fragments, loaded once: A rows bm (L_c at [c], P at [NC]), B columns bn (R_c, Q); with split
  // roles a Y workgroup holds the A fragments and a k workgroup the B fragments, in the same registers (a k workgroup
  // that makes P r itself holds P in aPk)
  c128 fA[NC + 1][KS], fBj[NC + 1][KS], aPk[SPLIT && !PRY ? KS : 1];
  c128(&fB)[NC + 1][KS] = SPLIT ? fA : fBj;
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int k = kb + 4 * q + lk;
    if constexpr (SPLIT && !PRY)
      if (!yrole) aPk[q] = p.P[(bm * 16 + lr) * Np + k];
    if (!SPLIT || yrole) {
      fA[NC][q] = p.P[(bm * 16 + lr) * Np + k];
#pragma unroll
      for (int c = 0; c < NC; ++c) fA[c][q] = p.Lop[(size_t)c * NN + (bm * 16 + lr) * Np + k];
    }
    if (!SPLIT || !yrole) {
      fB[NC][q] = p.Q[k * Np + bn * 16 + lr];
#pragma unroll
      for (int c = 0; c < NC; ++c) fB[c][q] = p.Rop[(size_t)c * NN + k * Np + bn * 16 + lr];
    }
  }
  const bool owner = tid < 256 && !yrole;
  const int orow = bm * 16 + ((tid >> 4) & 15), ocol = bn * 16 + (tid & 15);
  c128* rhob = p.rho + (size_t)b * NN;
  c128 rh = owner ? rhob[orow * Np + ocol] : cmk(0, 0);
  if (tid < 2) sAbort[tid] = 0;
  __syncthreads();
  const int mats = nk / (T * T);
  const int slab = mats * NN * (int)sizeof(c128);   // bytes of one [B][Np][Np] buffer

  // Tr(E_m rho) partial over this tile -> obs_part (fixed-order sums: lanes of a wave, then the 4 owner waves)
  auto observe = [&](int gs) {
    for (int m = 0; m < p.ne; ++m) {
      c128 v = cmk(0, 0);
      if (owner) v = cmul(rh, p.eT[(size_t)m * NN + orow * Np + ocol]);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        v.re += __shfl_xor(v.re, off, 64);
        v.im += __shfl_xor(v.im, off, 64);
      }
      __syncthreads();
      if (lane == 0) red[0][0][wave] = v;
      __syncthreads();
      if (tid == 0) {
        c128 s = red[0][0][0];
        for (int q = 1; q < 4; ++q) s = cadd(s, red[0][0][q]);
        p.obs_part[(((size_t)b * (p.total_steps + 1) + gs) * p.ne + m) * (T * T) + tile] = s;
      }
    }
  };
  if (p.ne > 0 && p.step0 == 0 && !yrole) observe(0);

  // fixed-order sum of the 8 waves' partial tiles (slot par); returns element tid (tid < 256) of the tile
  auto reduce = [&](const SgAcc<M3>& acc, int par) -> c128 {
    d4 re, im;
    acc.result(re, im);
#pragma unroll
    for (int r = 0; r < 4; ++r) red[par][wave][(lk + 4 * r) * 16 + lr] = cmk(re[r], im[r]);
    __syncthreads();
    c128 v = cmk(0, 0);
    if (tid < 256) {
      v = red[par][0][tid];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = cadd(v, red[par][q][tid]);
    }
    return v;
  };

#ifdef QD_PHASE_TIMING
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tlast = wall_clock64();
#endif
  const int G4 = 4 * p.nsteps;
  unsigned long long wy = 0, wk = 0, wky = 0;   // this wave's last waits (10 ns ticks): Y / k stage input, Y_c rows
  for (int g = 0; g < G4; ++g) {
    const int s = g >> 2, m = g & 3, par = g & 1;
    // r_j (j >= 1) lives in rbuf[j & 1] with parity (j >> 1) & 1, Y_g in ybuf[g & 1] with parity (g >> 1) & 1
    const unsigned tr = (unsigned)(g >> 1) & 1u, ty = tr;
    bool good = true;
    // ---- stage input r_g: the caller's rho at g = 0, else the previous stage's output in rbuf[g & 1]; column bn
    // and row bm (a Y workgroup reads the column only)
    const c128* rin = g == 0 ? p.rho : p.rbuf + (size_t)(g & 1) * mats * NN;
    const __amdgpu_buffer_rsrc_t rr = sc1_rsrc(rin, slab);
    c128 rcol[KS], rrow[KS];
    auto col_off = [&](int q) { return ((b * Np + kb + 4 * q + lk) * Np + bn * 16 + lr) * 16; };
    auto row_off = [&](int q) { return ((b * Np + bm * 16 + lr) * Np + kb + 4 * q + lk) * 16; };
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        if (yrole || !PRY) rcol[q] = ld16_sc1(rr, col_off(q));
        if (!yrole) rrow[q] = ld16_sc1(rr, row_off(q));
      }
    } else if (yrole) {
      const unsigned long long t0 = ADAPT ? wall_clock64() : 0;
      if constexpr (ADAPT) sg_delay_until(t0 + sg_delay_ticks(wy, SG_ADAPT_Y));
      good = sg_sweep<ADAPT ? 0 : FS>(rcol, rr, col_off, tr, p.status, lane);
      if constexpr (ADAPT) wy = wall_clock64() - t0;
    } else if (PRY) {   // the k workgroup reads the row only (its Y workgroup makes P r)
      const unsigned long long t0 = wall_clock64();
      sg_delay_until(t0 + sg_delay_ticks(wk, SG_ADAPT_K));
      good = sg_sweep<FS>(rrow, rr, row_off, tr, p.status, lane);
      wk = wall_clock64() - t0;
    } else if (NC > 1 && KS == 4) {   // (one sweep of both would spill here)
      good = sg_sweep<FS>(rcol, rr, col_off, tr, p.status, lane);
      if (good) good = sg_sweep<0>(rrow, rr, row_off, tr, p.status, lane);
    } else {   // column and row in one sweep: one round trip per pass for both
      c128 rcr[2 * KS];
      const unsigned long long t0 = ADAPT ? wall_clock64() : 0;
      if constexpr (ADAPT) sg_delay_until(t0 + sg_delay_ticks(wk, SG_ADAPT_K));
      good = sg_sweep<ADAPT ? 0 : FS>(rcr, rr, [&](int q) { return q < KS ? col_off(q) : row_off(q - KS); }, tr,
                                      p.status, lane);
      if constexpr (ADAPT) wk = wall_clock64() - t0;
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        rcol[q] = rcr[q];
        rrow[q] = rcr[KS + q];
      }
    }
    if (!good && lane == 0) sAbort[par] = 1;
    SG_MARK(0)
    // ---- Y_c(bm, bn) = L_c[bm, :] r[:, bn], handed to the k phase of the row
    // ybuf: [2][NC][B][Np][Np] Y_c, then (split roles) [2][B][Np][Np] P r tiles, one descriptor over both
    const int yo = (g & 1) * NC * mats * NN, vo = (2 * NC + (g & 1)) * mats * NN;
    const __amdgpu_buffer_rsrc_t ry = sc1_rsrc(p.ybuf, 2 * (NC + 1) * slab);
    if (NC > 0 && (yrole || !SPLIT)) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        SgAcc<M3> acc;
#pragma unroll
        for (int q = 0; q < KS; ++q) acc.mac(fA[c][q], rcol[q]);
        const c128 y = reduce(acc, par);
        if (c + 1 < NC) __syncthreads();   // the slot is reused by the next reduction
        if (tid < 256) st16_sc1(ry, (yo + ((c * mats + b) * Np + orow) * Np + ocol) * 16, sg_tag(y, ty));
      }
      if (yrole) {
        if constexpr (PRY) {   // P r (bm, bn) for the tile's k workgroup
          SgAcc<M3> av;
#pragma unroll
          for (int q = 0; q < KS; ++q) av.mac(fA[NC][q], rcol[q]);
          __syncthreads();   // the Y reduction's slot
          const c128 pv = reduce(av, par);
          if (tid < 256) st16_sc1(ry, (vo + (b * Np + orow) * Np + ocol) * 16, sg_tag(pv, ty));
        }
        if (sAbort[par]) break;   // read after the reductions' barriers, which a timed-out wave reached
        SG_MARK(1)
        continue;
      }
    }
    SG_MARK(1)
    // ---- k(bm, bn) = P r + r Q + sum_c Y_c R_c; the P r + r Q part runs while the row's Y_c are handed over
    SgAcc<M3> acc;
    if constexpr (!SPLIT) {
#pragma unroll
      for (int q = 0; q < KS; ++q) acc.mac(fA[NC][q], rcol[q]);
    } else if constexpr (!PRY) {
#pragma unroll
      for (int q = 0; q < KS; ++q) acc.mac(aPk[q], rcol[q]);
    }
#pragma unroll
    for (int q = 0; q < KS; ++q) acc.mac(rrow[q], fB[NC][q]);
    SG_MARK(2)
    c128 pv = cmk(0, 0);   // PRY: the P r tile of the Y workgroup (element tid & 255)
    if constexpr (NC > 0) {
      if (!SPLIT) __syncthreads();   // this stage's Y reductions read the slot the k reduction writes
      c128 yrow[NC][KS];
      auto y_off = [&](int c, int q) {
        return (yo + ((c * mats + b) * Np + bm * 16 + lr) * Np + kb + 4 * q + lk) * 16;
      };
      const unsigned long long ty0 = ADAPT ? wall_clock64() : 0;
      if constexpr (ADAPT) sg_delay_until(ty0 + sg_delay_ticks(wky, SG_ADAPT_KY));
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (good) good = sg_sweep<ADAPT ? 0 : FS>(yrow[c], ry, [&](int q) { return y_off(c, q); }, ty, p.status, lane);
      if constexpr (ADAPT) wky = wall_clock64() - ty0;
      SG_MARK(3)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < KS; ++q) acc.mac(yrow[c][q], fB[c][q]);
      if (PRY && good) {   // the P r element (tid & 255), published after the tile's Y_c, sought under the MFMAs
        c128 pe[1];
        const int v_off = (vo + (b * Np + bm * 16 + ((tid >> 4) & 15)) * Np + bn * 16 + (tid & 15)) * 16;
        good = sg_sweep<FS>(pe, ry, [&](int) { return v_off; }, ty, p.status, lane);
        pv = pe[0];
      }
      if (!good && lane == 0) sAbort[par] = 1;
    }
    const c128 kv = cadd(reduce(acc, par), pv);
    if (sAbort[par]) break;
    SG_MARK(4)
    const double hc = rk4_horner_coef(p.dt, m);
    const c128 v = cadd(rh, cscale(kv, hc));
    if (m == 3) rh = v;
    if (owner && g + 1 < G4)
      st16_sc1(sc1_rsrc(p.rbuf + (size_t)((g + 1) & 1) * mats * NN, slab), ((b * Np + orow) * Np + ocol) * 16,
               sg_tag(v, (unsigned)((g + 1) >> 1) & 1u));
    if (m == 3) {
      const int gs = p.step0 + s + 1;
      if (p.snap && p.save_every > 0 && gs % p.save_every == 0) {
        const int si = gs / p.save_every - 1;
        if (owner && si < p.nsave && orow < p.N && ocol < p.N)
          p.snap[(((size_t)b * p.nsave + si) * p.N + orow) * p.N + ocol] = v;
      }
      if (p.ne > 0) observe(gs);
    }
    SG_MARK(5)
  }
  if (owner) rhob[orow * Np + ocol] = rh;
#ifdef QD_PHASE_TIMING
  if (tid == 0 && p.tim)
    for (int k = 0; k < 6; ++k) p.tim[(size_t)blockIdx.x * 8 + k] = tacc[k];
#endif
}

// ---------------------------------------------------------------- Hermitian single launch (N_p = 128)
// For exactly Hermitian H and rho (the usual LindbladSolver.run case) the right-hand side is
//   k = P r + (P r)^+ + sum_c (C_c r) C_c^+,   P = -iK,
// Hermitian itself, so only the T (T + 1) / 2 tiles with bm <= bn are made.  Roles:
//   - Y workgroups (every tile (bm, bn), as the general launch's split roles): sweep the column bn of the stage input,
//     publish Y_c(bm, bn) = C_c[bm, :] r[:, bn] and the tile (P r)(bm, bn);
//   - k workgroups (the upper tiles): never read the stage input -- they sweep the Y_c row bm and the two tiles
//     (P r)(bm, bn), (P r)(bn, bm), form t = sum_c Y_c[bm, :] (C_c^+ / 2)[:, bn] on the MFMAs and
//       bm < bn:  k = (P r)(bm, bn) + conj((P r)(bn, bm))^T + 2 t      (the halved operator doubled: exact)
//       bm = bn:  k = (P r)(bm, bm) + conj((P r)(bm, bm))^T + (t + conj(t)^T)
//     (every element's mirror is formed from the same operands in the commuted order, so each diagonal tile -- and with
//     the mirrors written as conjugates, every stage -- is Hermitian bit for bit), update s = rho + dt / (4 - m) k and
//     publish the tile and, off the diagonal, its conjugate transpose at (bn, bm).
// So a k workgroup ingests one 32 KB strip (Y_c row, per c) and two tiles instead of two strips, and a stage runs
// 64 (1 + nc) + 36 nc tile products instead of 64 (2 + 2 nc).  Hand-offs, buffers and parities as the general launch;
// the buffer-reuse order holds through the Y workgroups' P r tiles (a tile's owner consumed, in stage g - 1, the P r or
// Y_c tile of every Y workgroup that reads its tile).
template <int NC, bool M3>
__global__ __launch_bounds__(SG_WG) void glf_single_herm_kernel(SingleParams p) {
  constexpr int KS = 4, T = 8, Np = 128, NN = Np * Np, TU = T * (T + 1) / 2;
  __shared__ c128 red[2][8][256];
  __shared__ c128 tT[256];    // the diagonal tiles' t, for its transpose
  __shared__ int sAbort[2];
  const int mats = p.B;
  const int nk = mats * TU;
  const bool yrole = (int)blockIdx.x >= nk;
  int b, bm, bn;
  if (yrole) {
    const int w = (int)blockIdx.x - nk;
    b = w / (T * T);
    bm = (w - b * T * T) / T;
    bn = w - b * T * T - bm * T;
  } else {
    b = (int)blockIdx.x / TU;
    int u = (int)blockIdx.x - b * TU;
    bm = 0;
    while (u >= T - bm) {   // upper pair u -> (bm, bn), row-major over bm <= bn
      u -= T - bm;
      ++bm;
    }
    bn = bm + u;
  }
  const bool diag = bm == bn;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
  const int kb = wave * 4 * KS;
  // Y workgroups: A fragments (rows bm of C_c and of P); k workgroups: B fragments (columns bn of C_c^+ / 2)
  c128 fA[NC + 1][KS];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int k = kb + 4 * q + lk;
    if (yrole) {
      fA[NC][q] = p.P[(bm * 16 + lr) * Np + k];
#pragma unroll
      for (int c = 0; c < NC; ++c) fA[c][q] = p.Lop[(size_t)c * NN + (bm * 16 + lr) * Np + k];
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c) fA[c][q] = p.Rop[(size_t)c * NN + k * Np + bn * 16 + lr];
    }
  }
  const bool owner = tid < 256 && !yrole;
  const int ti = (tid >> 4) & 15, tj = tid & 15;
  const int orow = bm * 16 + ti, ocol = bn * 16 + tj;
  c128* rhob = p.rho + (size_t)b * NN;
  c128 rh = owner ? rhob[orow * Np + ocol] : cmk(0, 0);
  if (tid < 2) sAbort[tid] = 0;
  __syncthreads();
  const int slab = mats * NN * (int)sizeof(c128);

  // Tr(E_m rho) over the tile and (off the diagonal) its mirror -> slot (bm, bn); slot (bn, bm) gets zero
  auto observe = [&](int gs) {
    for (int m = 0; m < p.ne; ++m) {
      c128 v = cmk(0, 0);
      if (owner) {
        const c128* E = p.eT + (size_t)m * NN;
        v = cmul(rh, E[orow * Np + ocol]);
        if (!diag) v = cadd(v, cmul(cconj(rh), E[ocol * Np + orow]));
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        v.re += __shfl_xor(v.re, off, 64);
        v.im += __shfl_xor(v.im, off, 64);
      }
      __syncthreads();
      if (lane == 0) red[0][0][wave] = v;
      __syncthreads();
      if (tid == 0) {
        c128 s = red[0][0][0];
        for (int q = 1; q < 4; ++q) s = cadd(s, red[0][0][q]);
        c128* part = p.obs_part + (((size_t)b * (p.total_steps + 1) + gs) * p.ne + m) * (T * T);
        part[bm * T + bn] = s;
        if (!diag) part[bn * T + bm] = cmk(0, 0);
      }
    }
  };
  if (p.ne > 0 && p.step0 == 0 && !yrole) observe(0);

  auto reduce = [&](const SgAcc<M3>& acc, int par) -> c128 {
    d4 re, im;
    acc.result(re, im);
#pragma unroll
    for (int r = 0; r < 4; ++r) red[par][wave][(lk + 4 * r) * 16 + lr] = cmk(re[r], im[r]);
    __syncthreads();
    c128 v = cmk(0, 0);
    if (tid < 256) {
      v = red[par][0][tid];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = cadd(v, red[par][q][tid]);
    }
    return v;
  };

#ifdef QD_PHASE_TIMING
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tlast = wall_clock64();
#endif
  const int G4 = 4 * p.nsteps;
  unsigned long long wy = 0, wky = 0;
  for (int g = 0; g < G4; ++g) {
    const int s = g >> 2, m = g & 3, par = g & 1;
    const unsigned tr = (unsigned)(g >> 1) & 1u, ty = tr;
    bool good = true;
    const int yo = (g & 1) * NC * mats * NN, vo = (2 * NC + (g & 1)) * mats * NN;
    const __amdgpu_buffer_rsrc_t ry = sc1_rsrc(p.ybuf, 2 * (NC + 1) * slab);
    if (yrole) {
      // ---- stage input column bn -> Y_c(bm, bn), (P r)(bm, bn)
      const c128* rin = g == 0 ? p.rho : p.rbuf + (size_t)(g & 1) * mats * NN;
      const __amdgpu_buffer_rsrc_t rr = sc1_rsrc(rin, slab);
      c128 rcol[KS];
      auto col_off = [&](int q) { return ((b * Np + kb + 4 * q + lk) * Np + bn * 16 + lr) * 16; };
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < KS; ++q) rcol[q] = ld16_sc1(rr, col_off(q));
      } else {
        const unsigned long long t0 = wall_clock64();
        sg_delay_until(t0 + sg_delay_ticks(wy, SG_ADAPT_Y));
        good = sg_sweep<0>(rcol, rr, col_off, tr, p.status, lane);
        wy = wall_clock64() - t0;
      }
      if (!good && lane == 0) sAbort[par] = 1;
      SG_MARK(0)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        SgAcc<M3> acc;
#pragma unroll
        for (int q = 0; q < KS; ++q) acc.mac(fA[c][q], rcol[q]);
        const c128 y = reduce(acc, par);
        __syncthreads();   // the slot is reused by the next reduction
        if (tid < 256) st16_sc1(ry, (yo + ((c * mats + b) * Np + orow) * Np + ocol) * 16, sg_tag(y, ty));
      }
      SgAcc<M3> av;
#pragma unroll
      for (int q = 0; q < KS; ++q) av.mac(fA[NC][q], rcol[q]);
      const c128 pv = reduce(av, par);
      if (tid < 256) st16_sc1(ry, (vo + (b * Np + orow) * Np + ocol) * 16, sg_tag(pv, ty));
      if (sAbort[par]) break;   // read after the reductions' barriers, which a timed-out wave reached
      SG_MARK(1)
      continue;
    }
    // ---- k workgroup: t = sum_c Y_c[bm, :] (C_c^+ / 2)[:, bn]
    c128 t = cmk(0, 0);
    c128 pe[2];
    auto sweep_pr = [&]() {
      const int o1 = (vo + (b * Np + bm * 16 + ti) * Np + bn * 16 + tj) * 16;
      const int o2 = (vo + (b * Np + bn * 16 + tj) * Np + bm * 16 + ti) * 16;
      return sg_sweep<0>(pe, ry, [&](int q) { return q ? o2 : o1; }, ty, p.status, lane);
    };
    if constexpr (NC > 0) {
      c128 yrow[NC][KS];
      auto y_off = [&](int c, int q) {
        return (yo + ((c * mats + b) * Np + bm * 16 + lr) * Np + kb + 4 * q + lk) * 16;
      };
      const unsigned long long t0 = wall_clock64();
      sg_delay_until(t0 + sg_delay_ticks(wky, SG_ADAPT_KY));
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (good) good = sg_sweep<0>(yrow[c], ry, [&](int q) { return y_off(c, q); }, ty, p.status, lane);
      wky = wall_clock64() - t0;
      SG_MARK(3)
      SgAcc<M3> acc;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < KS; ++q) acc.mac(yrow[c][q], fA[c][q]);
      // the two P r tiles (element (ti, tj) of (bm, bn) and element (tj, ti) of (bn, bm)), sought under the MFMAs
      if (good) good = sweep_pr();
      if (!good && lane == 0) sAbort[par] = 1;
      t = reduce(acc, par);
    } else {
      if (good) good = sweep_pr();
      if (!good && lane == 0) sAbort[par] = 1;
      __syncthreads();
    }
    if (diag) {
      if (tid < 256) tT[tid] = t;
    }
    __syncthreads();
    if (sAbort[par]) break;
    SG_MARK(4)
    c128 kv;
    if (diag) {
      const c128 tt = tT[tj * 16 + ti];
      kv = cadd(cadd(pe[0], cconj(pe[1])), cadd(t, cconj(tt)));
    } else {
      kv = cadd(cadd(pe[0], cconj(pe[1])), cmk(t.re + t.re, t.im + t.im));
    }
    const double hc = rk4_horner_coef(p.dt, m);
    const c128 v = cadd(rh, cscale(kv, hc));
    if (m == 3) rh = v;
    if (owner && g + 1 < G4) {
      const __amdgpu_buffer_rsrc_t ro = sc1_rsrc(p.rbuf + (size_t)((g + 1) & 1) * mats * NN, slab);
      const unsigned tn = (unsigned)((g + 1) >> 1) & 1u;
      st16_sc1(ro, ((b * Np + orow) * Np + ocol) * 16, sg_tag(v, tn));
      if (!diag) st16_sc1(ro, ((b * Np + ocol) * Np + orow) * 16, sg_tag(cconj(v), tn));
    }
    if (m == 3) {
      const int gs = p.step0 + s + 1;
      if (p.snap && p.save_every > 0 && gs % p.save_every == 0) {
        const int si = gs / p.save_every - 1;
        if (owner && si < p.nsave) {
          c128* sn = p.snap + ((size_t)b * p.nsave + si) * p.N * p.N;
          if (orow < p.N && ocol < p.N) {
            sn[(size_t)orow * p.N + ocol] = v;
            if (!diag) sn[(size_t)ocol * p.N + orow] = cconj(v);
          }
        }
      }
      if (p.ne > 0) observe(gs);
    }
    SG_MARK(5)
  }
  if (owner) {
    rhob[orow * Np + ocol] = rh;
    if (!diag) rhob[ocol * Np + orow] = cconj(rh);
  }
#ifdef QD_PHASE_TIMING
  if (tid == 0 && p.tim)
    for (int k = 0; k < 6; ++k) p.tim[(size_t)blockIdx.x * 8 + k] = tacc[k];
#endif
}

template <int NC, bool M3>
hipError_t sgh_launch2(SingleParams p, int grid, bool coop, hipStream_t st) {
  if (!coop) {
    hipLaunchKernelGGL((glf_single_herm_kernel<NC, M3>), dim3(grid), dim3(SG_WG), 0, st, p);
    return hipGetLastError();
  }
  void* args[] = {(void*)&p};
  return hipLaunchCooperativeKernel((const void*)glf_single_herm_kernel<NC, M3>, dim3(grid), dim3(SG_WG), args, 0, st);
}
template <int NC>
hipError_t sgh_launch(SingleParams p, int B, bool coop, hipStream_t st, int& grid) {
  grid = B * (36 + 64);
  const bool m3 = grid <= 128 && NC < 2;   // (NC = 2 with 3 products spills)
  note_path(m3 ? "glf_single_herm_3m" : "glf_single_herm_4m");
  if constexpr (NC < 2)
    if (m3) return sgh_launch2<NC, true>(p, grid, coop, st);
  return sgh_launch2<NC, false>(p, grid, coop, st);
}

// obs[b][gs][m] = sum over the T^2 tiles of obs_part, fixed order
// (skipped when the launch reported a hand-off timeout: the guarded persistent re-run writes obs itself)
__global__ void glf_single_obs_kernel(const c128* part, int T2, long n, c128* obs, const int* stat) {
  if (__hip_atomic_load(stat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const c128* s = part + e * T2;
    c128 v = s[0];
    for (int q = 1; q < T2; ++q) v = cadd(v, s[q]);
    obs[e] = v;
  }
}

template <int KS, int NC, bool M3, bool SPLIT>
hipError_t sg_launch4(SingleParams p, int grid, bool coop, hipStream_t st) {
  if (!coop) {
    hipLaunchKernelGGL((glf_single_kernel<KS, NC, M3, SPLIT>), dim3(grid), dim3(SG_WG), 0, st, p);
    return hipGetLastError();
  }
  void* args[] = {(void*)&p};
  return hipLaunchCooperativeKernel((const void*)glf_single_kernel<KS, NC, M3, SPLIT>, dim3(grid), dim3(SG_WG), args,
                                    0, st);
}
template <int KS, int NC, bool M3>
hipError_t sg_launch3(SingleParams p, int grid, bool coop, hipStream_t st) {
  if constexpr (NC > 0)
    if (p.split) return sg_launch4<KS, NC, M3, true>(p, grid, coop, st);
  return sg_launch4<KS, NC, M3, false>(p, grid, coop, st);
}
// The 3-product complex MACs on a half-filled chip (<= 128 workgroups), the 4-product ones above: N = 128, one matrix
// 29.7k -> 34.9k steps/s and two 61.7k -> 69.4k with 3 products, four (256 workgroups) 117k -> 103k; N = 32, 64
// matrices 2.91M -> 2.61M (profiles/r04/lindblad/glf_single_bench.txt).
template <int KS, int NC>
hipError_t sg_launch(SingleParams p, int grid, bool coop, hipStream_t st) {
  const bool m3 = grid <= 128 && NC < 2;   // (NC = 2 with 3 products spills)
  note_path(m3 ? "glf_single_3m" : "glf_single_4m");
  if (m3) return sg_launch3<KS, NC, true>(p, grid, coop, st);
  return sg_launch3<KS, NC, false>(p, grid, coop, st);
}

}  // namespace

int glf_single_max_batch(int Np, int nc, int herm) {
  if (herm) return (Np == 128 && nc >= 1 && nc <= 2) ? 256 / (64 + 36) : 0;
  if (nc > 2 || (Np != 32 && Np != 64 && Np != 128)) return 0;
  const int T = Np / 16;
  return 256 / (T * T);
}

// One persistent launch for B matrices (B <= glf_single_max_batch), undriven GLF operators already padded.  Nothing
// waits on the host: *status_out is the device status word (1 after the launch if a hand-off spin expired -- the state
// is then invalid and the caller queues a guarded re-run behind it), or null when nothing was launched.  QD_EBUSY when
// the cooperative launch is refused (nothing ran).
int glf_single_run(const c128* P, const c128* Q, const c128* Lop, const c128* Rop, int nc, const c128* eT, int ne,
                   c128* rho, int B, int N, int Np, double dt, int nsteps, c128* obs, c128* snap, int save_every,
                   const int** status_out, hipStream_t st, int herm) {
  *status_out = nullptr;
  if (nsteps <= 0 && ne == 0) return QD_OK;
  const int T = Np / 16, T2 = T * T;
  const size_t NN = (size_t)Np * Np;
  const size_t flag_bytes = 16;   // *status, padded
  const size_t obs_elems = ne ? (size_t)B * (nsteps + 1) * ne * T2 : 0;
  const size_t elems = 2 * (size_t)B * NN + 2 * (size_t)(nc > 0 ? nc + 1 : 0) * B * NN + obs_elems;
  void* w = nullptr;
  int rc = workspace(WS_LINDBLAD, elems * sizeof(c128) + flag_bytes, &w, st);
  if (rc) return rc;
  SingleParams p;
  p.P = P;
  p.Q = Q;
  p.Lop = Lop;
  p.Rop = Rop;
  p.eT = eT;
  p.rho = rho;
  p.rbuf = (c128*)w;
  p.ybuf = p.rbuf + 2 * (size_t)B * NN;
  p.obs_part = ne ? p.ybuf + 2 * (size_t)(nc > 0 ? nc + 1 : 0) * B * NN : nullptr;
  p.status = (int*)((c128*)w + elems);
  p.N = N;
  p.ne = ne;
  p.nsteps = nsteps;
  p.step0 = 0;
  p.total_steps = nsteps;
  p.save_every = save_every;
  p.nsave = save_every > 0 ? nsteps / save_every : 0;
  p.snap = p.nsave > 0 ? snap : nullptr;
  p.dt = dt;
  p.B = B;
  // every handed-off buffer preset to the parity its first epoch does not have: r_1 (buffer 1) and r_2 (buffer 0)
  // carry parities 0 and 1, Y_0 and Y_1 (buffers 0 and 1) both 0; bytes of 0x01 make every double's lowest bit 1
  QD_TRY(fill_bytes(p.status, 0, flag_bytes, st));
  QD_TRY(fill_bytes(p.rbuf, 0, (size_t)B * NN * sizeof(c128), st));
  QD_TRY(fill_bytes(p.rbuf + (size_t)B * NN, 1, (size_t)B * NN * sizeof(c128), st));
  if (nc > 0) QD_TRY(fill_bytes(p.ybuf, 1, 2 * (size_t)(nc + 1) * B * NN * sizeof(c128), st));
  p.tim = nullptr;
#ifdef QD_PHASE_TIMING
  void* tw = nullptr;
  if ((rc = workspace(WS_MISC, (size_t)2 * B * T2 * 8 * sizeof(unsigned long long), &tw, st))) return rc;
  QD_TRY(fill_bytes(tw, 0, (size_t)2 * B * T2 * 8 * sizeof(unsigned long long), st));
  p.tim = (unsigned long long*)tw;
#endif
  const bool coop = option(QD_OPT_COOP_LAUNCH) != 0;
  if (herm) {   // Hermitian H and rho, N_p = 128, nc in {1, 2}: upper k tiles + Y workgroups (glf_single_herm_kernel)
    p.split = 1;
    int grid = 0;
    note_path("glf_single_herm");
    hipError_t e = nc == 1 ? sgh_launch<1>(p, B, coop, st, grid) : sgh_launch<2>(p, B, coop, st, grid);
    if (e == hipErrorCooperativeLaunchTooLarge) {
      (void)hipGetLastError();
      set_error("glf Hermitian single-trajectory launch: %d workgroups cannot be co-resident", grid);
      return QD_EBUSY;
    }
    QD_HIP(e);
    if (option(QD_OPT_FAKE_TIMEOUT)) QD_TRY(fill_bytes(p.status, 1, 1, st));
    *status_out = p.status;
#ifdef QD_PHASE_TIMING
    {   // per-phase wall clock (100 MHz ticks, thread 0), mean over each role's workgroups, per stage, in us
      std::vector<unsigned long long> hv((size_t)grid * 8);
      QD_HIP(hipMemcpy(hv.data(), p.tim, hv.size() * 8, hipMemcpyDeviceToHost));
      const char* nm[6] = {"wait_r", "y_publish", "-", "wait_y", "yr_reduce_pr", "update_publish"};
      const int nkw = B * T * (T + 1) / 2;
      for (int role = 0; role < 2; ++role) {
        const int q0 = role ? nkw : 0, q1 = role ? std::min(grid, nkw + B * T2) : nkw;
        fprintf(stderr, "[glf herm single phase timing] N=%d B=%d nsteps=%d %s workgroups, us per stage:", N, B, nsteps,
                role ? "Y" : "k");
        for (int k = 0; k < 6; ++k) {
          double sm = 0;
          for (int q = q0; q < q1; ++q) sm += (double)hv[(size_t)q * 8 + k];
          fprintf(stderr, " %s %.3f", nm[k], sm / (q1 - q0) / 100.0 / (4.0 * nsteps));
        }
        fprintf(stderr, "\n");
      }
    }
#endif
    if (ne) {
      const long n = (long)B * (nsteps + 1) * ne;
      hipLaunchKernelGGL(glf_single_obs_kernel, dim3((int)std::min<long>((n + 255) / 256, 1024)), dim3(256), 0, st,
                         (const c128*)p.obs_part, T2, n, obs, (const int*)p.status);
      QD_HIP(hipGetLastError());
    }
    return QD_OK;
  }
  // a second workgroup per tile for the Y_c tiles when the chip has room: the k workgroup's P r + r Q then runs
  // while the Y_c tiles are computed and handed over, instead of after its own Y_c tile
  p.split = nc > 0 && 2 * B * T2 <= 256;
  note_path(p.split ? "glf_single_split" : "glf_single_joint");
  const int grid = (p.split ? 2 : 1) * B * T2;
  hipError_t e = hipErrorInvalidValue;
#define SG_CASE(KS_)                                                    \
  switch (nc) {                                                         \
    case 0: e = sg_launch<KS_, 0>(p, grid, coop, st); break;            \
    case 1: e = sg_launch<KS_, 1>(p, grid, coop, st); break;            \
    default: e = sg_launch<KS_, 2>(p, grid, coop, st); break;           \
  }
  switch (Np) {
    case 32: SG_CASE(1) break;
    case 64: SG_CASE(2) break;
    default: SG_CASE(4) break;
  }
#undef SG_CASE
  if (e == hipErrorCooperativeLaunchTooLarge) {
    (void)hipGetLastError();
    set_error("glf single-trajectory launch: %d workgroups cannot be co-resident", grid);
    return QD_EBUSY;
  }
  QD_HIP(e);
  if (option(QD_OPT_FAKE_TIMEOUT))   // tests: report a hand-off timeout after the run
    QD_TRY(fill_bytes(p.status, 1, 1, st));
  *status_out = p.status;
#ifdef QD_PHASE_TIMING
  {   // per-phase wall clock (100 MHz ticks, workgroup thread 0), mean over workgroups, per stage, in us
    std::vector<unsigned long long> hv((size_t)grid * 8);
    QD_HIP(hipMemcpy(hv.data(), p.tim, hv.size() * 8, hipMemcpyDeviceToHost));
    const char* nm[6] = {"wait_r", "y_publish", "pr_rq_mfma", "wait_y", "y_mfma_reduce", "update_publish"};
    for (int role = 0; role < (p.split ? 2 : 1); ++role) {
      fprintf(stderr, "[glf single phase timing] N=%d B=%d nsteps=%d %s workgroups, us per stage:", N, B, nsteps,
              role ? "Y" : (p.split ? "k" : "joint"));
      for (int k = 0; k < 6; ++k) {
        double sm = 0;
        for (int q = 0; q < B * T2; ++q) sm += (double)hv[((size_t)role * B * T2 + q) * 8 + k];
        fprintf(stderr, " %s %.3f", nm[k], sm / (B * T2) / 100.0 / (4.0 * nsteps));
      }
      fprintf(stderr, "\n");
    }
  }
#endif
  if (ne) {
    const long n = (long)B * (nsteps + 1) * ne;
    hipLaunchKernelGGL(glf_single_obs_kernel, dim3((int)std::min<long>((n + 255) / 256, 1024)), dim3(256), 0, st,
                       (const c128*)p.obs_part, T2, n, obs, (const int*)p.status);
    QD_HIP(hipGetLastError());
  }
  return QD_OK;
}

}  // namespace qd
