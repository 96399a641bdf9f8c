/*
 * qdyn.h — C-ABI of libqdyn.so, the MI355X (gfx950) propagator library that
 * sits under pyqed_amd's drop-in solver classes.
 *
 * Boundary rules:
 *   - plain pointers + sizes only; every pointer argument is a DEVICE pointer
 *     unless stated otherwise; complex numbers are interleaved fp64 pairs
 *     (qd_c128, byte-identical to numpy/torch complex128);
 *   - matrices are row-major and contiguous; vec(rho) is row-major
 *     (rho.flatten(), reference pyqed/superoperator.py:125-150);
 *   - the caller owns every buffer it passes; the library's own scratch is
 *     call-scoped: slabs of a library arena, held by one live call at a time
 *     and ordered behind their previous user on the device (hipStreamWaitEvent),
 *     never by a host wait; qd_shutdown releases the arena;
 *   - calls are asynchronous on `stream` (a hipStream_t, NULL = default stream):
 *     they enqueue their kernels and return without waiting for the device.
 *     The one exception: qd_gather_rows with check != 0 (stated there).  The two
 *     persistent hand-off launches (the single-trajectory Lindblad launch inside
 *     qd_lindblad_rk4, qd_deom_rk4_banded without a status word) report a
 *     hand-off timeout in a device status word and queue a stream-ordered
 *     fallback behind themselves that re-runs the call only in that case;
 *     host-array inputs (fvals of the driven entry points) are copied before
 *     the call returns;
 *   - the hand-off launches pass data between workgroups with the flag carried
 *     in the data: every handed-off double carries its epoch's parity in the
 *     LOWEST bit of its low dword, and a consumer takes a 16-B granule whose
 *     doubles carry the expected parity.  This assumes a 16-B granule written by
 *     one store is never observed torn at dword level (new low dwords with stale
 *     high dwords) -- observed on MI355X, not an architectural guarantee
 *     (MI355X_MICROARCH.md); a torn granule would pass the parity test silently;
 *   - the asynchronous calls may be captured into a HIP graph (stream capture on
 *     `stream`): their scratch is then a device buffer owned by the graph being
 *     captured (a graph user object; freed by the library's next uncaptured call
 *     or qd_shutdown once the graph is destroyed), never an arena slab; host
 *     arrays (fvals) are copied at capture time, so every replay uses the values
 *     they held then; the synchronising exceptions above cannot be captured;
 *   - return 0 on success, a negative QD_E* code on failure; the message is
 *     available from qd_last_error() (thread-local).
 *
 * The reference (ShuoyiHU/pyqed) has no FFI: its "operator API" is the Python
 * class surface.  Each entry point below names the reference function whose
 * inner loop it replaces.
 */
#ifndef QDYN_H
#define QDYN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QD_OK 0
#define QD_EINVAL -1   /* bad argument (shape, null pointer, unsupported size) */
#define QD_EHIP -2     /* HIP runtime error                                    */
#define QD_ERCCL -3    /* RCCL error                                           */
#define QD_ENOMEM -4   /* workspace allocation failed                          */
#define QD_EBUSY -5    /* a persistent launch whose workgroups must all be resident at once was refused by
                          hipLaunchCooperativeKernel (qd_deom_rk4_banded): nothing ran, the inputs are untouched */

#define QD_COMM_ID_BYTES 128  /* size of the RCCL unique id qd_comm_unique_id writes */

typedef struct qd_c128 {
  double re;
  double im;
} qd_c128;

/* ------------------------------------------------------------ runtime ---- */
int qd_version(void);                 /* e.g. 100 = 0.1.0                      */
const char* qd_last_error(void);      /* thread-local message of last failure */
int qd_init(int device);              /* hipSetDevice + warm-up               */
int qd_device_count(int* count);      /* host pointer                         */
int qd_shutdown(void);                /* waits for and frees the scratch arena */
int qd_synchronize(void* stream);     /* hipStreamSynchronize                 */
/* Scratch arena (current process, all devices): bytes reserved and bytes in use
 * (host pointers).  In use returns to 0 once every stream that called the library
 * has drained; reserved is bounded by the peak concurrent scratch plus a capped
 * idle cache, not by the number of streams. */
int qd_workspace_stats(size_t* reserved, size_t* used);

/* Process options: the library's only run-time switches.  Each is read once from
 * the environment variable named below when the library loads; qd_set_option
 * changes it for the whole process (thread-safe).  Dispatch is otherwise a
 * function of the problem's shape alone.
 *   QD_OPT_COOP_LAUNCH  (QD_COOP_LAUNCH, default 1): 0 launches the persistent
 *       hand-off kernels (qd_deom_rk4_banded, the single-trajectory Lindblad
 *       launch) with a plain launch instead of hipLaunchCooperativeKernel (same
 *       kernels and residency; rocprofv3 faults at exit after cooperative launches);
 *   QD_OPT_FAKE_TIMEOUT (QD_TEST_FAKE_TIMEOUT, default 0): tests only; 1 makes
 *       those two launches report a hand-off timeout after a real run, to exercise
 *       the callers' recovery;
 *   QD_OPT_GLF_PATH     (QD_GLF_PATH, default QD_GLF_AUTO): the Lindblad / GLF
 *       batch path -- QD_GLF_SINGLE (single-trajectory launch, where it applies),
 *       QD_GLF_SPLIT (a workgroup per output block and phase; pair blocks for
 *       Hermitian batches), QD_GLF_PERSISTENT (a workgroup per matrix); for
 *       comparing the paths on one input;
 *   QD_OPT_IDLE_CAP_MIB (no environment variable, default -1 = 16384): the
 *       scratch arena's idle cache in MiB -- idle slabs beyond it are released once
 *       their last user has completed (tests lower it to exercise the release).
 * qd_take_path copies the dispatch decisions of this thread's calls since the
 * last qd_take_path (space-separated kernel-path names) into buf and clears them. */
#define QD_OPT_COOP_LAUNCH 0
#define QD_OPT_FAKE_TIMEOUT 1
#define QD_OPT_GLF_PATH 2
#define QD_OPT_IDLE_CAP_MIB 3
#define QD_OPT_COUNT 4
#define QD_GLF_AUTO 0
#define QD_GLF_SINGLE 1
#define QD_GLF_SPLIT 2
#define QD_GLF_PERSISTENT 3
int qd_set_option(int opt, int value);
int qd_get_option(int opt, int* value);      /* value: host pointer */
int qd_take_path(char* buf, size_t len);     /* buf: host pointer   */

/* ------------------------------------------------------------ Lindblad --- */
/*
 * Batched RK4 propagation of the Lindblad master equation
 *     d rho/dt = -i[H, rho] + sum_c ( c rho c^+ - 1/2 {c^+ c, rho} )
 * for B independent density matrices that share H and the collapse ops.
 *
 * Replaces the time loop of pyqed/oqs.py:1682-1690 (_lindblad) with the RHS
 * oqs.liouvillian/lindbladian (oqs.py:697-714) and phys.rk4 (phys.py:1051-1064).
 *
 *   H     [N][N]          Hamiltonian
 *   C     [nc][N][N]      collapse operators (may be NULL when nc == 0)
 *   rho   [B][N][N]       in: rho(t0), out: rho(t0 + nsteps*dt)
 *   E     [ne][N][N]      observables (NULL when ne == 0)
 *   obs   [B][nsteps+1][ne]  Tr(E_m rho_k), k = 0..nsteps (row 0 = t0, as
 *                         oqs.py:1680), NULL when ne == 0
 *   snap  [B][nsteps/save_every][N][N]  rho after steps save_every, 2*save_every, ...
 *                         (NULL or save_every <= 0: no snapshots)
 * Constraints: 1 <= N <= 16384, 0 <= nc <= 256, ne >= 0, B >= 1.  RK4 is evaluated
 * in Horner form (phys.rk4 in exact arithmetic; no accumulator buffer).
 * Few undriven matrices (B <= 256 / (N_p/16)^2, N_p in {32, 64, 128}, nc <= 2) run
 * as ONE cooperative persistent launch with a workgroup per 16 x 16 output tile
 * and in-launch hand-offs (data-as-flag, above); behind it the call queues a
 * guarded restore of the initial state and a guarded run of the persistent
 * kernel (a workgroup per matrix), both no-ops unless the launch reported a
 * hand-off timeout: the call never waits on the host.  A refused cooperative
 * launch (known at once) runs the split path instead.
 */
int qd_lindblad_rk4(const qd_c128* H, const qd_c128* C, int nc, qd_c128* rho,
                    int B, int N, double dt, int nsteps, const qd_c128* E,
                    int ne, qd_c128* obs, qd_c128* snap, int save_every,
                    void* stream);

/*
 * Same as qd_lindblad_rk4 for density matrices that are EXACTLY Hermitian
 * (rho == rho^+ bit for bit; the caller checks).  Uses L[rho] = X + X^+ with
 * X = -iK rho + 1/2 sum_c (C_c rho) C_c^+ : 1 + 2 nc complex GEMMs per RHS
 * instead of 2 + 2 nc, and keeps every RK4 stage exactly Hermitian.  N <= 128
 * (larger N falls back to the general path inside the library).
 */
int qd_lindblad_rk4_herm(const qd_c128* H, const qd_c128* C, int nc,
                         qd_c128* rho, int B, int N, double dt, int nsteps,
                         const qd_c128* E, int ne, qd_c128* obs, qd_c128* snap,
                         int save_every, void* stream);

/*
 * Driven Lindblad RK4 (pyqed/oqs.py:1699-1806 _lindblad_driven):
 *   H(t_k) = H0 - sum_d f_d(t_k) Hd_d, constant within step k, t_k = t0 + (k+1) dt
 * fvals is a HOST array [nsteps][nd] of the drive values (complex).  Other
 * arguments as qd_lindblad_rk4 (obs row 0 = t0).  1 <= nd <= 16.
 */
int qd_lindblad_driven_rk4(const qd_c128* H0, const qd_c128* Hd, int nd,
                           const qd_c128* fvals, const qd_c128* C, int nc,
                           qd_c128* rho, int B, int N, double dt, int nsteps,
                           const qd_c128* E, int ne, qd_c128* obs, qd_c128* snap,
                           int save_every, void* stream);

/*
 * Batched RK4 for any equation of motion of "generalised Lindblad form"
 *     d rho/dt = P rho + rho Q + sum_c L_c rho R_c        (c < npairs)
 * P, Q [N][N]; L, R [npairs][N][N]; other arguments as qd_lindblad_rk4.
 * Used for Redfield dynamics in the H eigenbasis: replaces the csr R.vec(rho)
 * RK4 loop of pyqed/oqs.py:436-459 (_redfield) + rhs (oqs.py:462-463); the
 * pyqed_amd host builds P, Q, L_c, R_c from redfield_tensor's ingredients
 * (oqs.py:519-570).  Constraints: 0 <= npairs <= 256.
 */
int qd_glf_rk4(const qd_c128* P, const qd_c128* Q, const qd_c128* L,
               const qd_c128* R, int npairs, qd_c128* rho, int B, int N,
               double dt, int nsteps, const qd_c128* E, int ne, qd_c128* obs,
               qd_c128* snap, int save_every, void* stream);

/*
 * Hermitian-state GLF (RedfieldSolver.evolve's R vec(rho) in the eigenbasis, oqs.py:364-463, and any
 * generator with Q = P^+ and pairs closed under conjugate transposition):
 *   d rho/dt = X + X^+,   X = P rho + sum_c L_c rho W_c,
 * valid for exactly Hermitian rho (every stage stays exactly Hermitian).  Redfield: P = -iE - sum A_k Lam_k,
 * L_k = A_k, W_k = Lam_k^+.  1 + 2 npairs complex GEMMs per RHS (qd_glf_rk4: 2 + 2 * 2 npairs).  N <= 128.
 */
int qd_glf_rk4_herm(const qd_c128* P, const qd_c128* L, const qd_c128* W, int npairs,
                    qd_c128* rho, int B, int N, double dt, int nsteps, const qd_c128* E,
                    int ne, qd_c128* obs, qd_c128* snap, int save_every, void* stream);

/*
 * Batched basis transform of B matrices [B][N][N] in place:
 *   mode 0: A <- V^+ A V   (pyqed/phys.py:1121-1137 transform(A, V))
 *   mode 1: A <- V A V^+   (transform(A, dag(V)), back-transform in oqs.py:450)
 */
int qd_basis_transform(const qd_c128* V, qd_c128* A, int B, int N, int mode,
                       void* stream);

/*
 * Batched two-sided product A[b] <- L A[b] R (in place), [B][N][N].  Builds the
 * quantum-regression initial states C rho(t) A of oqs.py:1291-1292 and
 * oqs.py:1240 (correlation_3op_1t/_2t) for a whole batch of restarts.
 */
int qd_sandwich(const qd_c128* L, const qd_c128* R, qd_c128* A, int B, int N,
                void* stream);

/* ------------------------------------------------------------ split-operator */
/*
 * 2D multi-state split-operator propagation, nsteps Strang steps
 *     psi <- V/2 . IFFT2( exp_K * FFT2( V/2 . psi ) )
 * exactly as pyqed/wpd.py:723-732 (SPO2.run, return_states=True, linear KEO
 * _KEO_linear wpd.py:837-848).  psi [nx][ny][ns] in/out (state index fastest),
 * expVh [nx][ny][ns][ns] = U e^{-i w dt/2} U^+ per grid point, expK [nx][ny].
 * snap [nsteps/nout][nx][ny][ns]: psi after steps nout, 2*nout, ... (NULL: none).
 * nx, ny powers of two in [16, 1024]; 1 <= ns <= 8; ns*ny/4 and ns*nx/4 <= 256.
 */
int qd_spo2_run(qd_c128* psi, const qd_c128* expVh, const qd_c128* expK, int nx,
                int ny, int ns, int nsteps, int nout, qd_c128* snap,
                void* stream);

/*
 * qd_spo2_run for B independent wavefunctions on one potential: psi [B][nx][ny][ns], snap
 * [B][nsteps/nout][nx][ny][ns] (or NULL); one launch per pass for the whole batch on the
 * 256 x 256 register-FFT kernels (ns <= 2), member by member otherwise.
 */
int qd_spo2_run_batch(qd_c128* psi, int B, const qd_c128* expVh, const qd_c128* expK, int nx,
                      int ny, int ns, int nsteps, int nout, qd_c128* snap, void* stream);

/*
 * qd_spo2_run with the two other SPO2 step structures of pyqed/wpd.py:
 *   expKy != NULL: Jacobi KEO (_KEO_jacobi, wpd.py:850-887): FFT_y, * expKy[i][ky]
 *                  (row i's factor exp(-i ky^2/(2 I(x_i)) dt)), FFT_x, * expK, IFFT2;
 *                  expK is then exp_Kx[kx] broadcast over ky ([nx][ny]).
 *   expV != NULL:  merged potential (run(return_states=False), wpd.py:736-755 and
 *                  SPO2NH.run wpd.py:1054-1077): V/2, nsteps x [K, V] with a snapshot
 *                  after every nout steps (state after V), then K, V/2.
 * expVh / expV may be non-unitary (SPO2NH's U e^{-i w dt} U^-1 of a complex potential).
 */
int qd_spo2_run_ex(qd_c128* psi, const qd_c128* expVh, const qd_c128* expV,
                   const qd_c128* expK, const qd_c128* expKy, int nx, int ny,
                   int ns, int nsteps, int nout, qd_c128* snap, void* stream);

/*
 * Device build of the SPO point propagators (replaces the per-point eigh loop of
 * SPO2.build / SPO3.build, pyqed/wpd.py:585-623 and :1290-1330): for every grid point
 *   expV  = U e^{-i w dt} U^+,  expVh = U e^{-i w dt/2} U^+,  (w, U) = eigh(V_point)
 * with LAPACK's conventions (lower triangle, real diagonal).  v is [npts][ns][ns] float64
 * (v_complex = 0) or complex128 (v_complex = 1); ns in [1, 1024] (ns <= 2 closed form,
 * ns > 2 the scaling-and-squaring exponential of qd_spo_expm); expV may be null.
 */
int qd_spo_expv(const void* v, int v_complex, long npts, int ns, double dt,
                qd_c128* expV, qd_c128* expVh, void* stream);

/*
 * exp(-i V dt/2) and exp(-i V dt) per grid point for any ns in [1, 1024], V complex
 * [npts][ns][ns]: hermitian = 1 reads the Hermitian matrix eigh sees (SPO2 / SPO3
 * build, wpd.py:585-623, 1290-1330), hermitian = 0 the full matrix (SPO2NH.build,
 * wpd.py:960-985, eig -> U_R e^{-iw dt} U_R^-1).  Scaling and squaring of a degree-18
 * Taylor polynomial (no eigenvectors); expV = expVh^2; expV may be null.  The four
 * ns x ns work matrices sit in LDS up to ns = 50 and in the library's scratch above.
 */
int qd_spo_expm(const qd_c128* v, int hermitian, long npts, int ns, double dt,
                qd_c128* expV, qd_c128* expVh, void* stream);

/*
 * 1D single-surface split-operator with the step structure of pyqed/wpd.py:225-273
 * (SPO.run): V/2 ; (nt//nout - 1)*nout x [K, V] (snapshot after each block) ; K, V/2.
 * psi [B][nx] in/out (B independent wavepackets, one workgroup each, all steps in
 * LDS), expV/expVh/expK [nx]; snap [B][nt//nout - 1][nx] or NULL.
 */
int qd_spo1d_run(qd_c128* psi, const qd_c128* expV, const qd_c128* expVh,
                 const qd_c128* expK, int nx, int B, int nt, int nout,
                 qd_c128* snap, void* stream);

/* ------------------------------------------------------------ DEOM / HEOM -- */
/*
 * RK4 propagation of B independent DEOM hierarchies (dissipaton equation of
 * motion) sharing one bath, one H and the same coupling operators.
 * Replaces DEOMSolver.run (pyqed/heom/deom.py:1072-1114) -> rk4 (:725-766) ->
 * rem_cal / generate_dot_element (:641-673) with generate_time (:676-688).
 *   ados   [B][nmax][ns][ns]  ADOs, in/out (ADO 0 = system density matrix)
 *   minus, plus [nmax][K]     int32 neighbour tables: index of key -/+ e_k, -1 if absent
 *   coef   [nmax][K][3]       cL, cR, cP prefactors (see deom.hip)
 *   damp   [nmax]             -sum_k key_k expn_k
 *   mode   [K]                int32 coupling-operator index of each dissipaton
 *   H, Hdip [ns][ns]; Q, Qdip [nmod][ns][ns]  (Hdip / Qdip may be NULL)
 *   fsys, fcoup  HOST arrays [nsteps][3]: pulse values at t, t+dt/2, t+dt of
 *                each step (NULL when the dipole is NULL)
 *   rho_sys [B][nsteps+1][ns][ns]  ADO 0 after every step (row 0 = initial), or NULL
 *   E [ne][ns][ns], trace [B][nsteps+1][ne]  Tr(E_m rho_0) per step (p1 of
 *                deom.py:1100,1113; e_ops of HEOM/heom.py:339-343), or NULL
 * Also runs the single-exponential HEOM chain of pyqed/HEOM/heom.py:275-347
 * (_heom, RK4) with chain tables (K = 1) built by the host.
 * Any ns and nmod: lane-group kernel (ns^2 <= 64, K <= 8), MFMA 16 x 16 tiles
 * (9 <= ns <= 16, <= 2 modes), tiled GEMM-form kernels otherwise.  Undriven runs
 * use Horner-form RK4 stages (no accumulator), driven ones the classic form.
 */
int qd_deom_rk4(qd_c128* ados, int B, int nmax, int K, int ns,
                const int32_t* minus, const int32_t* plus, const qd_c128* coef,
                const qd_c128* damp, const int32_t* mode, int nmod,
                const qd_c128* H, const qd_c128* Hdip, const qd_c128* Q,
                const qd_c128* Qdip, const qd_c128* fsys, const qd_c128* fcoup,
                double dt, int nsteps, qd_c128* rho_sys, const qd_c128* E,
                int ne, qd_c128* trace, void* stream);

/*
 * qd_deom_rk4 for batches of hierarchies stored ADO-major: ados [nmax][B][ns][ns] (hierarchy index
 * fastest).  A wavefront then holds one ADO of 64 / 2^ceil(log2 ns^2) hierarchies: its index and
 * prefactor loads are one request per wave and every neighbour read is one contiguous run.  Same
 * arguments and results as qd_deom_rk4 otherwise (rho_sys / trace stay [B][nsteps+1]...).
 * ns^2 <= 64, K <= 8.
 */
int qd_deom_rk4_ado_major(qd_c128* ados, int B, int nmax, int K, int ns,
                          const int32_t* minus, const int32_t* plus, const qd_c128* coef,
                          const qd_c128* damp, const int32_t* mode, int nmod,
                          const qd_c128* H, const qd_c128* Hdip, const qd_c128* Q,
                          const qd_c128* Qdip, const qd_c128* fsys, const qd_c128* fcoup,
                          double dt, int nsteps, qd_c128* rho_sys, const qd_c128* E,
                          int ne, qd_c128* trace, void* stream);

/*
 * ONE hierarchy (B = 1) of qd_deom_rk4 as one persistent launch over `nbands`
 * tier bands (DEOMSolver.run, pyqed/heom/deom.py:1072-1114, with rk4 /
 * rem_cal :641-766).  Workgroup w owns ADO rows [band_lo[w], band_lo[w+1]) and
 * keeps their stage input plus its halo rows in LDS; the bands hand each RK4
 * stage's rows to each other inside the launch (write-through stores whose
 * doubles carry the stage's parity in their lowest mantissa bit: the data is
 * the flag).  Band tables (device int32, deom_shard.make_plans):
 * halo_off[nbands+1] / halo_idx (global halo rows per band), src_off[nbands+1]
 * / src (bands owning them), lminus / lplus [nmax][K] local rows (owned rows
 * first, then the band's halo rows; -1 absent); max_own / max_loc the largest
 * owned / owned + halo row counts.  ns in [2, 4], K <= 8,
 * max_own * (ns == 2 ? 4 : 16) <= 1024, (2 + nmod + max_loc) ns^2 16 B <= 160 KB.
 * Other arguments and results as qd_deom_rk4 with B = 1 (bit-identical with
 * one band; with several a halo value differs by at most one unit in its last
 * place, which reaches the result through dt x stencil: within 1e-13).
 * status: device int32 set to 1 if a hand-off timed out (bands not
 * co-resident; results invalid, ados overwritten: the caller re-runs), or null:
 * the call then saves the initial ADOs and queues a stream-ordered fallback that,
 * only after a timeout, restores them and re-runs the propagation on one
 * workgroup (the stage launches' element stencil; slow but correct) -- either
 * way the call returns without waiting for the device.  The launch is
 * cooperative: a band count the device cannot hold at once returns QD_EBUSY
 * before anything runs.  Undriven runs always use the Horner form of RK4 (the
 * QD_DEOM_HORNER=0 A/B switch of qd_deom_rk4 does not apply here; DEOMSolver
 * routes such runs to the stage launches).
 */
int qd_deom_rk4_banded(qd_c128* ados, int nmax, int K, int ns,
                       const int32_t* lminus, const int32_t* lplus,
                       const int32_t* band_lo, const int32_t* halo_off,
                       const int32_t* halo_idx, const int32_t* src_off,
                       const int32_t* src, int nbands, int max_own, int max_loc,
                       const qd_c128* coef, const qd_c128* damp, const int32_t* mode,
                       int nmod, const qd_c128* H, const qd_c128* Hdip,
                       const qd_c128* Q, const qd_c128* Qdip, const qd_c128* fsys,
                       const qd_c128* fcoup, double dt, int nsteps, qd_c128* rho_sys,
                       const qd_c128* E, int ne, qd_c128* trace, int32_t* status,
                       void* stream);

/*
 * One RK4 stage of a BAND of the ADO hierarchy (tier-banded sharding of one
 * hierarchy over ranks; DEOMSolver.run / rk4 / rem_cal,
 * pyqed/heom/deom.py:641-766, 1072-1114, split across processes).  Rows
 * [0, n_own) of rho / xin / xout are the band's ADOs, rows [n_own, n_loc) of xin
 * the halo copies of neighbours owned by other bands; minus / plus [n_own][K]
 * are LOCAL row indices (-1 absent); coef [n_own][K][3], damp [n_own] the band's
 * slices of qd_deom_rk4's tables.  stage 0..3 (RK4 order of deom.py:725-766;
 * stage 0 reads xin = rho); fs / fc the pulse values at the stage's time.  snap
 * [nsteps+1][ns][ns] (band owning ADO 0 only, else NULL) gets rho_0 after step
 * `step` at stage 3.  Any ns (group kernel ns <= 8, MFMA tiles above).
 * acc [n_own][ns][ns]: the classic RK4 accumulator (required when Hdip / Qdip
 * drive the stage); acc = NULL selects the accumulator-free Horner form that
 * qd_deom_rk4 runs for undriven hierarchies (stage s writes rho + dt/(4-s) L x;
 * identical to RK4 for a generator constant over the step).
 */
int qd_deom_stage(qd_c128* rho, const qd_c128* xin, qd_c128* xout, qd_c128* acc,
                  int n_own, int K, int ns, const int32_t* minus,
                  const int32_t* plus, const qd_c128* coef, const qd_c128* damp,
                  const int32_t* mode, int nmod, const qd_c128* H,
                  const qd_c128* Hdip, const qd_c128* Q, const qd_c128* Qdip,
                  double fs_re, double fs_im, double fc_re, double fc_im,
                  int stage, double dt, qd_c128* snap, int step, int nsteps,
                  void* stream);

/*
 * Arnoldi steps of the same Krylov form (classical Gram-Schmidt, applied twice):
 * qd_cgs_project: h[r] = sum_i conj(V[r][i]) w[i] for the m basis rows of V (row-major,
 * leading dimension ldv), fixed-order reductions; hsum (or NULL) accumulates h with stride ldh
 * (a Hessenberg column).  qd_cgs_normalize: *hsub = ||w||, v = w / max(||w||, 1e-300).
 */
int qd_cgs_project(const qd_c128* V, long ldv, int m, int n, const qd_c128* w, qd_c128* h,
                   qd_c128* hsum, long ldh, void* stream);
int qd_cgs_normalize(const qd_c128* w, int n, qd_c128* v, qd_c128* hsub, void* stream);

/*
 * One step of the delayed CGS2 Arnoldi process (two passes over the basis instead of four).
 * Entering step j: V[0..j-1] final, V[j] = u_j (the candidate after one projection), z = P u_j,
 * H (row-major, leading dimension ldh >= j + 1, at least j + 2 rows) with columns 0..j-2 final and
 * column j-1 holding u_j's projection coefficients.  On return V[j] = v_j, column j-1 final
 * (re-orthogonalisation added, h_{j,j-1} = |u_j - V_j s|), column j the projection coefficients
 * of P v_j and V[j+1] = u_{j+1}.  Start with V[0] = b at j = 0.  An exact breakdown writes
 * h_{j,j-1} = 0 and zero vectors from there on.  st: 16(j+1) and cs: 2(j+2) complex scratch;
 * j <= 8192.
 */
int qd_arnoldi_dcgs2_step(qd_c128* V, long ldv, int j, int n, const qd_c128* z, qd_c128* H,
                          long ldh, qd_c128* st, qd_c128* cs, void* stream);

/*
 * The shifted Hessenberg solves of the multi-shift Krylov form of
 * DEOMSolver.correlation_4op_3t (pyqed_amd/deom_krylov.py; the reference diagonalises P
 * instead, pyqed/heom/deom.py:1127-1209): for each of the S shifts s, (-H_k - s I) y = beta e_1
 * with H_k the leading k x k block of the upper Hessenberg Arnoldi matrix H (row-major, leading
 * dimension ldh, k + 1 rows: row k holds h_{k+1,k}).  Y [S][k] (or NULL) receives the
 * solutions, res [S] (or NULL) the FOM residuals |h_{k+1,k} y_{k-1}| / beta.  Gaussian
 * elimination with adjacent-row pivoting, one workgroup per shift; k <= 4096.
 */
int qd_shifted_hessenberg_solve(const qd_c128* H, int ldh, int k, const qd_c128* shifts, int S,
                                double beta, qd_c128* Y, double* res, void* stream);

/*
 * y = x0 + alpha P x (x0 NULL: y = alpha P x) for B ADO vectors, P the DEOM generator that DEOMSolver.run steps and
 * DEOMSolver.correlation_4op_3t diagonalises (generate_dot_element, pyqed/heom/deom.py:641-664;
 * generate_propgator :769-893 as a dense matrix).  x, y: [B][nmax][ns][ns] (element-major) or
 * [nmax][B][ns][ns] (ado_major = 1, needs ns^2 <= 64 and K <= 8), x0 in the same layout; y
 * aliases neither x nor x0.
 * Tables as qd_deom_rk4.  The transposed generator P^T is the same operator on transposed
 * tables (H^T, Q^T, minus <-> plus, prefactors moved to the other end of each link;
 * pyqed_amd/deom_krylov.py), which the Krylov form of correlation_4op_3t applies.
 */
int qd_deom_apply(const qd_c128* x, qd_c128* y, const qd_c128* x0, int B, int nmax, int K, int ns,
                  const int32_t* minus, const int32_t* plus, const qd_c128* coef,
                  const qd_c128* damp, const int32_t* mode, int nmod, const qd_c128* H,
                  const qd_c128* Q, double alpha, int ado_major, void* stream);

/* dst[i][:] = src[idx[i]][:], i < n, rows of row_elems complex (halo packing);
 * src holds nsrc rows.  An index outside [0, nsrc) is not read: its row is
 * written as NaN, and with check != 0 the call synchronises the stream and
 * returns QD_EINVAL. */
int qd_gather_rows(const qd_c128* src, int nsrc, const int32_t* idx, int n,
                   int row_elems, qd_c128* dst, int check, void* stream);

/* obs[s][m] = Tr(E_m rho_0(s)), s < nsnap: DEOMSolver.run's Tr(p1 rho_0)
 * (heom/deom.py:1100,1113) from a snapshot stack [nsnap][ns][ns]. */
int qd_deom_trace(const qd_c128* snap, const qd_c128* E, int ne, int nsnap,
                  int ns, qd_c128* obs, void* stream);

/*
 * Single-exponential (high-T Drude) HEOM chain of pyqed/oqs.py:1808-1875
 * (oqs._heom): explicit in-place sweep per step, ADO n updated from the NEW
 * n-1 and the old n, n+1; ADO nado-1 never updated.  ados [B][nado][ns][ns]
 * in/out; D0 = D0_re + i D0_im; rho_sys [B][nsteps+1][ns][ns] or NULL;
 * obs [B][nsteps+1][ne] = Tr(E_m ado_0) or NULL.  ns <= 16, nado >= 2.
 */
int qd_heom_chain_euler(qd_c128* ados, int B, int nado, int ns, const qd_c128* H,
                        const qd_c128* Q, double gamma, double D0_re,
                        double D0_im, double dt, int nsteps, qd_c128* rho_sys,
                        const qd_c128* E, int ne, qd_c128* obs, void* stream);

/* ------------------------------------------------------------ TDSE ------- */
/*
 * Batched RK4 for dpsi/dt = -i H psi (pyqed/mol.py:1603-1691 _quantum_dynamics,
 * reached from SESolver.run mol.py:1392 / Mol.run mol.py:628; tdse phys.py:1322).
 *   psi  [B][N] in/out; nsteps RK4 steps
 *   snap [B][nsteps/save_every][N]  psi after steps save_every, 2 save_every, ... or NULL
 *   E [ne][N][N], obs [B][nsteps/save_every + 1][ne] = <psi|E_m|psi> at t0 and at
 *   every snapshot (phys.obs, phys.py:1266-1283), or NULL.   Any N.
 */
int qd_tdse_rk4(const qd_c128* H, qd_c128* psi, int B, int N, double dt,
                int nsteps, int save_every, qd_c128* snap, const qd_c128* E,
                int ne, qd_c128* obs, void* stream);

/*
 * Laser-driven TDSE (pyqed/mol.py:1862-1958 driven_dynamics, reached from
 * Mol.run / SESolver.run with a pulse, mol.py:660-675 / 1430-1456):
 *   H_k = H0 - sum_d f_d(t_k) Hd_d,  t_k = t0 + k nout dt,
 * constant over block k of nout RK4 steps (calcH is evaluated with the block's
 * start time).  fvals is a HOST array [nblocks][nd] (f_d(t_k), complex).
 *   psi  [B][N] in/out; snap [B][nblocks][N] psi after each block, or NULL;
 *   E [ne][N][N], obs [B][nblocks+1][ne] = <psi|E_m|psi> at t0 and after
 *   each block, or NULL.   Any N, 0 <= nd <= 16, nout >= 1.
 */
int qd_tdse_driven_rk4(const qd_c128* H0, const qd_c128* Hd, int nd,
                       const qd_c128* fvals, qd_c128* psi, int B, int N,
                       double dt, int nblocks, int nout, qd_c128* snap,
                       const qd_c128* E, int ne, qd_c128* obs, void* stream);

/*
 * 3D multi-state split operator (pyqed/wpd.py:1349-1411 SPO3.run, linear KEO
 * _KEO_linear wpd.py:1419-1432 = fftn over axes (0,1,2)).  psi [nx][ny][nz][ns],
 * expVh [nx][ny][nz][ns][ns], expK [nx][ny][nz]; snap [nsteps/nout][...].
 * nx, ny, nz powers of two in [16, 256].
 */
int qd_spo3_run(qd_c128* psi, const qd_c128* expVh, const qd_c128* expK, int nx,
                int ny, int nz, int ns, int nsteps, int nout, qd_c128* snap,
                void* stream);

/*
 * qd_spo3_run with a separable kinetic propagator (linear coordinates, wpd.py:1255-1262:
 * exp_K = e_x (x) e_y (x) e_z): the kinetic step fftn, * exp_K, ifftn of _KEO_linear
 * (wpd.py:1418-1432) is applied as three per-axis mode products with the circulant axis
 * propagators M_a = F^-1 diag(e_a) F, given by their first columns m_a = ifft(e_a) [n_a]
 * (M_a[i][k] = m_a[(i - k) mod n_a]; out[i] = sum_k M_a[i][k] in[k] along axis a): 64^3 as
 * three passes on the 64-point register transforms (e_a = fft(m_a) formed on the device),
 * every other shape as mode products on the f64 MFMAs.  Same step structure, snapshots and
 * result as qd_spo3_run (to rounding).
 * n_a in [1, 64], ns in {1, 2}.
 */
int qd_spo3_run_axes(qd_c128* psi, const qd_c128* expVh, const qd_c128* mx,
                     const qd_c128* my, const qd_c128* mz, int nx, int ny, int nz, int ns,
                     int nsteps, int nout, qd_c128* snap, void* stream);

/*
 * RK4 with a dense Liouville-space generator, d v/dt = L v (B vectors).
 * Replaces the csr GEMV loop of pyqed/oqs.py:436-463 (_redfield + rhs) for any
 * dense superoperator.  L [N2][N2], v [B][N2] in/out (row-major vec(rho)),
 * W [ne][N2]: obs[b][k][m] = sum_j W[m][j] v_k[b][j] for k = 0..nsteps
 * (W = vec(E^T) gives Tr(E rho)), snap [B][nsteps/save_every][N2] or NULL.
 * B < 48 (QD_SUPEROP_GEMM_MIN): HBM-bound GEMV, 16 N2^2 bytes per stage per group
 * of <= 8 vectors.  B >= 48: one complex-fp64 MFMA GEMM per stage (L read once
 * per stage for the whole batch) with a fused RK4 epilogue.
 */
int qd_superop_rk4(const qd_c128* L, qd_c128* v, int B, int N2, double dt,
                   int nsteps, const qd_c128* W, int ne, qd_c128* obs,
                   qd_c128* snap, int save_every, void* stream);

/*
 * Dense Liouville-space generator of d rho/dt = P rho + rho Q + sum_c L_c rho R_c
 * on row-major vec(rho): out[(a,b),(c,d)] = P[a][c] d_bd + d_ac Q[d][b]
 * + sum_c L_c[a][c] R_c[d][b]  ([N^2][N^2], the kron(A, I) / kron(I, A^T)
 * conventions of pyqed/superoperator.py:200-270).  Replaces the host kron
 * assembly of superoperator.liouvillian (superoperator.py:29-58) and of
 * redfield_tensor's R (oqs.py:563-570) for dense operators.
 */
int qd_superop_from_glf(const qd_c128* P, const qd_c128* Q, const qd_c128* Lops,
                        const qd_c128* Rops, int nc, int N, qd_c128* out,
                        void* stream);

/*
 * Dense Lindblad superoperator of oqs.liouvillian (oqs.py:697-714) /
 * superoperator.liouvillian (superoperator.py:29-58): H [N][N], C [nc][N][N],
 * out [N^2][N^2] (N = 128: 4 GiB).
 */
int qd_superop_lindblad(const qd_c128* H, const qd_c128* C, int nc, int N,
                        qd_c128* out, void* stream);

/* ------------------------------------------------------------ response --- */
/*
 * SOS Liouville-space propagator U[a][b][k] = sum_j U1[a][j] e^{lam_j t_k} U2[j][b]
 * (U2 = U1^-1; layout (nL, nL, nt) as RedfieldSolver.U).  Replaces the
 * contraction of pyqed/oqs.py:196-212 (propagator, method='SOS').
 */
int qd_sos_propagator(const qd_c128* U1, const qd_c128* U2, const qd_c128* lam,
                      int nL, const double* t, int nt, qd_c128* U,
                      void* stream);

/*
 * Full third-order response cube in eigen form
 *   out[i][j][k] = (-i)^3 sum_pqr alpha_p e^{lam_p t3_i} B[p][q] e^{lam_q t2_j}
 *                                  C[q][r] e^{lam_r t1_k} beta_r
 * (alpha = I^T a U1, B = U1^-1 b U1, C = U1^-1 c U1, beta = U1^-1 d vec(rho0)).
 * Replaces the tensordot chain of pyqed/oqs.py:327-357 (correlation_4op_3t);
 * out layout [n3][n2][n1] = the reference's corr[i, j, k].
 */
int qd_response_cube(const qd_c128* alpha, const qd_c128* B, const qd_c128* C,
                     const qd_c128* beta, const qd_c128* lam, int nL,
                     const double* t3, int n3, const double* t2, int n2,
                     const double* t1, int n1, qd_c128* out, void* stream);

/*
 * Disorder-ensemble 2D response at fixed t2 (2DES (t3, t1) grid):
 *   out[i][k] (+)= (-i)^3 sum_m sum_pq alpha[m][p] e^{lam[m][p] t3_i}
 *                                      Mt[m][p][q] beta[m][q] e^{lam[m][q] t1_k}
 * with Mt_m = B_m diag(e^{lam_m t2}) C_m.  For M = 1 this is the slice
 * correlation_4op_3t(...)[:, j, :] (oqs.py:268-357).
 * accumulate != 0 adds into out.  Shards over ranks by members; the
 * partial grids are summed with one RCCL reduce by the caller.
 */
int qd_response2d_ensemble(const qd_c128* alpha, const qd_c128* Mt,
                           const qd_c128* beta, const qd_c128* lam, int M,
                           int nL, const double* t3, int n3, const double* t1,
                           int n1, qd_c128* out, int accumulate, void* stream);

/*
 * qd_response2d_ensemble on uniform grids t3_i = t3_0 + i dt3, t1_k = t1_0 + k dt1 (the
 * 2DES case, e.g. 0.5*arange(256)): the exponentials come from two-level tables
 * (a few transcendentals per 16-64 outputs), relative error ~1e-14 against direct
 * exponentials.  nL <= 16, n1 <= 1024.
 */
int qd_response2d_ensemble_uniform(const qd_c128* alpha, const qd_c128* Mt,
                                   const qd_c128* beta, const qd_c128* lam, int M,
                                   int nL, double t3_0, double dt3, int n3,
                                   double t1_0, double dt1, int n1, qd_c128* out,
                                   int accumulate, void* stream);

/*
 * Rectangular form of qd_response2d_ensemble(_uniform), used after the host prunes index sets that are
 * structurally zero (selection rules: alpha[:, p] == 0 or beta[:, q] == 0 for every member, exactly):
 *   S[i][k] = (-i)^3 sum_m sum_{p < nx} sum_{q < nz} alpha[m][p] e^{lamx[m][p] t3_i}
 *                                      Mt[m][p][q] beta[m][q] e^{lamz[m][q] t1_k}
 * with alpha, lamx [M][nx], Mt [M][nx][nz], beta, lamz [M][nz].  GEMM K = M nx.  A null t3 / t1 means
 * the uniform grid t0 + j dt (exponential tables).  transpose_out != 0 writes out[k][i] = S[i][k]
 * (out is [n1][n3]): the host's swapped call, which puts the smaller index set on K.
 */
int qd_response2d_ensemble_rect(const qd_c128* alpha, const qd_c128* lamx, int nx,
                                const qd_c128* Mt, const qd_c128* beta, const qd_c128* lamz,
                                int nz, int M, const double* t3, double t3_0, double dt3,
                                int n3, const double* t1, double t1_0, double dt1, int n1,
                                int transpose_out, qd_c128* out, int accumulate,
                                void* stream);

/*
 * Waiting-time scan of the disorder-ensemble 2D response (uniform t3 / t1 grids, t2 a device array of
 * n2 waiting times):
 *   out[j][i][k] (+)= (-i)^3 sum_m sum_pq alpha[m][p] e^{lam[m][p] t3_i}
 *                       (B_m diag(e^{lam_m t2_j}) C_m)[p][q] beta[m][q] e^{lam[m][q] t1_k}
 * i.e. qd_response2d_ensemble_uniform for every t2_j with Mt_j = B diag(e^{lam t2_j}) C, where
 * B = U1^-1 b U1, C = U1^-1 c U1 [M][nL][nL].  Evaluated as S_j = P diag(E_j) Q with
 * P = X B (t3 side) and Q = C Y (t1 side) built once and E_j = e^{lam t2_j} applied to Q's rows while the
 * GEMM stages them: every waiting time shares P and Q, and all of them run in one split-K MFMA GEMM
 * (N = n2 * n1).  Per rank: one member shard; the caller sums the [n2][n3][n1] stack over ranks
 * (RCCL reduce).  nL <= 16, n1 <= 1024.
 */
int qd_response2d_t2scan(const qd_c128* alpha, const qd_c128* B, const qd_c128* C,
                         const qd_c128* beta, const qd_c128* lam, int M, int nL,
                         double t3_0, double dt3, int n3, const double* t2, int n2,
                         double t1_0, double dt1, int n1, qd_c128* out, int accumulate,
                         void* stream);

/* Padded operand sizes of the scan: P is [n3p][Kp], Q is [Kp][n1p] complex128. */
int qd_response2d_t2_dims(int M, int nL, int n3, int n1, int* n3p, int* n1p, int* Kp);

/* Build the scan operands P, Q into caller-owned device buffers (once per ensemble / grid). */
int qd_response2d_t2_operands(const qd_c128* alpha, const qd_c128* B, const qd_c128* C,
                              const qd_c128* beta, const qd_c128* lam, int M, int nL,
                              double t3_0, double dt3, int n3, double t1_0, double dt1,
                              int n1, qd_c128* P, qd_c128* Q, void* stream);

/*
 * Pruned scan operands: alpha, lamp [M][np] (t3 side), B [M][np][nr], lamr [M][nr] (the waiting-time
 * index r; E_j = e^{lamr t2_j}), C [M][nr][nq], beta, lamq [M][nq] (t1 side).  P is [n3p][Kp] and Q
 * [Kp][n1p] with Kp from qd_response2d_t2_dims(M, nr, ...); apply with (lamr, nr).
 */
int qd_response2d_t2_operands_rect(const qd_c128* alpha, const qd_c128* lamp, int np,
                                   const qd_c128* B, const qd_c128* lamr, int nr,
                                   const qd_c128* C, const qd_c128* beta, const qd_c128* lamq,
                                   int nq, int M, double t3_0, double dt3, int n3, double t1_0,
                                   double dt1, int n1, qd_c128* P, qd_c128* Q, void* stream);

/* out [n2][n3][n1] (+)= the scan for waiting times t2 (device array) from prepared P, Q. */
int qd_response2d_t2_apply(const qd_c128* P, const qd_c128* Q, const qd_c128* lam, int M,
                           int nL, int n3, int n1, const double* t2, int n2, qd_c128* out,
                           int accumulate, void* stream);

/*
 * Frequency-domain 2D signal of an eigen-decomposed generator (DEOMSolver.correlation_4op_3t,
 * pyqed/heom/deom.py:1127-1209, whose per-(w_x, w_y) trace this evaluates in closed form):
 *   out[i][j] = sum_pq a_p / (-lam_p - i wx_i) * M_pq * v_q / (-lam_q - i wy_j)
 * a, v, lam [n]; M [n][n] row-major; wx [nx], wy [ny] device float64; out [nx][ny].
 * Two split-K MFMA GEMMs (W = M Z, out = X W) on generated resolvent operands.
 */
int qd_resolvent_grid2d(const qd_c128* a, const qd_c128* M, const qd_c128* v,
                        const qd_c128* lam, int n, const double* wx, int nx,
                        const double* wy, int ny, qd_c128* out, void* stream);

/*
 * Frequency-domain pole sum out[i] = sum_n -coeff_n / (lam_n + i w_i)
 * (Lindblad_solver.correlation_2op_1w / 3op_1w, pyqed/superoperator.py:603-700).
 */
int qd_resolvent_sum(const qd_c128* coeff, const qd_c128* lam, int n,
                     const double* w, int nw, qd_c128* out, void* stream);

/*
 * Sum-over-states 2D photon-echo spectrum (GSB + SE + ESA) of pyqed/signal/sos.py:
 * photon_echo (:962-1052) -> _photon_echo (:845-879) -> GSB (:624), SE (:731),
 * ESA (:498).  E [N] eigenvalues (complex allowed), dip [N][N], gamma [N];
 * g/e/f index lists (int32); omega1 = -pump.  S [n3][n1]: row = probe
 * (omega3), column = pump (the reference's meshgrid layout; the reference
 * itself only works for n1 == n3).
 */
int qd_photon_echo(const qd_c128* E, const qd_c128* dip, const double* gamma,
                   int N, const int32_t* g_idx, int ng, const int32_t* e_idx,
                   int ne, const int32_t* f_idx, int nf, const double* pump,
                   int n1, const double* probe, int n3, double t2, qd_c128* S,
                   void* stream);

/* ------------------------------------------------------------ FFT -------- */
/*
 * In-place FFT (inverse != 0: unnormalised inverse) along the middle axis of a
 * contiguous array [outer][n][inner], fused with fftshift (shift != 0), a scale
 * and, when freq != NULL, the phase exp(-/+ i freq[k] x0) (forward/inverse).
 * Implements pyqed/fft.py fft (:11-68), ifft (:70-102) and fft2 (:104-126).
 * Powers of two in [16, 1024]: Stockham LDS FFT; other n <= 3200: direct DFT.
 */
int qd_fft_axis(qd_c128* data, int outer, int n, int inner, int inverse,
                int shift, double scale, const double* freq, double x0,
                void* stream);

/*
 * out[i][j] = weight * sum_{a,b} f[a][b] exp(-i (kx_i x_b + ky_j y_a)),
 * f [ny][nx]: pyqed/fft.py dft (ny = 1, y = 0) and dft2 (:128-160).
 */
int qd_dft2(const double* x, int nx, const double* y, int ny, const qd_c128* f,
            const double* kx, int nkx, const double* ky, int nky,
            double weight, qd_c128* out, void* stream);

/*
 * RCCL (one communicator per process, one process per GPU) for hosts without torch.distributed:
 * rank 0 calls qd_comm_unique_id and ships the QD_COMM_ID_BYTES bytes (host memory) to every rank,
 * which calls qd_comm_init.  qd_reduce_sum sums the complex128 buffer of every rank in place into
 * `root` (the single reduce of a member-sharded 2DES grid / waiting-time stack).
 */
int qd_comm_unique_id(void* uid);
int qd_comm_init(int nranks, int rank, const void* uid);
int qd_reduce_sum(qd_c128* buf, size_t n, int root, void* stream);
int qd_comm_destroy(void);

#ifdef __cplusplus
}
#endif

#endif /* QDYN_H */
