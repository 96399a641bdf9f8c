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
 *   - the caller owns every buffer it passes; the library only keeps internal
 *     workspaces (released by qd_shutdown);
 *   - calls are asynchronous on `stream` (a hipStream_t, NULL = default stream);
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

typedef struct qd_c128 {
  double re;
  double im;
} qd_c128;

/* ------------------------------------------------------------ runtime ---- */
int qd_version(void);                 /* e.g. 100 = 0.1.0                      */
const char* qd_last_error(void);      /* thread-local message of last failure */
int qd_init(int device);              /* hipSetDevice + warm-up               */
int qd_device_count(int* count);      /* host pointer                         */
int qd_shutdown(void);                /* frees cached workspaces              */
int qd_synchronize(void* stream);     /* hipStreamSynchronize                 */

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
 * Constraints: 1 <= N <= 1024, 0 <= nc <= 8, 0 <= ne <= 16, B >= 1.
 */
int qd_lindblad_rk4(const qd_c128* H, const qd_c128* C, int nc, qd_c128* rho,
                    int B, int N, double dt, int nsteps, const qd_c128* E,
                    int ne, qd_c128* obs, qd_c128* snap, int save_every,
                    void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QDYN_H */
