"""DEOMSolver.correlation_4op_3t without the eigendecomposition (heom/deom.py:1127-1209, if_full=True).

The reference diagonalises the dense ADO Liouvillian P (n = nmax ns^2; 24,752 at the bench hierarchy, a 9.8 GB
matrix whose eig the reference cannot run) and evaluates, for every (w_x, w_y),

    c(w_x, w_y) = Tr_sys[ A1 V D(w_x) (V^-1 A2 V) e^{Delta T} (V^-1 A3 V) D(w_y) V^-1 A4 rho ],
    D(w) = diag(1 / (-Delta - i w)),

which is, for a diagonalisable P, exactly

    c(w_x, w_y) = u^T R(w_x) A2 e^{P T} A3 R(w_y) v,    R(w) = (-P - i w)^-1,

with u^T x = Tr_sys(A1 x_0) (the ADO-0 rows) and v = A4 rho in the ADO-0 rows.  Here:

  * r(w_y) = R(w_y) v for every w_y from ONE Arnoldi basis of P started at v (Krylov spaces are shift
    invariant: (-P - s) V_k = V_{k+1} (-H_k - s)), the small shifted Hessenberg systems solved per shift;
  * l(w_x) = R(w_x)^T u likewise from one Arnoldi basis of P^T started at u;
  * e^{P T} on the n_w vectors of the shorter side (or e^{P^T T} on the left ones) by Taylor substeps with
    ||P tau|| <= 5 (degree 48, remainder < 1e-26 per substep);
  * c = l(w_x)^T A2 e^{PT} A3 r(w_y): one complex GEMM.

Every application of P or P^T is the DEOM stencil kernel (qd_deom_apply); P^T is the same operator form on
transposed tables (transposed_tables).  Orthogonalisation (classical Gram-Schmidt twice) and the final products
are device BLAS calls on device-resident bases; the host only solves the k x k shifted systems.  The Krylov
residual of every shift is driven below `tol` relative to its solution norm.  Accuracy against the eigen form:
tests/test_deom_krylov_gpu.py (1e-9 at the fixture hierarchies; the eigen form itself carries cond(V) eps).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

TAYLOR_RADIUS = 5.0   # substeps tau with ||P tau||_inf <= TAYLOR_RADIUS
TAYLOR_DEGREE = 48    # terms per substep: remainder <= e^5 5^49 / 49! < 1e-26; largest term 5^5 / 5! = 26 (the sum of the
                      # terms' magnitudes <= e^5: ~2 digits of cancellation at most); 71 substeps x 48 terms at the bench
                      # hierarchy against 118 x 36 at radius 3 and 352 x 20 at radius 1
ARNOLDI_DCGS2 = True  # device Arnoldi by delayed CGS2 (qd_arnoldi_dcgs2_step: 2 basis passes per step); False: CGS2 (4)


def transposed_tables(minus, plus, coef):
    """(minus', plus', coef') with ado_liouvillian(keys, minus', plus', coef', damp, H^T, Q^T) = P^T.

    P's block from ADO n to its minus neighbour m = minus[n, k] is coef0 (Q (x) I) + coef1 (I (x) Q^T); transposed
    it is coef0 (Q^T (x) I) + coef1 (I (x) Q), ADO m's link to its PLUS neighbour n: the same operator form with
    Q -> Q^T, the roles of the two tables exchanged and the prefactors read at the other end of the link (the
    commutator-form plus links likewise become minus links).  Checked against P.T in tests/test_deom_krylov_cpu.py."""
    minus = np.asarray(minus)
    plus = np.asarray(plus)
    coef = np.asarray(coef)
    cT = np.zeros_like(coef)
    for k in range(minus.shape[1]):
        h = plus[:, k] >= 0
        cT[h, k, 0] = coef[plus[h, k], k, 0]
        cT[h, k, 1] = coef[plus[h, k], k, 1]
        h = minus[:, k] >= 0
        cT[h, k, 2] = coef[minus[h, k], k, 2]
    return plus.copy(), minus.copy(), cT


def inf_norm_bound(minus, plus, coef, damp, H, Q, mode):
    """An upper bound of ||P||_inf (max row sum of the dense generator), from the tables."""
    H = np.asarray(H)
    Q = np.asarray(Q).reshape(-1, H.shape[0], H.shape[0])
    nH = np.abs(H).sum(1).max() + np.abs(H).sum(0).max()
    qi = np.abs(Q).sum(2).max(1)   # ||Q_m||_inf
    q1 = np.abs(Q).sum(1).max(1)   # ||Q_m||_1
    mode = np.asarray(mode)
    has_m = np.asarray(minus) >= 0
    has_p = np.asarray(plus) >= 0
    c = np.abs(np.asarray(coef))
    rows = np.abs(np.asarray(damp)) + nH
    rows = rows + (has_m * (c[..., 0] * qi[mode][None] + c[..., 1] * q1[mode][None])).sum(1)
    rows = rows + (has_p * c[..., 2] * (qi + q1)[mode][None]).sum(1)
    return float(rows.max())


class DeomOperator:
    """y = alpha P x (or P^T) on device vectors [B][nmax][ns][ns] through qd_deom_apply."""

    def __init__(self, dev, minus, plus, coef, damp, mode, H, Q, ns):
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
        c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
        self.dev, self.ns = dev, ns
        self.nmax, self.K = np.asarray(minus).shape
        self.tabs = (i32(minus), i32(plus), c128(coef), c128(damp), i32(mode))
        self.H = c128(H)
        self.Q = c128(np.asarray(Q).reshape(-1, ns, ns))
        self.nmod = self.Q.shape[0]
        self.n = self.nmax * ns * ns
        self.norm = inf_norm_bound(minus, plus, coef, damp, H, Q, mode)
        self.launches = 0        # qd_deom_apply calls and the vectors they applied P to (roofline bookkeeping)
        self.vec_applies = 0

    def apply(self, x, y, alpha=1.0, ado_major=False, x0=None):
        """y <- x0 + alpha P x (x0 None: alpha P x); x, y, x0 contiguous [B, n] (or [n]) complex128 on the device, y
        aliasing neither; ado_major: all three are [nmax][B][ns][ns] (the batched ADO-major kernels, ns^2 <= 64 and
        K <= 8)."""
        B = x.numel() // self.n
        mi, pl, coef, damp, mode = self.tabs
        with torch.cuda.device(self.dev):
            rc = _lib.load().qd_deom_apply(x.data_ptr(), y.data_ptr(), _lib.ptr(x0), B, self.nmax, self.K, self.ns, mi.data_ptr(),
                                           pl.data_ptr(), coef.data_ptr(), damp.data_ptr(), mode.data_ptr(),
                                           self.nmod, self.H.data_ptr(), self.Q.data_ptr(), float(alpha),
                                           1 if ado_major else 0,
                                           _lib.stream_ptr(self.dev))
        _lib.check(rc, "qd_deom_apply")
        self.launches += 1
        self.vec_applies += B
        return y


def _hess_solve_dev(Hd, k, beta, shifts, want_y):
    """qd_shifted_hessenberg_solve on the device Arnoldi matrix Hd [(m + 1), m] (leading k x k block, row k the
    sub-diagonal entry h_{k+1,k}): (Y [S, k] or None, residuals [S] on the device).  Shifts are chunked so that the
    pivot-row scratch (S k^2 complex) stays <= 1 GB."""
    dev = Hd.device
    sh_all = torch.from_numpy(np.asarray(shifts, dtype=complex)).to(dev)
    S = len(sh_all)
    Y = torch.empty((S, k), dtype=torch.complex128, device=dev) if want_y else None
    res = torch.empty(S, dtype=torch.float64, device=dev)
    chunk = max(1, (1 << 30) // (16 * k * k)) if want_y else S
    lib = _lib.load()
    with torch.cuda.device(dev):
        for c0 in range(0, S, chunk):
            c1 = min(S, c0 + chunk)
            rc = lib.qd_shifted_hessenberg_solve(Hd.data_ptr(), Hd.shape[1], k, sh_all[c0:].data_ptr(), c1 - c0,
                                                 float(beta), Y[c0:].data_ptr() if want_y else None,
                                                 res[c0:].data_ptr(), _lib.stream_ptr(dev))
            _lib.check(rc, "qd_shifted_hessenberg_solve")
    return Y, res


def _shift_solutions_dev(Hk, beta, shifts):
    """y(s) with (-H_k - s I) y = beta e_1 for every shift s, on the device: Gaussian elimination of the upper
    Hessenberg systems with adjacent-row pivoting (as _shift_residuals) and back substitution, vectorised over the
    shifts as tensor operations (chunks of shifts holding <= 1 GB of triangular factors).  (hipBLAS' batched getrf
    refused the k ~ 500 batches with ALLOC_FAILED.)  Hk: [k, k] complex128 device tensor.  Returns Y [S, k]."""
    k = Hk.shape[0]
    dev = Hk.device
    sh_all = torch.from_numpy(np.asarray(shifts, dtype=complex)).to(dev)
    chunk = max(1, (1 << 30) // (16 * k * k))
    out = []
    for c0 in range(0, len(sh_all), chunk):
        sh = sh_all[c0:c0 + chunk]
        S = len(sh)
        U = torch.empty((S, k, k), dtype=Hk.dtype, device=dev)
        gv = torch.empty((S, k), dtype=Hk.dtype, device=dev)
        cur = (-Hk[0]).expand(S, k).clone()
        cur[:, 0] -= sh
        g = torch.full((S,), beta, dtype=Hk.dtype, device=dev)
        zero = torch.zeros_like(g)
        for j in range(k - 1):
            nxt = (-Hk[j + 1]).expand(S, k).clone()
            nxt[:, j + 1] -= sh
            swap = nxt[:, j].abs() > cur[:, j].abs()
            piv = torch.where(swap[:, None], nxt, cur)
            oth = torch.where(swap[:, None], cur, nxt)
            gp = torch.where(swap, zero, g)
            go = torch.where(swap, g, zero)
            m = oth[:, j] / piv[:, j]
            U[:, j] = piv
            gv[:, j] = gp
            cur = oth - m[:, None] * piv
            g = go - m * gp
        U[:, k - 1] = cur
        gv[:, k - 1] = g
        y = torch.zeros((S, k), dtype=Hk.dtype, device=dev)
        for i in range(k - 1, -1, -1):
            acc = gv[:, i] - (U[:, i, i + 1:] * y[:, i + 1:]).sum(1) if i < k - 1 else gv[:, i]
            y[:, i] = acc / U[:, i, i]
        out.append(y)
    return torch.cat(out)


def _shift_residuals(Hh, k, beta, shifts):
    """|h_{k+1,k} y_k(s)| / beta for every shift, y(s) the FOM solution of (-H_k - s) y = beta e_1, without solving
    for y: Gaussian elimination of the Hessenberg systems with adjacent-row pivoting, vectorised over the shifts,
    keeps one active row per shift (O(S k) memory, O(S k^2) work); the last pivot gives y_k."""
    S = len(shifts)
    cur = np.broadcast_to(-Hh[0, :k], (S, k)).copy()     # transformed row 0 of A_s = -H_k - s
    cur[:, 0] -= shifts
    g = np.full(S, beta, dtype=complex)                   # transformed right-hand side entry of the active row
    for j in range(k - 1):
        nxt = np.broadcast_to(-Hh[j + 1, :k], (S, k)).copy()
        nxt[:, j + 1] -= shifts
        swap = np.abs(nxt[:, j]) > np.abs(cur[:, j])
        piv = np.where(swap[:, None], nxt, cur)
        oth = np.where(swap[:, None], cur, nxt)
        gp = np.where(swap, 0.0, g)                       # the next original row's right-hand side entry is 0
        go = np.where(swap, g, 0.0)
        m = oth[:, j] / piv[:, j]
        cur = oth - m[:, None] * piv
        g = go - m * gp
    yk = g / cur[:, k - 1]
    return np.abs(Hh[k, k - 1] * yk) / beta


def shifted_krylov_solve(op, b, shifts, tol=1e-12, m_max=None, first_check=20):
    """x(s) = (-P - s)^-1 b for every s in `shifts` (complex array) from one Arnoldi basis of P.

    Classical Gram-Schmidt with one re-orthogonalisation on device-resident basis vectors; on the device by default
    in its delayed form (ARNOLDI_DCGS2: the re-orthogonalisation of v_j is folded into the projection pass of the
    next step through the Arnoldi relation, krylov.hip).  At checkpoints the FOM
    residual |h_{k+1,k} y_k(s)| of every shift is evaluated on the host without solving for y (_shift_residuals); the
    next checkpoint is placed where the log-linear trend of the worst residual reaches the target (at least 10 and
    at most 50 % more steps).  Converged when the worst residual is below tol^1.1 (relative to ||b||) and the
    solutions' own residuals below tol ||y(s)||.  Returns (X [S, n] on the device, k)."""
    n = op.n
    if m_max is None:   # basis memory capped at ~8 GB
        m_max = int(max(50, min(4000, (8 << 30) // (16 * n) - 2)))
    dev = op.dev
    gpu = dev.type == "cuda"
    lowsync = gpu and ARNOLDI_DCGS2
    V = torch.empty((m_max + 2, n), dtype=torch.complex128, device=dev)
    Hd = torch.zeros((m_max + 2, m_max + 1), dtype=torch.complex128, device=dev)
    W = torch.empty(n, dtype=torch.complex128, device=dev)
    beta = float(torch.linalg.vector_norm(b))
    if beta == 0.0:
        return torch.zeros((len(shifts), n), dtype=torch.complex128, device=dev), 0
    if lowsync:   # the delayed step normalises V[0] itself (its j = 0 case)
        V[0] = b
    else:
        V[0] = b / beta
    shifts = np.asarray(shifts, dtype=complex)
    check = first_check
    k_done = None
    hist = []
    target = tol ** 1.1
    if gpu:   # CGS2 on the device: qd_cgs_project (h = V^H w into the Hessenberg column) + in-place GEMV updates
        lib = _lib.load()
        hbuf = torch.empty(m_max + 2, dtype=torch.complex128, device=dev)
        ldh = Hd.stride(0)
        col = lambda r, c: Hd.data_ptr() + (r * ldh + c) * 16
        if lowsync:
            stv = torch.empty(16 * (m_max + 2), dtype=torch.complex128, device=dev)
            csv = torch.empty(2 * (m_max + 3), dtype=torch.complex128, device=dev)
    for j in range(m_max + 1 if lowsync else m_max):
        op.apply(V[j], W)
        if lowsync:
            # delayed CGS2 (krylov.hip): finishes v_{j} (its reorthogonalisation, norm and the Hessenberg column j-1)
            # and forms the first-pass candidate u_{j+1} from W = P u_j: two passes over the basis per step
            _lib.check(lib.qd_arnoldi_dcgs2_step(V.data_ptr(), n, j, n, W.data_ptr(), Hd.data_ptr(), ldh,
                                                 stv.data_ptr(), csv.data_ptr(), _lib.stream_ptr(dev)),
                       "qd_arnoldi_dcgs2_step")
            if j == 0:
                continue
            k = j
        else:
            Vj = V[:j + 1]
            if gpu:
                st = _lib.stream_ptr(dev)
                for _ in range(2):   # classical Gram-Schmidt, applied twice; Hd[:j+1, j] accumulates h1 + h2
                    _lib.check(lib.qd_cgs_project(V.data_ptr(), n, j + 1, n, W.data_ptr(), hbuf.data_ptr(),
                                                  col(0, j), ldh, st), "qd_cgs_project")
                    W.addmv_(Vj.transpose(0, 1), hbuf[:j + 1], alpha=-1)
                # Hd[j+1, j] = ||W||, V[j+1] = W / max(||W||, 1e-300): an exact breakdown (||W|| = 0) must not turn
                # the basis into NaN before the next checkpoint, where the zero sub-diagonal entry ends the solve
                # (ADVICE r05); no host read per step
                _lib.check(lib.qd_cgs_normalize(W.data_ptr(), n, V[j + 1].data_ptr(), col(j + 1, j), st),
                           "qd_cgs_normalize")
            else:
                h = torch.mv(Vj, W.conj()).conj()
                W -= torch.mv(Vj.transpose(0, 1), h)
                h2 = torch.mv(Vj, W.conj()).conj()
                W -= torch.mv(Vj.transpose(0, 1), h2)
                h += h2
                nrm = torch.linalg.vector_norm(W)
                Hd[:j + 1, j] = h
                Hd[j + 1, j] = nrm
                V[j + 1] = W / torch.clamp(nrm, min=1e-300)
            k = j + 1
        if k != check and k != m_max:
            continue
        if dev.type == "cuda":   # device solves (qd_shifted_hessenberg_solve); only scalars come back
            Hk1 = Hd[:k + 1, :k]
            sub_d = torch.diagonal(Hk1, -1).abs()
            small = torch.cat([sub_d, Hk1.abs().max()[None]]).cpu().numpy()
            sub, hmax = small[:k], small[k]
        else:
            Hh = Hd[:k + 1, :k].cpu().numpy()
            sub, hmax = np.abs(np.diag(Hh, -1)), np.abs(Hh).max()
        brk = np.nonzero(sub < 1e-14 * max(hmax, 1e-300))[0]
        if len(brk):   # invariant subspace: the Krylov solution is exact
            k_done = int(brk[0]) + 1
            break
        if dev.type == "cuda":
            res = float(_hess_solve_dev(Hd, k, beta, shifts, False)[1].max())
        else:
            res = float(_shift_residuals(Hh, k, beta, shifts).max())
        hist.append((k, res))
        if res < target:
            if dev.type == "cuda":
                Yd, rd = _hess_solve_dev(Hd, k, beta, shifts, True)
                ok = bool(torch.all(rd * beta < tol * torch.clamp(torch.linalg.vector_norm(Yd, dim=1), min=1e-300)))
            else:
                Yd = _shift_solutions_dev(Hd[:k, :k], beta, shifts)
                Y = Yd.cpu().numpy()
                ok = np.all(np.abs(Hh[k, k - 1] * Y[:, -1]) < tol * np.maximum(np.linalg.norm(Y, axis=1), 1e-300))
            if ok:
                k_done = k
                return Yd @ V[:k], k
        step = max(10, k // 4)
        if len(hist) >= 2 and hist[-2][1] > res > 0:   # extrapolate the log residual to the target
            (k0, r0), (k1, r1) = hist[-2], hist[-1]
            rate = (np.log(r1) - np.log(r0)) / (k1 - k0)
            if rate < 0:
                step = int(np.clip((np.log(target) - np.log(r1)) / rate, 10, max(10, k // 2)))
        check = min(m_max, k + step)
    if k_done is None:
        raise RuntimeError(f"shifted Krylov solve: no convergence to {tol:g} within {m_max} Arnoldi steps")
    if dev.type == "cuda":
        return _hess_solve_dev(Hd, k_done, beta, shifts, True)[0] @ V[:k_done], k_done
    return _shift_solutions_dev(Hd[:k_done, :k_done], beta, shifts) @ V[:k_done], k_done


def expv_taylor(op, X, T, graph=True):
    """e^{P T} X for X [B, n] on the device: Taylor substeps tau = T / s with ||P tau||_inf <= TAYLOR_RADIUS, each
    the degree-TAYLOR_DEGREE polynomial in Horner form, y <- x + (tau / j) P y for j = TAYLOR_DEGREE .. 1 (every step one stencil
    launch with the axpy fused: qd_deom_apply's x0).  B > 1 vectors run ADO-major ([nmax][B][ns][ns], the batched
    stencil kernels).  graph=True captures one substep (its stencil launches and the closing copy, fixed buffers) into
    a HIP graph and replays it s times (replays are bit for bit, tests/test_graph_capture_gpu.py)."""
    if T == 0:
        return X.clone(), 0
    s = max(1, int(np.ceil(abs(T) * op.norm / TAYLOR_RADIUS)))
    tau = T / s
    B = X.numel() // op.n
    am = X.is_cuda and B > 1 and op.ns * op.ns <= 64 and getattr(op, "K", 99) <= 8
    out = X.reshape(B, op.nmax, -1).transpose(0, 1).contiguous() if am else X.clone()
    t1 = torch.empty_like(out)
    t2 = torch.empty_like(out)
    fused = hasattr(op, "K")   # DeomOperator (the CPU stand-ins of the host tests have no x0)

    def substep():
        src = out
        for j in range(TAYLOR_DEGREE, 0, -1):
            dst = t1 if j % 2 == 0 else t2
            if fused:
                op.apply(src, dst, tau / j, ado_major=am, x0=out)
            else:
                op.apply(src, dst, tau / j)
                dst.add_(out)
            src = dst
        out.copy_(src)

    def result():
        return out.transpose(0, 1).reshape(X.shape).contiguous() if am else out

    if not graph or s < 2 or not X.is_cuda:   # (CPU stand-in operators in the host tests)
        for _ in range(s):
            substep()
        return result(), s
    side = torch.cuda.Stream(op.dev)
    side.wait_stream(torch.cuda.current_stream(op.dev))
    g = torch.cuda.CUDAGraph()
    launches, vecs = getattr(op, "launches", 0), getattr(op, "vec_applies", 0)
    with torch.cuda.graph(g, stream=side):
        substep()
    if hasattr(op, "launches"):   # the capture enqueued nothing; count the replays' stencil launches instead
        op.launches, op.vec_applies = launches, vecs
    for _ in range(s):
        g.replay()
        if hasattr(op, "launches"):
            op.launches += TAYLOR_DEGREE
            op.vec_applies += TAYLOR_DEGREE * B
    return result(), s


def act_block(blk, X, nmax, n2):
    """(I_nmax (x) blk) on the rows of X [S, nmax n2] (generate_actions' per-ADO action)."""
    b = torch.from_numpy(np.ascontiguousarray(blk)).to(X.device)
    S = X.shape[0]
    return torch.einsum('xy,say->sax', b, X.reshape(S, nmax, n2)).reshape(S, nmax * n2).contiguous()


def corr4_krylov(op, opT, A1, A2, A3, A4, rho0, T, w_x, w_y, nmax, ns, tol=1e-12):
    """c[i, j] of correlation_4op_3t(if_full=True) from the operators P (op) and P^T (opT): A1..A4 the per-ADO action
    blocks (ns^2 x ns^2) of operator_d, _c, _b, _a in the reference's order.  Returns (c [len(w_x), len(w_y)] numpy,
    info dict)."""
    n2 = ns * ns
    n = nmax * n2
    dev = op.dev
    wx = np.asarray(w_x, dtype=float)
    wy = np.asarray(w_y, dtype=float)
    v = torch.zeros(n, dtype=torch.complex128, device=dev)
    v[:n2] = torch.from_numpy(np.ascontiguousarray(A4 @ np.asarray(rho0, dtype=complex).reshape(-1))).to(dev)
    diag = np.arange(ns) * (ns + 1)
    u = torch.zeros(n, dtype=torch.complex128, device=dev)
    u[:n2] = torch.from_numpy(np.ascontiguousarray(A1[diag].sum(axis=0))).to(dev)   # u^T x = Tr_sys(A1 x_0)
    R, kr = shifted_krylov_solve(op, v, 1j * wy, tol)    # r(w_y) = (-P - i w_y)^-1 v      [n_wy, n]
    L, kl = shifted_krylov_solve(opT, u, 1j * wx, tol)   # l(w_x) = (-P^T - i w_x)^-1 u    [n_wx, n]
    if len(wy) <= len(wx):   # e^{PT} on the right-hand vectors
        Rm, s = expv_taylor(op, act_block(A3, R, nmax, n2), T)
        C = L @ act_block(A2, Rm, nmax, n2).transpose(0, 1)
    else:                    # e^{P^T T} on the left-hand ones: c = (e^{P^T T} A2^T l)^T (A3 r)
        Lm, s = expv_taylor(opT, act_block(A2.T, L, nmax, n2), T)
        C = Lm @ act_block(A3, R, nmax, n2).transpose(0, 1)
    info = {"method": "krylov", "krylov_dim_right": kr, "krylov_dim_left": kl, "taylor_substeps": s,
            "norm_bound": op.norm}
    if hasattr(op, "launches"):   # DeomOperator's bookkeeping (the bench's roofline)
        info["stencil_launches"] = op.launches + opT.launches
        info["stencil_vector_applications"] = op.vec_applies + opT.vec_applies
    return C.cpu().numpy(), info
