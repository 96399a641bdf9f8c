"""Third-order response / 2DES on the GPU (eigen form of the reference's
RedfieldSolver.propagator + correlation_4op_3t, pyqed/oqs.py:160-357).

Setup (host, like the reference): eig of the Liouvillian/Redfield tensor and
the O(nL^3) basis changes of the four superoperators.  Grid evaluation (the
O(n^2 nL) / O(n^3 nL) part) runs in libqdyn.
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.linalg import eig, inv

from . import _lib
from ._util import default_device
from .superoperator import operator_to_superoperator


def _t(a, dev, dtype=torch.complex128):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a))).to(device=dev, dtype=dtype)


def sos_eig(R):
    """eig of the (dense) generator and its inverse eigenvector matrix (oqs.py:196-200)."""
    R = R.toarray() if hasattr(R, "toarray") else np.asarray(R)
    lam, U1 = eig(R)
    return lam, U1, inv(U1)


def sos_propagator(lam, U1, U2, t, device=None):
    """U[a, b, k] = sum_j U1[a,j] e^{lam_j t_k} U2[j,b] on the GPU (oqs.py:205-210)."""
    dev = device or default_device()
    _lib.ensure_device(dev)
    nL = len(lam)
    t = np.asarray(t, dtype=float)
    U = torch.empty((nL, nL, len(t)), dtype=torch.complex128, device=dev)
    lamt, U1t, U2t = _t(lam, dev), _t(U1, dev), _t(U2, dev)
    tt = _t(t, dev, torch.float64)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_sos_propagator(U1t.data_ptr(), U2t.data_ptr(), lamt.data_ptr(), nL, tt.data_ptr(),
                                           len(t), U.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_sos_propagator")
    return U


def eigen_factors(lam, U1, U2, oplist, signature, rho0):
    """alpha = I^T a U1, B = U2 b U1, C = U2 c U1, beta = U2 d vec(rho0)."""
    a, b, c, d = [operator_to_superoperator(op, s).toarray() for op, s in zip(oplist, signature)]
    rho0 = rho0.toarray() if hasattr(rho0, "toarray") else np.asarray(rho0)
    N = rho0.shape[0]
    idm = np.identity(N).flatten()
    alpha = (idm @ a) @ U1
    B = U2 @ b @ U1
    C = U2 @ c @ U1
    beta = U2 @ (d @ rho0.flatten())
    return alpha, B, C, beta


def response_cube(lam, alpha, B, C, beta, t3, t2, t1, device=None):
    """S[i, j, k] over (t3_i, t2_j, t1_k) on the GPU (oqs.py:327-357)."""
    dev = device or default_device()
    _lib.ensure_device(dev)
    nL = len(lam)
    t3, t2, t1 = (np.asarray(x, dtype=float) for x in (t3, t2, t1))
    out = torch.empty((len(t3), len(t2), len(t1)), dtype=torch.complex128, device=dev)
    args = [_t(x, dev) for x in (alpha, B, C, beta, lam)]
    ts = [_t(x, dev, torch.float64) for x in (t3, t2, t1)]
    with torch.cuda.device(dev):
        rc = _lib.load().qd_response_cube(*(x.data_ptr() for x in args), nL, ts[0].data_ptr(), len(t3),
                                          ts[1].data_ptr(), len(t2), ts[2].data_ptr(), len(t1), out.data_ptr(),
                                          _lib.stream_ptr(dev))
    _lib.check(rc, "qd_response_cube")
    return out


def ensemble_factors(lam, U1, U2, supops, rho0v, t2):
    """Batched eigen factors for M members: lam/U1/U2 [M, nL(, nL)], supops (a, b, c, d) [M, nL, nL]
    or shared [nL, nL]; returns alpha [M,nL], Mt [M,nL,nL] = B diag(e^{lam t2}) C, beta [M,nL]."""
    a, b, c, d = [np.broadcast_to(x, U1.shape) for x in supops]
    nL = U1.shape[-1]
    N = int(round(np.sqrt(nL)))
    idm = np.identity(N).flatten()
    alpha = np.einsum("a,mab,mbp->mp", idm, a, U1)
    Bm = U2 @ b @ U1
    Cm = U2 @ c @ U1
    Mt = Bm @ (np.exp(lam * t2)[:, :, None] * Cm)
    beta = np.einsum("mpa,mab,b->mp", U2, d, rho0v)
    return alpha, Mt, beta


def ensemble_factors_bc(lam, U1, U2, supops, rho0v):
    """t2-independent factors for a waiting-time scan: alpha [M,nL], B = U2 b U1, C = U2 c U1
    [M,nL,nL], beta [M,nL] (ensemble_factors without the e^{lam t2} contraction)."""
    a, b, c, d = [np.broadcast_to(x, U1.shape) for x in supops]
    nL = U1.shape[-1]
    N = int(round(np.sqrt(nL)))
    idm = np.identity(N).flatten()
    alpha = np.einsum("a,mab,mbp->mp", idm, a, U1)
    beta = np.einsum("mpa,mab,b->mp", U2, d, rho0v)
    return alpha, U2 @ b @ U1, U2 @ c @ U1, beta


def _uniform(t):
    """(t0, dt) when the host grid t is uniform to 1e-13 relative (np.arange / linspace grids), else None."""
    if isinstance(t, torch.Tensor):
        return None
    t = np.asarray(t, float).ravel()
    if t.size == 1:
        return float(t[0]), 0.0
    dt = (t[-1] - t[0]) / (t.size - 1)
    dev = np.max(np.abs(t - (t[0] + dt * np.arange(t.size))))
    return (float(t[0]), float(dt)) if dev <= 1e-13 * max(np.max(np.abs(t)), 1.0) else None


# ---- structural-zero pruning (selection rules).  For the 2DES pathways most eigen-index columns of
# alpha / beta (and of the waiting-time factors B, C restricted to them) are exactly zero: e.g. the 3-level
# ladder 'lccc' response keeps p in {1,3,5,7} of alpha, q in {1,3} of beta and r in {0,2,4,6} between B
# and C.  Dropping index values whose every term is an exact zero leaves the sum unchanged (only the
# floating-point summation order differs) and shrinks the GEMM's K = M * nL accordingly.
_PRUNE_CACHE: dict = {}


def _support(mask):
    """Indices (int64 numpy) where a [nL] boolean mask (numpy or tensor) is true."""
    m = mask.cpu().numpy() if isinstance(mask, torch.Tensor) else np.asarray(mask)
    return np.flatnonzero(m)


def _pruned(tag, tensors, cacheable, build):
    """build() once per input tensors.  Cached only for caller-owned device tensors: the entry keeps
    references to them, so their storage (data_ptr) cannot be recycled while the entry lives, and an
    in-place update bumps their _version and misses.  Host (numpy) inputs are pruned per call."""
    if not cacheable:
        return build()
    key = (tag,) + tuple((t.data_ptr(), t._version, tuple(t.shape), str(t.device)) for t in tensors)
    hit = _PRUNE_CACHE.get(key)
    if hit is None:
        if len(_PRUNE_CACHE) >= 8:
            _PRUNE_CACHE.pop(next(iter(_PRUNE_CACHE)))
        hit = _PRUNE_CACHE[key] = (tuple(tensors), build())
    return hit[1]


def _prune_fixed_t2(lam_t, alpha_t, Mt_t, beta_t):
    """Compact rectangular operands of the fixed-t2 ensemble sum: (swap, ax, lx, Mt_c, bz, lz) with K on
    the smaller of the two pruned index sets (swap: K over q, output transposed).  None if all-zero."""
    P = _support((alpha_t != 0).any(0))
    Q = _support((beta_t != 0).any(0))
    if P.size == 0 or Q.size == 0:
        return None
    dev = alpha_t.device
    Pi, Qi = torch.from_numpy(P).to(dev), torch.from_numpy(Q).to(dev)
    Mpq = Mt_t.index_select(1, Pi).index_select(2, Qi)
    if Q.size < P.size:
        # S^T[k, i] = sum (i * (-i beta_q)) e^{lam_q t1_k} (Mt^T)_qp (i alpha_p) e^{lam_p t3_i}
        return (True, (-1j * beta_t.index_select(1, Qi)).contiguous(), lam_t.index_select(1, Qi).contiguous(),
                Mpq.transpose(1, 2).contiguous(), (1j * alpha_t.index_select(1, Pi)).contiguous(),
                lam_t.index_select(1, Pi).contiguous())
    return (False, alpha_t.index_select(1, Pi).contiguous(), lam_t.index_select(1, Pi).contiguous(),
            Mpq.contiguous(), beta_t.index_select(1, Qi).contiguous(), lam_t.index_select(1, Qi).contiguous())


def response2d_ensemble(lam, alpha, Mt, beta, t3, t1, out=None, accumulate=False, device=None, prune=True):
    """out[i, k] (+)= sum_m (t3_i, t1_k) slice of member m at fixed t2 (GPU, split-K MFMA GEMM).

    lam, alpha, beta [M, nL], Mt [M, nL, nL] (numpy or device tensors).  Uniform host grids (the
    2DES case) build the GEMM operands from exponential tables; others from the arrays.  With
    prune=True (default) eigen indices whose alpha (t3 side) or beta (t1 side) column is exactly zero for
    every member are dropped first (the pruned form is cached per input tensors), and K runs over the
    smaller remaining set."""
    dev = device or (out.device if out is not None else default_device())
    _lib.ensure_device(dev)
    owned = all(isinstance(x, torch.Tensor) for x in (lam, alpha, Mt, beta))
    lam_t, alpha_t, Mt_t, beta_t = (x if isinstance(x, torch.Tensor) else _t(x, dev) for x in (lam, alpha, Mt, beta))
    M, nL = alpha_t.shape
    u3, u1 = _uniform(t3), _uniform(t1)
    n3 = t3.numel() if isinstance(t3, torch.Tensor) else np.asarray(t3).size
    n1 = t1.numel() if isinstance(t1, torch.Tensor) else np.asarray(t1).size
    if out is None:
        out = torch.empty((n3, n1), dtype=torch.complex128, device=dev)
        accumulate = False
    if prune:
        pr = _pruned("fixed", (lam_t, alpha_t, Mt_t, beta_t), owned,
                     lambda: _prune_fixed_t2(lam_t, alpha_t, Mt_t, beta_t))
        if pr is None:
            if not accumulate:
                out.zero_()
            return out
        swap, ax, lx, Mc, bz, lz = pr
        nx, nz = ax.shape[1], bz.shape[1]
        ga, gb = (t1, t3) if swap else (t3, t1)          # grid on the GEMM's row side, on its column side
        ua, ub = (u1, u3) if swap else (u3, u1)
        na, nb = (n1, n3) if swap else (n3, n1)
        keep = []
        if ub is not None and (nx > 16 or nz > 16 or nb > 1024):
            ub = None                                     # table build needs nx, nz <= 16, <= 1024 columns
        def grid(g, u):
            if u is not None:
                return None, u[0], u[1]
            gt = g if isinstance(g, torch.Tensor) else _t(np.asarray(g, float), dev, torch.float64)
            keep.append(gt)
            return gt.data_ptr(), 0.0, 0.0
        pa, pb = grid(ga, ua), grid(gb, ub)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_response2d_ensemble_rect(ax.data_ptr(), lx.data_ptr(), nx, Mc.data_ptr(),
                                                         bz.data_ptr(), lz.data_ptr(), nz, M, pa[0], pa[1], pa[2],
                                                         na, pb[0], pb[1], pb[2], nb, int(swap), out.data_ptr(),
                                                         int(bool(accumulate)), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_response2d_ensemble_rect")
        return out
    if u3 is not None and u1 is not None and nL <= 16 and n1 <= 1024:
        with torch.cuda.device(dev):
            rc = _lib.load().qd_response2d_ensemble_uniform(alpha_t.data_ptr(), Mt_t.data_ptr(), beta_t.data_ptr(),
                                                            lam_t.data_ptr(), M, nL, u3[0], u3[1], n3, u1[0], u1[1],
                                                            n1, out.data_ptr(), int(bool(accumulate)),
                                                            _lib.stream_ptr(dev))
        _lib.check(rc, "qd_response2d_ensemble_uniform")
        return out
    t3t = t3 if isinstance(t3, torch.Tensor) else _t(np.asarray(t3, float), dev, torch.float64)
    t1t = t1 if isinstance(t1, torch.Tensor) else _t(np.asarray(t1, float), dev, torch.float64)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_response2d_ensemble(alpha_t.data_ptr(), Mt_t.data_ptr(), beta_t.data_ptr(),
                                                lam_t.data_ptr(), M, nL, t3t.data_ptr(), t3t.numel(),
                                                t1t.data_ptr(), t1t.numel(), out.data_ptr(), int(bool(accumulate)),
                                                _lib.stream_ptr(dev))
    _lib.check(rc, "qd_response2d_ensemble")
    return out


def redfield_superop_batch(E, a_op, spec_vals):
    """Vectorised redfield_tensor (oqs.py:519-570) for M diagonal Hamiltonians E [M, N] sharing one
    Hermitian a_op already in the (shared, identity) eigenbasis; spec_vals [M, N, N] = S(-W).
    Returns R [M, N^2, N^2].  Used to build disorder ensembles (setup)."""
    E = np.asarray(E, float)
    M, N = E.shape
    I = np.identity(N)
    A = np.asarray(a_op, complex)
    opA = np.kron(A, I) - np.kron(I, A.T)
    Lm = np.asarray(spec_vals) * A[None]
    # kron(Lm, I) - kron(I, Lm^*) for every member, as [M, N, N, N, N] -> [M, N^2, N^2]
    D = (np.einsum("mac,bd->mabcd", Lm, I) - np.einsum("ac,mbd->mabcd", I, Lm.conj())).reshape(M, N * N, N * N)
    diag = (E[:, :, None] - E[:, None, :]).reshape(M, N * N)      # kron(diag E, I) - kron(I, diag E)
    R = -(opA[None] @ D)
    R[:, np.arange(N * N), np.arange(N * N)] += -1j * diag
    return R


def _prune_t2(lam_t, alpha_t, B_t, C_t, beta_t):
    """Index sets of the scan with every term exactly zero dropped: p (alpha != 0), q (beta != 0) and the
    waiting-time index r with B[:, p, r] and C[:, r, q] not all zero.  Returns compact contiguous
    (alpha_p, lam_p, B_pr, lam_r, C_rq, beta_q, lam_q) or None when the response vanishes."""
    P = _support((alpha_t != 0).any(0))
    Q = _support((beta_t != 0).any(0))
    if P.size == 0 or Q.size == 0:
        return None
    dev = alpha_t.device
    Pi, Qi = torch.from_numpy(P).to(dev), torch.from_numpy(Q).to(dev)
    Bp = B_t.index_select(1, Pi)
    Cq = C_t.index_select(2, Qi)
    R = _support((Bp != 0).any(0).any(0) & (Cq != 0).any(0).any(1))
    if R.size == 0:
        return None
    Ri = torch.from_numpy(R).to(dev)
    c = lambda x: x.contiguous()
    return (c(alpha_t.index_select(1, Pi)), c(lam_t.index_select(1, Pi)), c(Bp.index_select(2, Ri)),
            c(lam_t.index_select(1, Ri)), c(Cq.index_select(1, Ri)), c(beta_t.index_select(1, Qi)),
            c(lam_t.index_select(1, Qi)))


def response2d_t2scan(lam, alpha, B, C, beta, t3, t2, t1, out=None, accumulate=False, device=None, prune=True):
    """out[j, i, k] (+)= sum_m (t3_i, t1_k) slice of member m at waiting time t2_j (GPU).

    Mt_mj = B_m diag(e^{lam_m t2_j}) C_m is formed on the device; every t2 shares one split-K MFMA
    GEMM.  t3 and t1 must be uniform host grids (np.arange / linspace); t2 any host array or device
    float64 tensor.  prune=True drops structurally zero index values first (see T2Scan).
    Returns [n2, n3, n1] complex128."""
    dev = device or (out.device if out is not None else default_device())
    if prune:
        return T2Scan(lam, alpha, B, C, beta, t3, t1, device=dev).apply(t2, out=out, accumulate=accumulate)
    _lib.ensure_device(dev)
    lam_t, alpha_t, B_t, C_t, beta_t = (x if isinstance(x, torch.Tensor) else _t(x, dev)
                                        for x in (lam, alpha, B, C, beta))
    M, nL = alpha_t.shape
    u3, u1 = _uniform(t3), _uniform(t1)
    if u3 is None or u1 is None:
        raise ValueError("response2d_t2scan: t3 and t1 must be uniform host grids")
    n3, n1 = np.asarray(t3).size, np.asarray(t1).size
    t2t = t2 if isinstance(t2, torch.Tensor) else _t(np.atleast_1d(np.asarray(t2, float)), dev, torch.float64)
    n2 = t2t.numel()
    if out is None:
        out = torch.empty((n2, n3, n1), dtype=torch.complex128, device=dev)
        accumulate = False
    if tuple(out.shape) != (n2, n3, n1) or not out.is_contiguous() or out.dtype != torch.complex128:
        raise ValueError(f"out must be a contiguous complex128 [{n2}, {n3}, {n1}] tensor")
    with torch.cuda.device(dev):
        rc = _lib.load().qd_response2d_t2scan(alpha_t.data_ptr(), B_t.data_ptr(), C_t.data_ptr(), beta_t.data_ptr(),
                                              lam_t.data_ptr(), M, nL, u3[0], u3[1], n3, t2t.data_ptr(), n2, u1[0],
                                              u1[1], n1, out.data_ptr(), int(bool(accumulate)), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_response2d_t2scan")
    return out


class T2Scan:
    """Waiting-time scan with operands prepared once (qd_response2d_t2_operands): P = X B on the t3 grid and
    Q = C Y on the t1 grid live in caller-owned device tensors; apply(t2, out) evaluates any subset of
    waiting times (e.g. one bucket of a bucketed, overlapped reduce) without rebuilding them."""

    def __init__(self, lam, alpha, B, C, beta, t3, t1, device=None, prune=True):
        import ctypes
        dev = device or default_device()
        _lib.ensure_device(dev)
        self.dev = dev
        owned = all(isinstance(x, torch.Tensor) for x in (lam, alpha, B, C, beta))
        lam, alpha, B, C, beta = (x if isinstance(x, torch.Tensor) else _t(x, dev) for x in (lam, alpha, B, C, beta))
        self.M, nL = alpha.shape
        u3, u1 = _uniform(t3), _uniform(t1)
        if u3 is None or u1 is None:
            raise ValueError("T2Scan: t3 and t1 must be uniform host grids")
        self.n3, self.n1 = np.asarray(t3).size, np.asarray(t1).size
        if prune:
            # exact structural zeros dropped (module note above); cached per input tensors
            pr = _pruned("t2", (lam, alpha, B, C, beta), owned, lambda: _prune_t2(lam, alpha, B, C, beta))
        else:
            pr = (alpha, lam, B, lam, C, beta, lam)
        self.zero = pr is None
        if self.zero:
            self.lam, self.nL = lam, nL
            return
        ap, lp, Bc, lr, Cc, bq, lq = pr
        self.lam, self.nL = lr, lr.shape[1]            # E_j = e^{lam_r t2_j} on the GEMM's K index (m, r)
        self.index_sizes = (ap.shape[1], lr.shape[1], bq.shape[1])
        dims = [ctypes.c_int() for _ in range(3)]
        lib = _lib.load()
        _lib.check(lib.qd_response2d_t2_dims(self.M, self.nL, self.n3, self.n1, *(ctypes.byref(d) for d in dims)),
                   "qd_response2d_t2_dims")
        n3p, n1p, Kp = (d.value for d in dims)
        self.P = torch.empty((n3p, Kp), dtype=torch.complex128, device=dev)
        self.Q = torch.empty((Kp, n1p), dtype=torch.complex128, device=dev)
        with torch.cuda.device(dev):
            rc = lib.qd_response2d_t2_operands_rect(ap.data_ptr(), lp.data_ptr(), ap.shape[1], Bc.data_ptr(),
                                                    lr.data_ptr(), lr.shape[1], Cc.data_ptr(), bq.data_ptr(),
                                                    lq.data_ptr(), bq.shape[1], self.M, u3[0], u3[1], self.n3, u1[0],
                                                    u1[1], self.n1, self.P.data_ptr(), self.Q.data_ptr(),
                                                    _lib.stream_ptr(dev))
        _lib.check(rc, "qd_response2d_t2_operands_rect")

    def apply(self, t2, out=None, accumulate=False):
        t2t = t2 if isinstance(t2, torch.Tensor) else _t(np.atleast_1d(np.asarray(t2, float)), self.dev, torch.float64)
        n2 = t2t.numel()
        if out is None:
            out = torch.empty((n2, self.n3, self.n1), dtype=torch.complex128, device=self.dev)
            accumulate = False
        if tuple(out.shape) != (n2, self.n3, self.n1) or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous [{n2}, {self.n3}, {self.n1}] tensor")
        if self.zero:
            if not accumulate:
                out.zero_()
            return out
        with torch.cuda.device(self.dev):
            rc = _lib.load().qd_response2d_t2_apply(self.P.data_ptr(), self.Q.data_ptr(), self.lam.data_ptr(), self.M,
                                                    self.nL, self.n3, self.n1, t2t.data_ptr(), n2, out.data_ptr(),
                                                    int(bool(accumulate)), _lib.stream_ptr(self.dev))
        _lib.check(rc, "qd_response2d_t2_apply")
        return out
