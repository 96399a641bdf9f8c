"""Liouville-space helpers (mirror of pyqed/superoperator.py, host-side setup).

Conventions as the reference: vec(rho) is row-major (rho.flatten(),
superoperator.py:111-150); left action kron(a, I), right action kron(I, a.T)
(superoperator.py:200-246).  These build operators (setup); propagation runs
in libqdyn.
"""
from __future__ import annotations

import numpy as np
from scipy.sparse import csr_matrix, identity, issparse, kron


def dag(a):
    return a.conjugate().transpose()


def operator_to_vector(rho):
    if isinstance(rho, np.ndarray):
        return rho.flatten()
    return rho.toarray().flatten()


def dm2vec(rho):
    """superoperator.py:130-150 (sparse input -> lil column vector, dense -> flatten)."""
    if issparse(rho):
        n, m = rho.shape
        return rho.tolil().reshape((n * m, 1))
    return rho.flatten()


def operator_to_superoperator(a, kind="commutator"):
    """superoperator.py:200-246."""
    N = a.shape[-1]
    idm = identity(N)
    if kind in ["commutator", "c", "-"]:
        return csr_matrix(kron(a, idm) - kron(idm, a.T))
    elif kind in ["left", "l"]:
        return csr_matrix(kron(a, idm))
    elif kind in ["right", "r"]:
        return csr_matrix(kron(idm, a.T))
    elif kind in ["anticommutator", "a", "+"]:
        return csr_matrix(kron(a, idm) + kron(idm, a.T))
    raise ValueError("Error: superoperator {} does not exist.".format(kind))


def op2sop(a, kind="commutator"):
    return operator_to_superoperator(a, kind=kind)


def to_super(a, kind="commutator"):
    return operator_to_superoperator(a, kind=kind)


def left(a):
    n = a.shape[-1]
    return csr_matrix(kron(a, identity(n)))


def right(a):
    n = a.shape[-1]
    return csr_matrix(kron(identity(n), a.T))


def lindblad_dissipator(l):
    """superoperator.py:249-253."""
    return csr_matrix(kron(l, l.conj()) - 0.5 * operator_to_superoperator(dag(l).dot(l), kind="anticommutator"))


def liouvillian(H, c_ops):
    """superoperator.py:29-58: L = -i op2sop(H) + sum lindblad_dissipator(c)."""
    if c_ops is None:
        c_ops = []
    l = -1j * operator_to_superoperator(H)
    for c_op in c_ops:
        l = l + lindblad_dissipator(c_op)
    return csr_matrix(l)


def obs(rho, a):
    """superoperator.py:313-314: <<a^+|rho>>."""
    return np.vdot(operator_to_vector(dag(a)), rho)


def trace(rho):
    import math
    n = math.isqrt(len(rho))
    return np.vdot(operator_to_vector(np.identity(n)), rho)


def cdot(a, b):
    """a^+ b (superoperator.py:370-385)."""
    return dag(a) @ b


def _pole_sum_time(coeff, lam, t):
    """cor[i] = sum_n coeff_n e^{lam_n t_i} on the GPU (qd_response2d_ensemble with n1 = 1)."""
    from .response import response2d_ensemble
    n = len(lam)
    Mt = (-1j * np.eye(n))[None]          # the kernel applies (-i)^3 = i
    out = response2d_ensemble(np.asarray(lam)[None], np.asarray(coeff)[None], Mt, np.ones((1, n), complex),
                              np.asarray(t, float), np.zeros(1))
    return out[:, 0].cpu().numpy()


def _pole_sum_freq(coeff, lam, w):
    import torch
    from . import _lib
    from ._util import default_device
    dev = default_device()
    _lib.ensure_device(dev)
    c = torch.from_numpy(np.ascontiguousarray(coeff, dtype=complex)).to(dev)
    l = torch.from_numpy(np.ascontiguousarray(lam, dtype=complex)).to(dev)
    wt = torch.from_numpy(np.ascontiguousarray(w, dtype=float)).to(dev)
    out = torch.empty(len(w), dtype=torch.complex128, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_resolvent_sum(c.data_ptr(), l.data_ptr(), len(lam), wt.data_ptr(), len(w),
                                          out.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_resolvent_sum")
    return out.cpu().numpy()


def _bilinear_grid(lam, coeff, taulist, tlist):
    """cor[i, j] = sum_mn e^{lam_m tau_i} coeff[m, n] e^{lam_n t_j} on the GPU (MFMA GEMM kernel)."""
    from .response import response2d_ensemble
    n = len(lam)
    out = response2d_ensemble(np.asarray(lam)[None], np.ones((1, n), complex), (-1j * np.asarray(coeff))[None],
                              np.ones((1, n), complex), np.asarray(taulist, float), np.asarray(tlist, float))
    return out.cpu().numpy()


class Lindblad_solver:
    """Eigen-decomposition Liouville solver (drop-in for superoperator.Lindblad_solver,
    superoperator.py:455-772).  eig of L on the host (setup, as the reference); every
    time/frequency grid evaluation runs in libqdyn."""

    def __init__(self, H, c_ops=None):
        self.H = H
        self.c_ops = c_ops
        self.L = None
        self.dim = H.shape[-1] ** 2
        self.idv = operator_to_vector(np.identity(H.shape[-1]))
        self.left_eigvecs = None
        self.right_eigvecs = None
        self.eigvals = None
        self.norm = None

    def liouvillian(self):
        L = liouvillian(self.H, self.c_ops)
        self.L = L
        return L

    def eigenstates(self, k=None):
        """superoperator.py:489-522 (k=None: full eig with left/right vectors)."""
        import scipy.linalg
        L = self.liouvillian() if self.L is None else self.L
        if k is not None:
            raise NotImplementedError("partial (k) diagonalisation: the reference path is broken (undefined w)")
        w, vl, vr = scipy.linalg.eig(L.toarray(), left=True, right=True)
        self.eigvals, self.left_eigvecs, self.right_eigvecs = w, vl, vr
        self.norm = np.diagonal(cdot(vl, vr)).real
        return w, vr, vl

    def _ensure(self):
        if self.eigvals is None:
            self.eigenstates()

    def evolve(self, rho0, tlist, e_ops):
        """Intended semantics of superoperator.py:524-563 (the reference crashes building
        Result(times=...)): observables[i, m] = obs(U1 (coeff e^{lam t_i}), e_m).
        Uses the complex biorthogonal norm l_n^+ r_n: the reference's `self.norm` keeps only
        its real part (superoperator.py:514), which the correlation_* methods mirror for parity
        but which is wrong whenever l_n^+ r_n has a phase."""
        from .mol import Result
        self._ensure()
        evals, U1, U2 = self.eigvals, self.right_eigvecs, self.left_eigvecs
        norm = np.diagonal(cdot(U2, U1))
        r0 = operator_to_vector(to_dense(rho0))
        coeff = (U2.conj().T @ r0) / norm
        tlist = np.asarray(tlist, float)
        observables = np.zeros((len(tlist), len(e_ops)), dtype=complex)
        for m, e in enumerate(e_ops):
            ev = operator_to_vector(dag(to_dense(e)))
            observables[:, m] = _pole_sum_time((ev.conj() @ U1) * coeff, evals, tlist)
        result = Result(dt=tlist[1] - tlist[0] if len(tlist) > 1 else 0.0, Nt=len(tlist) - 1, t0=tlist[0])
        result.times = tlist
        result.observables = observables
        return result

    def _coeff_2op(self, a, b, rho0):
        evals, U1, U2, norm = self.eigvals, self.right_eigvecs, self.left_eigvecs, self.norm
        x = self.idv.conj() @ (left(to_dense(a)) @ U1)
        z = U2.conj().T @ operator_to_vector(to_dense(b) @ to_dense(rho0))
        return x * z / norm

    def correlation_2op_1t(self, rho0, ops, tlist):
        """<A(t)B> (superoperator.py:565-601)."""
        self._ensure()
        a, b = ops
        return _pole_sum_time(self._coeff_2op(a, b, rho0), self.eigvals, tlist)

    def correlation_2op_1w(self, rho0, ops, w):
        """S(w) = sum_n -coeff_n/(lam_n + i w) (superoperator.py:603-636)."""
        self._ensure()
        a, b = ops
        return _pole_sum_freq(self._coeff_2op(a, b, rho0), self.eigvals, w)

    def _coeff_3op(self, ops, rho0):
        a, b, c = (to_dense(x) for x in ops)
        U1, U2, norm = self.right_eigvecs, self.left_eigvecs, self.norm
        x = self.idv.conj() @ (left(b) @ U1)
        z = U2.conj().T @ operator_to_vector(c @ to_dense(rho0) @ a)
        return x * z / norm

    def correlation_3op_1t(self, rho0, ops, t):
        """superoperator.py:638-668."""
        self._ensure()
        return _pole_sum_time(self._coeff_3op(ops, rho0), self.eigvals, t)

    def correlation_3op_1w(self, rho0, ops, w):
        """superoperator.py:670-700."""
        self._ensure()
        return _pole_sum_freq(self._coeff_3op(ops, rho0), self.eigvals, w)

    def correlation_3op_2t(self, rho0, ops, tlist, taulist, k=None):
        """<A(t)B(t+tau)C(t)> = e^{lam tau}^T coeff e^{lam t} (superoperator.py:702-753);
        returns shape (len(taulist), len(tlist)).  The O(k^4) double loop of coeff becomes two
        matrix products (host setup); the grid is a GEMM on the GPU."""
        self._ensure()
        a, b, c = (to_dense(x) for x in ops)
        U1, U2, norm = self.right_eigvecs, self.left_eigvecs, self.norm
        r0 = operator_to_vector(to_dense(rho0))
        x = (self.idv.conj() @ (left(b) @ U1)) / norm
        W = U2.conj().T @ (right(a) @ (left(c) @ U1))
        z = (U2.conj().T @ r0) / norm
        coeff = x[:, None] * W * z[None, :]
        return _bilinear_grid(self.eigvals, coeff, taulist, tlist)

    def correlation_4op_2t(self, rho0, ops, tlist, taulist, k=None):
        """superoperator.py:755-772: 3op_2t with [a, b@c, d]."""
        if len(ops) != 4:
            raise ValueError('Number of operators is not 4.')
        a, b, c, d = ops
        return self.correlation_3op_2t(rho0, [a, to_dense(b) @ to_dense(c), d], tlist, taulist, k)


def to_dense(a):
    if issparse(a):
        return a.toarray()
    return np.asarray(a)
