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
