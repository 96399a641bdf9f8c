"""NumPy restatement of the Redfield path and Liouville-space correlations
(test infrastructure only).

Follows:
  pyqed/superoperator.py:200-246  operator_to_superoperator (row-major vec,
                                  kron(a,I) left, kron(I,a.T) right)
  pyqed/superoperator.py:29-58,249-253  liouvillian / lindblad_dissipator
  pyqed/oqs.py:519-570            redfield_tensor (eigenbasis, -i included)
  pyqed/oqs.py:364-463            _redfield + rhs (RK4 on vec(rho), observables
                                  EXCLUDE t0, rholist back-transformed)
  pyqed/oqs.py:160-214            propagator(method='SOS'): eig(R), U1 E U1^-1
  pyqed/oqs.py:268-357            correlation_4op_3t (cube [i=tau3, j=tau2, k=tau1])
  pyqed/phys.py:1121-1137         transform(A, v) = v^+ A v
"""
import numpy as np
from scipy.linalg import eig, eigh, inv

from .lindblad import rk4


def dag(a):
    return np.conj(np.transpose(a))


def transform(A, v):
    return dag(v) @ A @ v                                   # phys.py:1121-1137


def op2sop(a, kind="commutator"):
    a = np.asarray(a)
    n = a.shape[-1]
    I = np.identity(n)
    if kind in ["commutator", "c", "-"]:
        return np.kron(a, I) - np.kron(I, a.T)
    if kind in ["left", "l"]:
        return np.kron(a, I)
    if kind in ["right", "r"]:
        return np.kron(I, a.T)
    if kind in ["anticommutator", "a", "+"]:
        return np.kron(a, I) + np.kron(I, a.T)
    raise ValueError("Error: superoperator {} does not exist.".format(kind))


def left(a):
    return np.kron(a, np.identity(a.shape[-1]))


def right(a):
    return np.kron(np.identity(a.shape[-1]), a.T)


def lindblad_dissipator(l):
    return np.kron(l, l.conj()) - 0.5 * op2sop(dag(l) @ l, "anticommutator")


def liouvillian(H, c_ops):
    L = -1j * op2sop(H)                                      # superoperator.py:29-58
    for c in (c_ops or []):
        L = L + lindblad_dissipator(np.asarray(c))
    return L


def redfield_tensor(H, a_ops, spectra):
    """oqs.py:519-570 -> (R dense (N^2, N^2), evecs)."""
    evals, evecs = eigh(np.asarray(H))
    W = np.real(evals[:, None] - evals[None, :])
    N = len(evals)
    C = []
    for s in spectra:
        c = np.zeros((N, N))
        for n in range(N):
            for m in range(N):
                c[n, m] = s(-W[n, m])
        C.append(c)
    A = [transform(np.asarray(a), evecs) for a in a_ops]
    L = [C[k] * A[k] for k in range(len(a_ops))]
    R = 0
    for k in range(len(a_ops)):
        R = R + op2sop(A[k]) @ (left(L[k]) - right(dag(L[k])))
    return -1j * op2sop(np.diag(evals)) - R, evecs


def redfield_evolve(R, rho0, evecs, Nt, dt, e_ops):
    """oqs._redfield with return_result=True: (observables (Nt, ne), rholist [Nt])."""
    N = rho0.shape[0]
    rho0 = transform(np.asarray(rho0), evecs)
    e_ops = [transform(np.asarray(e), evecs) for e in e_ops]
    rho = rho0.copy().flatten().astype(complex)
    obs = np.zeros((Nt, len(e_ops)), dtype=complex)
    rholist = []
    for k in range(Nt):
        rho = rk4(rho, lambda v, R: R @ v, dt, R)
        tmp = rho.reshape(N, N)
        rholist.append(transform(tmp, dag(evecs)))
        obs[k, :] = [(e @ tmp).diagonal().sum() for e in e_ops]
    return obs, rholist


def propagator_sos(R, t):
    """oqs.py:196-214: U[a, b, k] = sum_j U1[a,j] exp(lam_j t_k) U2[j,b]."""
    lam, U1 = eig(np.asarray(R))
    U2 = inv(U1)
    E = np.exp(lam[:, None] * np.asarray(t)[None, :])
    return np.einsum("aj,jk,jb->abk", U1, E, U2), lam, U1, U2


def correlation_4op_3t(R, rho0, oplist, signature, tau):
    """oqs.py:268-357 (G = -1j U from the SOS propagator)."""
    U, *_ = propagator_sos(R, tau)
    G = -1j * U
    a, b, c, d = [op2sop(op, s) for op, s in zip(oplist, signature)]
    N = np.asarray(rho0).shape[0]
    idm = np.identity(N).flatten()
    rho = d @ np.asarray(rho0).flatten()
    tmp = np.tensordot(G, rho, axes=((1), (0)))
    tmp = c @ tmp
    tmp = np.tensordot(G, tmp, axes=([1], [0]))
    tmp = np.tensordot(b, tmp, axes=([1], [0]))
    tmp = np.tensordot(G, tmp, axes=([1], [0]))
    return np.einsum("a,ab,bijk->ijk", idm, a, tmp)


def response_slice_eig(lam, U1, U2, a, b, c, d, rho0v, idm, t3, t2, t1):
    """Closed form of correlation_4op_3t at fixed tau2:
    S[t3, t1] = (-i)^3 sum_pq alpha_p e^{lam_p t3} M_pq beta_q e^{lam_q t1}."""
    alpha = (idm @ a @ U1)
    M = (U2 @ b @ U1) @ np.diag(np.exp(lam * t2)) @ (U2 @ c @ U1)
    beta = U2 @ (d @ rho0v)
    X = alpha[None, :] * np.exp(np.outer(t3, lam))
    Y = beta[None, :] * np.exp(np.outer(t1, lam))
    return (-1j) ** 3 * X @ M @ Y.T
