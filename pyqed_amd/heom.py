"""Single-exponential HEOM chain (drop-in for pyqed/HEOM/heom.py HEOMSolver, RK4).

The chain  d rho_n = -i[H, rho_n] - [Q, rho_{n+1}] - n gamma rho_n
                     + n (Re D0 [Q, rho_{n-1}] + i Im D0 {Q, rho_{n-1}}),
D0 = lambda (2T - i gamma), ADO nado-1 frozen at zero (HEOM/heom.py:275-347), is a
K = 1 hierarchy: it runs on the DEOM stencil kernel (qd_deom_rk4) with chain tables.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._util import default_device, to_numpy


def chain_tables(nado, gamma, D0):
    """Tables of the nado-1 live ADOs (the frozen last ADO is identically zero, so dropping it
    leaves every update unchanged)."""
    nmax = max(nado - 1, 1)
    n = np.arange(nmax)
    minus = np.where(n >= 1, n - 1, -1).astype(np.int32)[:, None]
    plus = np.where(n + 1 <= nado - 2, n + 1, -1).astype(np.int32)[:, None]
    coef = np.zeros((nmax, 1, 3), dtype=complex)
    coef[:, 0, 0] = n * (D0.real + 1j * D0.imag)      # Q rho_{n-1}
    coef[:, 0, 1] = n * (-D0.real + 1j * D0.imag)     # rho_{n-1} Q
    coef[:, 0, 2] = -1.0                              # -[Q, rho_{n+1}]
    damp = (-n * gamma).astype(complex)
    return nmax, minus, plus, coef, damp


def run_chain_rk4(H, Q, rho0, e_ops, gamma, D0, nado, dt, nt):
    """observables (len(e_ops), nt): Tr(e rho_0) after every step (t0 excluded)."""
    dev = default_device()
    _lib.ensure_device(dev)
    H = to_numpy(H, complex)
    ns = H.shape[0]
    nmax, minus, plus, coef, damp = chain_tables(nado, gamma, D0)
    c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)
    ados = torch.zeros((1, nmax, ns, ns), dtype=torch.complex128, device=dev)
    ados[0, 0] = c128(to_numpy(rho0, complex))
    E = c128(np.array([to_numpy(e, complex) for e in e_ops]).reshape(-1, ns, ns)) if e_ops else None
    ne = len(e_ops)
    obs = torch.empty((1, nt + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    rho_sys = torch.empty((1, nt + 1, ns, ns), dtype=torch.complex128, device=dev)
    t = (i32(minus), i32(plus), c128(coef), c128(damp), i32(np.zeros(1)))
    Ht, Qt = c128(H), c128(to_numpy(Q, complex).reshape(1, ns, ns))
    with torch.cuda.device(dev):
        rc = _lib.load().qd_deom_rk4(ados.data_ptr(), 1, nmax, 1, ns, t[0].data_ptr(), t[1].data_ptr(),
                                     t[2].data_ptr(), t[3].data_ptr(), t[4].data_ptr(), 1, Ht.data_ptr(), None,
                                     Qt.data_ptr(), None, None, None, float(dt), int(nt), rho_sys.data_ptr(),
                                     _lib.ptr(E), ne, _lib.ptr(obs), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_deom_rk4 (HEOM chain)")
    if not ne:
        return np.zeros((0, nt), dtype=complex)
    return obs[0, 1:].T.cpu().numpy()


class HEOMSolver:
    """Drop-in for pyqed.HEOM.heom.HEOMSolver (HEOM/heom.py:161-273)."""

    def __init__(self, H=None, c_ops=None, e_ops=None):
        self.c_ops = c_ops
        self.e_ops = e_ops
        self.H = H

    def set_c_ops(self, c_ops):
        self.c_ops = c_ops

    def set_e_ops(self, e_ops):
        self.e_ops = e_ops

    def setH(self, H):
        self.H = H

    def configure(self, c_ops, e_ops):
        self.c_ops = c_ops
        self.e_ops = e_ops

    def run(self, rho0, dt, nt, temperature, cutoff, reorganization, nado):
        """HEOM/heom.py:195-199 -> _heom (RK4): D0 = reorg (2T - i gamma)."""
        return _heom(self.H, rho0, self.c_ops, self.e_ops, temperature, cutoff, reorganization, nado, dt, nt)


def _heom(H, rho0, c_ops, e_ops, temperature, cutoff, reorganization, nado, dt, nt, fname=None,
          return_result=True):
    gamma, T, reorg = cutoff, temperature, reorganization
    D0 = reorg * (2. * T - 1j * gamma)
    return run_chain_rk4(H, c_ops[0], rho0, list(e_ops or []), gamma, D0, nado, dt, nt)
