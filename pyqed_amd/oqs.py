"""Open-quantum-system solvers on MI355X (drop-in for pyqed/oqs.py).

Class surface mirrors the reference:
  LindbladSolver(H, c_ops, e_ops).run(rho0, dt, Nt, t0, e_ops, return_result)
      -> Result  (pyqed/oqs.py:1114-1187, loop _lindblad oqs.py:1596-1696)

All propagation runs in libqdyn (HIP).  Host code only converts operators and
packages results.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._util import default_device, issparse, stack_ops, to_device, to_numpy
from .mol import Result

try:
    from scipy.sparse import csr_matrix
except Exception:  # pragma: no cover
    csr_matrix = None


# --------------------------------------------------------------------------- functional
def lindblad_rk4(H: torch.Tensor, c_ops: torch.Tensor | None, rho: torch.Tensor, dt: float, nsteps: int,
                 e_ops: torch.Tensor | None = None, save_every: int = 0, stream=None):
    """Propagate a batch of density matrices in place with RK4 on the GPU.

    H [N,N], c_ops [nc,N,N] or None, rho [B,N,N] (or [N,N]), e_ops [ne,N,N] or None
    (all complex128 on one cuda device).  Returns (obs [B,nsteps+1,ne] | None,
    snap [B,nsteps//save_every,N,N] | None).  Reference RHS: oqs.py:697-714.
    """
    squeeze = rho.dim() == 2
    if squeeze:
        rho = rho.unsqueeze(0)
    if rho.dim() != 3 or rho.shape[-1] != rho.shape[-2]:
        raise ValueError(f"rho must be [B,N,N] or [N,N], got {tuple(rho.shape)}")
    B, N = rho.shape[0], rho.shape[-1]
    dev = rho.device
    _lib.ensure_device(dev)
    for name, t in (("H", H), ("rho", rho), ("c_ops", c_ops), ("e_ops", e_ops)):
        if t is not None and (t.dtype != torch.complex128 or t.device != dev or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous complex128 tensor on {dev}")
    if tuple(H.shape) != (N, N):
        raise ValueError(f"H has shape {tuple(H.shape)}, expected {(N, N)}")
    for name, t in (("c_ops", c_ops), ("e_ops", e_ops)):
        if t is not None and (t.dim() != 3 or tuple(t.shape[1:]) != (N, N)):
            raise ValueError(f"{name} must be [k,{N},{N}], got {tuple(t.shape)}")
    nc = 0 if c_ops is None else c_ops.shape[0]
    ne = 0 if e_ops is None else e_ops.shape[0]
    obs = torch.empty((B, nsteps + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    nsave = nsteps // save_every if save_every > 0 else 0
    snap = torch.empty((B, nsave, N, N), dtype=torch.complex128, device=dev) if nsave else None
    st = stream if stream is not None else _lib.stream_ptr(dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_lindblad_rk4(_lib.ptr(H), _lib.ptr(c_ops), nc, _lib.ptr(rho), B, N, float(dt),
                                         int(nsteps), _lib.ptr(e_ops), ne, _lib.ptr(obs), _lib.ptr(snap),
                                         int(save_every if nsave else 0), st)
    _lib.check(rc, "qd_lindblad_rk4")
    return obs, snap


# --------------------------------------------------------------------------- solvers
class LindbladSolver:
    """Drop-in for pyqed.oqs.LindbladSolver (oqs.py:1114)."""

    def __init__(self, H=None, c_ops=None, e_ops=None):
        self.c_ops = c_ops
        self.e_ops = e_ops
        self.H = H
        return

    def set_c_ops(self, c_ops):
        self.c_ops = c_ops

    def set_e_ops(self, e_ops):
        self.e_ops = e_ops

    def setH(self, H):
        self.H = H

    def configure(self, c_ops, e_ops):
        self.c_ops = c_ops
        self.e_ops = e_ops

    def liouvillian(self):
        from . import superoperator as superop
        return superop.liouvillian(self.H, self.c_ops)

    def run(self, rho0, dt, Nt, t0=0., e_ops=None, return_result=True, return_states=True):
        """Propagate rho0 for Nt RK4 steps (oqs.py:1149-1187).

        Returns a Result with observables (Nt+1, n_e) including t0 and rholist of Nt
        csr matrices excluding rho0, as oqs._lindblad (oqs.py:1676-1696).
        `return_states=False` (extension) skips the per-step snapshots.
        """
        if isinstance(self.H, list):
            raise NotImplementedError("time-dependent H ([H0, [f, H1]]) is not on the GPU path yet")
        return _lindblad(self.H, rho0, c_ops=self.c_ops, e_ops=e_ops, Nt=Nt, dt=dt,
                         return_states=return_states)


def _lindblad(H, rho0, c_ops, e_ops=None, Nt=1, t0=0, dt=0.005, return_result=True, return_states=True):
    """GPU restatement of oqs._lindblad (oqs.py:1596-1696)."""
    if e_ops is None:
        e_ops = []
    if c_ops is None:
        c_ops = []
    dev = default_device()
    Hn = to_numpy(H, np.complex128)
    N = Hn.shape[0]
    Hd = torch.from_numpy(np.ascontiguousarray(Hn)).to(dev)
    Cd = stack_ops(c_ops, N, dev)
    Ed = stack_ops(e_ops, N, dev)
    rho = to_device(rho0, dev).reshape(1, N, N).contiguous()
    obs, snap = lindblad_rk4(Hd, Cd, rho, dt, Nt, Ed, save_every=1 if return_states else 0)
    torch.cuda.synchronize(dev)

    result = Result(dt=dt, Nt=Nt, rho0=rho0)
    if obs is not None:
        result.observables = obs[0].cpu().numpy()
    else:
        result.observables = np.zeros((Nt + 1, 0), dtype=complex)
    if return_states and snap is not None:
        host = snap[0].cpu().numpy()
        result.rholist = [csr_matrix(host[k]) for k in range(Nt)]
    else:
        result.rholist = []
    result.rho = rho[0].cpu().numpy()
    return result
