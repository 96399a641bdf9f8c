"""Result container (mirror of pyqed/mol.py:98-171)."""
from __future__ import annotations

import pickle

import numpy as np


class Result:
    """Same fields and `times` convention as pyqed.mol.Result (mol.py:98-119):
    times = t0 + arange(Nt//nout + 1) * dt * nout."""

    def __init__(self, description=None, psi0=None, rho0=None, dt=None, Nt=None, times=None, t0=0, nout=1):
        self.description = description
        self.dt = dt
        self.timesteps = self.nt = Nt
        self.observables = None
        self.rholist = None
        self.psilist = []
        self.psi = None
        self.rho0 = rho0
        self.psi0 = psi0
        self.nout = nout
        self.times = t0 + np.arange(Nt // nout + 1) * dt * nout
        return

    def expect(self):
        return self.observables

    def dump(self, fname):
        """Pickle the result (mol.py:146-162)."""
        with open(fname, "wb") as f:
            pickle.dump(self, f)

    def save(self, fname):
        self.dump(fname)


def load_result(fname):
    """Counterpart of mol.load_result (mol.py:173-179); loads a file this package wrote."""
    with open(fname, "rb") as f:
        return pickle.load(f)


# --------------------------------------------------------------------------- TDSE
def tdse_rk4(H, psi, dt, nsteps, save_every=0, e_ops=None):
    """Batched RK4 of dpsi/dt = -iH psi on the GPU (qd_tdse_rk4).  H [N,N], psi [B,N] (in place),
    e_ops [ne,N,N] (torch complex128, one device).  Returns (snap [B,nsave,N] | None,
    obs [B,nsave+1,ne] | None)."""
    import torch
    from . import _lib
    dev = psi.device
    _lib.ensure_device(dev)
    B, N = psi.shape
    ne = 0 if e_ops is None else e_ops.shape[0]
    nsave = nsteps // save_every if save_every > 0 else 0
    snap = torch.empty((B, nsave, N), dtype=torch.complex128, device=dev) if nsave else None
    obs = torch.empty((B, nsave + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    with torch.cuda.device(dev):
        rc = _lib.load().qd_tdse_rk4(_lib.ptr(H), _lib.ptr(psi), B, N, float(dt), int(nsteps), int(save_every),
                                     _lib.ptr(snap), _lib.ptr(e_ops), ne, _lib.ptr(obs), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_tdse_rk4")
    return snap, obs


def _quantum_dynamics(H, psi0, dt=0.001, Nt=1, e_ops=[], t0=0.0, nout=1, store_states=True, output='obs.dat'):
    """mol.py:1603-1691 (store_states=True): (Nt//nout - 1)*nout RK4 steps; psilist = [psi0] + the
    state after every nout steps; observables (Nt//nout, n_e) at those states."""
    import torch
    from ._util import default_device, stack_ops, to_numpy
    if e_ops is None:
        e_ops = []
    dev = default_device()
    Hn = to_numpy(H, np.complex128)
    N = Hn.shape[0]
    p0 = to_numpy(psi0, np.complex128).reshape(N)
    nblk = Nt // nout
    nsteps = max(nblk - 1, 0) * nout
    psi = torch.from_numpy(p0.copy()).to(dev).reshape(1, N)
    Ed = stack_ops(e_ops, N, dev)
    snap, obs = tdse_rk4(torch.from_numpy(np.ascontiguousarray(Hn)).to(dev), psi, dt, nsteps,
                         save_every=nout, e_ops=Ed)
    result = Result(dt=dt, Nt=Nt, psi0=psi0, t0=t0, nout=nout)
    result.psilist = [p0.copy()]
    if snap is not None:
        host = snap[0].cpu().numpy()
        result.psilist += [host[k] for k in range(host.shape[0])]
    observables = np.zeros((nblk, len(e_ops)), dtype=complex)
    if obs is not None:
        o = obs[0].cpu().numpy()
        observables[:o.shape[0]] = o[:nblk]
    result.observables = observables
    result.psi = psi[0].cpu().numpy()
    return result


class SESolver:
    """Drop-in for pyqed.mol.SESolver (mol.py:1369-1459), time-independent H."""

    def __init__(self, H=None):
        self.H = H
        self.groundstate = None

    def run(self, psi0=None, dt=0.01, Nt=1, e_ops=None, nout=1, t0=0.0, edip=None, pulse=None, use_sparse=True):
        if psi0 is None:
            psi0 = self.groundstate
        if pulse is not None:
            raise NotImplementedError("laser-driven TDSE (pulse=...) is not on the GPU path yet")
        return _quantum_dynamics(self.H, psi0, dt=dt, Nt=Nt, e_ops=e_ops, nout=nout, t0=t0)


class Mol:
    """Subset of pyqed.mol.Mol (mol.py:184-957) on the hot path: container, run, photon_echo."""

    def __init__(self, H, edip=None, lowering=None, edip_rms=None, gamma=None):
        self.H = H
        self.h = H
        Hd = np.asarray(H.toarray() if hasattr(H, "toarray") else H)
        self.E = np.diag(Hd) if np.count_nonzero(Hd - np.diag(np.diagonal(Hd))) == 0 else None
        self.nonhermH = None
        self._edip = edip
        self.dip = self.edip = edip
        if lowering is not None:
            self.lowering = lowering
            self.raising = np.conj(np.transpose(lowering))
        self.nstates = self.dim = self.size = H.shape[0]
        self.gamma = gamma
        self.mdip = None
        self.dephasing = 0.
        self._edip_rms = edip_rms

    @property
    def edip(self):
        return self._edip

    @edip.setter
    def edip(self, edip):
        self._edip = edip

    def set_dipole(self, dip):
        self.dip = dip

    def set_edip(self, edip, pol=None):
        self.edip_rms = edip

    @property
    def edip_rms(self):
        if self._edip_rms is None:
            self._edip_rms = np.sqrt(np.abs(self.edip[:, :, 0]) ** 2 + np.abs(self.edip[:, :, 1]) ** 2 +
                                     np.abs(self.edip[:, :, 2]) ** 2)
        return self._edip_rms

    @edip_rms.setter
    def edip_rms(self, edip):
        self._edip_rms = edip

    def run(self, psi0=None, dt=0.01, e_ops=None, nt=1, nout=1, t0=0.0, edip=None, pulse=None):
        """mol.py:628-674 (time-independent H) -> _quantum_dynamics."""
        if psi0 is None:
            raise ValueError("Please specify initial wavefunction psi0.")
        if pulse is not None:
            raise NotImplementedError("laser-driven dynamics (pulse=...) is not on the GPU path yet")
        return _quantum_dynamics(self.H, psi0, dt=dt, Nt=nt, e_ops=e_ops, nout=nout, t0=t0)

    def eigvals(self):
        """mol.py:459-463."""
        H = np.asarray(self.H.toarray() if hasattr(self.H, "toarray") else self.H)
        if np.count_nonzero(H - np.diag(np.diagonal(H))) == 0:
            return np.diagonal(H)
        return np.linalg.eigvals(H)

    def photon_echo(self, pump, probe, t2=0.0, **kwargs):
        """mol.py:804-829 -> sos.photon_echo (GPU)."""
        from . import sos
        return sos.photon_echo(self, pump=pump, probe=probe, t2=t2, **kwargs)
