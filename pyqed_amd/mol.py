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


def tdse_driven_rk4(H0, Hd, fvals, psi, dt, nout, e_ops=None):
    """Laser-driven batched RK4 on the GPU (qd_tdse_driven_rk4): block k of `nout` steps uses
    H0 - sum_d fvals[k, d] Hd[d].  H0 [N,N], Hd [nd,N,N] | None, fvals host complex [nblocks, nd],
    psi [B,N] (in place), e_ops [ne,N,N] | None.  Returns (snap [B,nblocks,N], obs [B,nblocks+1,ne] | None)."""
    import torch
    from . import _lib
    dev = psi.device
    _lib.ensure_device(dev)
    B, N = psi.shape
    fv = np.ascontiguousarray(np.asarray(fvals, dtype=np.complex128))
    nblocks = fv.shape[0]
    nd = 0 if Hd is None else Hd.shape[0]
    ne = 0 if e_ops is None else e_ops.shape[0]
    snap = torch.empty((B, nblocks, N), dtype=torch.complex128, device=dev) if nblocks else None
    obs = torch.empty((B, nblocks + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    with torch.cuda.device(dev):
        rc = _lib.load().qd_tdse_driven_rk4(_lib.ptr(H0), _lib.ptr(Hd), nd, fv.ctypes.data if fv.size else None,
                                            _lib.ptr(psi), B, N, float(dt), nblocks, int(nout), _lib.ptr(snap),
                                            _lib.ptr(e_ops), ne, _lib.ptr(obs), _lib.stream_ptr(dev))
        torch.cuda.current_stream(dev).synchronize()  # fvals is a host buffer read asynchronously
    _lib.check(rc, "qd_tdse_driven_rk4")
    return snap, obs


def driven_dynamics(H, psi0, dt=0.01, Nt=1, e_ops=None, nout=1, t0=0.0, return_result=True, use_sparse=True):
    """mol.py:1862-1958.  H = [H0, [Hd_1, f_1], [Hd_2, f_2], ...] with H(t) = H0 - sum_d f_d(t) Hd_d,
    evaluated once per block of nout steps at the block's start time (calcH(t), t advanced by
    dt*nout after each block).  return_result=True: Nt//nout - 1 blocks; psilist = [psi0] + the
    state after each block (csr columns when use_sparse, as the reference's sparse psi);
    observables (Nt//nout, n_e) including t0; result.psi = psit [nstates, Nt//nout].
    return_result=False: int(Nt/nout) blocks written to psi.dat / obs.dat (t after the block,
    then the values; dense formatting)."""
    import torch
    from scipy.sparse import csr_matrix
    from ._util import default_device, stack_ops, to_numpy
    if e_ops is None:
        e_ops = []
    dev = default_device()
    H0 = to_numpy(H[0], np.complex128)
    N = H0.shape[0]
    drives = H[1:]
    Hd = [to_numpy(h[0], np.complex128) for h in drives]
    p0 = to_numpy(psi0, np.complex128).reshape(N)
    nblocks = max(Nt // nout - 1, 0) if return_result else int(Nt / nout)
    fvals = np.array([[complex(f(t0 + k * dt * nout)) for (_, f) in drives] for k in range(nblocks)],
                     dtype=np.complex128).reshape(nblocks, len(drives))
    psi = torch.from_numpy(p0.copy()).to(dev).reshape(1, N)
    Hdt = torch.from_numpy(np.ascontiguousarray(np.array(Hd))).to(dev) if Hd else None
    Ed = stack_ops(e_ops, N, dev)
    snap, obs = tdse_driven_rk4(torch.from_numpy(np.ascontiguousarray(H0)).to(dev), Hdt, fvals, psi, dt, nout,
                                e_ops=Ed)
    states = snap[0].cpu().numpy() if snap is not None else np.zeros((0, N), complex)
    o = obs[0].cpu().numpy() if obs is not None else np.zeros((nblocks + 1, 0), complex)
    if not return_result:
        with open("psi.dat", "w") as f_dm, open("obs.dat", "w") as f_obs:
            fmt = "{} " * (len(e_ops) + 1) + "\n"
            fmt_dm = "{} " * (N + 1) + "\n"
            for k in range(nblocks):
                t = t0 + (k + 1) * dt * nout
                f_dm.write(fmt_dm.format(t, *states[k]))
                f_obs.write(fmt.format(t, *o[k + 1]))
        return None
    result = Result(dt=dt, Nt=Nt, psi0=psi0, t0=t0, nout=nout)
    nrec = Nt // nout
    observables = np.zeros((nrec, len(e_ops)), dtype=complex)
    observables[:nblocks + 1] = o[:nrec]
    psit = np.zeros((N, nrec), dtype=complex)
    psit[:, 0] = p0
    psilist = [np.array(psi0, copy=True)]
    for k in range(nblocks):
        psit[:, k + 1] = states[k]
        psilist.append(csr_matrix(states[k].reshape(N, 1)) if use_sparse else states[k].copy())
    result.psilist = psilist
    result.psi = psit
    result.observables = observables
    return result


def _driven_dynamics(H, psi0, edip, E, dt=0.001, Nt=1, e_ops=None, nout=1, t0=0.0, sparse=True):
    """mol.py:1772-1859: full vector dipole edip [N, N, 3] in a polarized field E(t) -> 3-vector,
    H(t) = H - einsum('ija, a -> ij', edip, E(t)), held for each block of nout RK4 steps at the block's start time
    (t advanced by dt*nout after a block); Nt//nout - 1 blocks.  On the GPU this is qd_tdse_driven_rk4 with the
    three dipole components as drives.  As the reference: result.psilist holds only the states after each block
    (csr columns), observables (Nt//nout, n_e) include t0, result.psi = psit [nstates, Nt//nout].  The reference's
    sparse=False branch never defines psi and raises; only the sparse (default) arithmetic exists."""
    import torch
    from scipy.sparse import csr_matrix
    from ._util import default_device, stack_ops, to_numpy
    if not sparse:
        raise NotImplementedError("_driven_dynamics(sparse=False): the reference's dense branch never sets psi")
    if e_ops is None:
        e_ops = []
    dev = default_device()
    H0 = to_numpy(H, np.complex128)
    N = H0.shape[0]
    ed = np.asarray(to_numpy(edip, np.complex128))
    if ed.shape[:2] != (N, N) or ed.ndim != 3:
        raise ValueError(f"edip must be [N, N, ncomp] with N = {N}, got {ed.shape}")
    nc = ed.shape[2]
    p0 = to_numpy(psi0, np.complex128).reshape(N)
    nblocks = max(Nt // nout - 1, 0)
    fvals = np.zeros((nblocks, nc), dtype=np.complex128)
    for k in range(nblocks):
        fvals[k] = np.asarray(E(t0 + k * dt * nout), dtype=np.complex128).reshape(nc)
    psi = torch.from_numpy(p0.copy()).to(dev).reshape(1, N)
    Hdt = torch.from_numpy(np.ascontiguousarray(np.moveaxis(ed, 2, 0))).to(dev)
    Ed = stack_ops(e_ops, N, dev)
    snap, obs = tdse_driven_rk4(torch.from_numpy(np.ascontiguousarray(H0)).to(dev), Hdt, fvals, psi, dt, nout,
                                e_ops=Ed)
    states = snap[0].cpu().numpy() if snap is not None else np.zeros((0, N), complex)
    nrec = Nt // nout
    result = Result(dt=dt, Nt=Nt, psi0=psi0, t0=t0, nout=nout)
    observables = np.zeros((nrec, len(e_ops)), dtype=complex)
    if obs is not None:
        o = obs[0].cpu().numpy()
        observables[:nblocks + 1] = o[:nrec]
    psit = np.zeros((N, nrec), dtype=complex)
    if nrec:
        psit[:, 0] = p0
    for k in range(nblocks):
        psit[:, k + 1] = states[k]
    result.psilist = [csr_matrix(states[k].reshape(N, 1)) for k in range(nblocks)]
    result.psi = psit
    result.observables = observables
    return result


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
        """mol.py:1392-1459: time-independent H -> _quantum_dynamics; with a pulse (or a list of
        pulses with a list of dipoles) -> driven_dynamics, H(t) = H - sum_i f_i(t) edip_i; a full [N, N, 3]
        dipole with a single pulse -> _driven_dynamics with the pulse's vector field pulse.E(t)."""
        if psi0 is None:
            psi0 = self.groundstate
        if pulse is None:
            return _quantum_dynamics(self.H, psi0, dt=dt, Nt=Nt, e_ops=e_ops, nout=nout, t0=t0)
        if edip is None:
            raise ValueError('Electric dipole must be provided for laser-driven dynamics.')
        if isinstance(pulse, list):
            H = [self.H] + [[edip[i], pulse[i].efield] for i in range(len(pulse))]
            return driven_dynamics(H=H, psi0=psi0, dt=dt, Nt=Nt, e_ops=e_ops, nout=nout, t0=t0)
        if np.ndim(edip) == 2:
            return driven_dynamics(H=[self.H, [edip, pulse.efield]], psi0=psi0, dt=dt, Nt=Nt, e_ops=e_ops,
                                   nout=nout, t0=t0, use_sparse=use_sparse)
        if np.ndim(edip) == 3:
            return _driven_dynamics(H=self.H, psi0=psi0, edip=edip, E=pulse.E, dt=dt, Nt=Nt, e_ops=e_ops, nout=nout,
                                    t0=t0)
        return None


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
        """mol.py:628-674: _quantum_dynamics, or driven_dynamics with H(t) = H - f(t) edip for a pulse
        (self.edip is used, as in the reference; a list of pulses pairs with a list of dipoles)."""
        if psi0 is None:
            raise ValueError("Please specify initial wavefunction psi0.")
        if pulse is None:
            return _quantum_dynamics(self.H, psi0, dt=dt, Nt=nt, e_ops=e_ops, nout=nout, t0=t0)
        edip = self.edip
        if isinstance(pulse, list):
            H = [self.H] + [[edip[i], pulse[i].efield] for i in range(len(pulse))]
        else:
            H = [self.H, [edip, pulse.efield]]
        return driven_dynamics(H, psi0, dt=dt, Nt=nt, e_ops=e_ops, nout=nout, t0=t0)

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
