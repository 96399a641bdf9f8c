"""Split-operator wavepacket dynamics on MI355X (drop-in for pyqed/wpd.py SPO, SPO2).

Setup (grids, exp_K, per-point exp(-i V dt/2)) is host-side like the reference's
build (wpd.py:217-223, 496-625), vectorised; every propagation step runs in
libqdyn (qd_spo1d_run / qd_spo2_run).
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.fftpack import fftfreq

from . import _lib
from ._util import default_device
from .mol import Result

pi = np.pi


def interval(x):
    return x[1] - x[0]


def meshgrid(*args):
    return np.meshgrid(*args, indexing="ij")


class ResultSPO2(Result):
    """wpd.py:57-178 (result container with grid and population helpers)."""

    def __init__(self, **args):
        super().__init__(**args)
        self.x = None
        self.y = None
        self.population = None
        self.xAve = None
        self.nstates = self.psi0.shape[-1]

    def get_population(self, fname=None, plot=False):
        dx = interval(self.x)
        dy = interval(self.y)
        p = np.zeros((len(self.psilist), self.nstates))
        for n in range(self.nstates):
            p[:, n] = [np.vdot(psi[:, :, n], psi[:, :, n]).real * dx * dy for psi in self.psilist]
        self.population = p
        if fname is not None:
            np.savez(fname, p)
        return p

    def position(self, plot=False, fname=None):
        x, y = self.x, self.y
        dx, dy = interval(x), interval(y)
        xAve = [np.einsum('ijn, i, ijn', psi.conj(), x, psi) * dx * dy for psi in self.psilist]
        yAve = [np.einsum('ijn, j, ijn', psi.conj(), y, psi) * dx * dy for psi in self.psilist]
        self.xAve = [xAve, yAve]
        return xAve, yAve


def _dev_c128(a, dev):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)


class SPO:
    """Drop-in for pyqed.wpd.SPO (wpd.py:191-322): 1D, single surface."""

    def __init__(self, x, mass=1, nstates=1):
        self.x = x
        self.dx = interval(x)
        self.nx = len(x)
        self.k = 2. * pi * fftfreq(self.nx, self.dx)
        self.nstates = nstates
        self.V = None
        self.mass = mass
        self._exp_K = None
        self._exp_V = None
        self._exp_V_half = None

    def set_grid(self, xmin=-1, xmax=1, npts=32):
        self.x = np.linspace(xmin, xmax, npts)

    def set_potential(self, potential):
        self.V = potential(self.x)
        return

    def build(self, dt):
        """wpd.py:217-223."""
        self._exp_V = np.exp(-1j * self.V * dt)
        self._exp_V_half = np.exp(-1j * self.V * dt / 2.)
        m = self.mass
        k = self.k
        self._exp_K = np.exp(-0.5j / m * (k * k) * dt)

    def run(self, psi0, dt, nt=1, t0=0, nout=1):
        """wpd.py:225-273 step structure; psilist has nt//nout - 1 entries, r.psi the final state.
        psi0 may also be a batch [B, nx] (extension): B wavepackets propagated together."""
        self.build(dt)
        dev = default_device()
        _lib.ensure_device(dev)
        p0 = np.asarray(psi0)
        batched = p0.ndim == 2
        psi = _dev_c128(p0.reshape(-1, self.nx), dev)
        B = psi.shape[0]
        nsnap = max(nt // nout - 1, 0)
        snap = torch.empty((B, nsnap, self.nx), dtype=torch.complex128, device=dev) if nsnap else None
        eV, eVh, eK = (_dev_c128(a, dev) for a in (self._exp_V, self._exp_V_half, self._exp_K))
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo1d_run(psi.data_ptr(), eV.data_ptr(), eVh.data_ptr(), eK.data_ptr(), self.nx, B,
                                          int(nt), int(nout), _lib.ptr(snap), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo1d_run")
        r = Result(psi0=psi0, dt=dt, Nt=nt, t0=t0, nout=nout)
        snaps = snap.cpu().numpy() if snap is not None else np.zeros((B, 0, self.nx), complex)
        out = psi.cpu().numpy()
        if batched:
            r.psilist = [snaps[:, k] for k in range(nsnap)]
            r.psi = out
        else:
            r.psilist = [snaps[0, k] for k in range(nsnap)]
            r.psi = out[0]
        return r


class SPO2:
    """Drop-in for pyqed.wpd.SPO2 (wpd.py:379-887), linear coordinates."""

    def __init__(self, x, y, mass=None, nstates=2, coords='linear', G=None, abc=False):
        self.x = x
        self.y = y
        self.X, self.Y = meshgrid(x, y)
        self.nx = len(x)
        self.ny = len(y)
        self.dx = interval(x)
        self.dy = interval(y)
        if mass is None:
            mass = [1, 1]
        self.mass = self.masses = mass
        self.kx = None
        self.ky = None
        self.apes = None
        self.dim = 2
        self.exp_V = None
        self.exp_V_half = None
        self.exp_K = None
        self.v = self.V = None
        self.G = G
        self.nstates = self.ns = nstates
        self.coords = coords
        self.abc = abc
        self.d2a = None
        self.a2d = None
        self.psilist = None

    def set_grid(self, x, y):
        self.x = x
        self.y = y

    def set_masses(self, mass):
        self.mass = mass

    def setG(self, G):
        self.G = G

    def set_DPES(self, surfaces, diabatic_couplings, eta=None):
        """wpd.py:436-484 (real potential array, as the reference: complex couplings lose Im)."""
        nx, ny, ns = self.nx, self.ny, self.ns
        v = np.zeros([nx, ny, ns, ns])
        for a in range(self.ns):
            v[:, :, a, a] = surfaces[a]
        for dc in diabatic_couplings:
            a, b = dc[0][:]
            v[:, :, a, b] = np.real(dc[1])
            v[:, :, b, a] = v[:, :, a, b].conj()
        if self.abc:
            v = v.astype(complex)
            for n in range(self.ns):
                v[:, :, n, n] = -1j * eta * (self.X - 9.) ** 2
        self.v = v
        return v

    def set_dpes(self, v):
        self.V = self.v = v
        return self

    def build(self, dt, inertia=None):
        """wpd.py:496-625: exp_K on the 'ij' k-grid and per-point U e^{-i w dt/2} U^+
        (vectorised eigh over the grid instead of the reference's Python loop)."""
        if self.coords != 'linear':
            raise NotImplementedError("only linear coordinates run on the GPU path")
        nx, ny = self.nx, self.ny
        self.kx = 2. * np.pi * fftfreq(nx, interval(self.x))
        self.ky = 2. * np.pi * fftfreq(ny, interval(self.y))
        mx, my = self.masses
        Kx, Ky = meshgrid(self.kx, self.ky)
        self.exp_K = np.exp(-1j * (Kx ** 2 / 2. / mx + Ky ** 2 / 2. / my) * dt)
        if self.v is None:
            raise ValueError('The diabatic PES is not specified.')
        v = self.v
        w, u = np.linalg.eigh(v)  # ascending eigenvalues per point (phys.sort order)
        ud = np.conj(np.swapaxes(u, -1, -2))
        self.exp_V = (u * np.exp(-1j * w * dt)[..., None, :]) @ ud
        self.exp_V_half = (u * np.exp(-1j * w * dt / 2)[..., None, :]) @ ud
        self.d2a = u
        if not np.iscomplexobj(v):
            self.apes = w

    def run(self, psi0, e_ops=[], dt=0.01, nt=1, t0=0., nout=1, return_states=True):
        """wpd.py:692-758 with return_states=True semantics: psilist = [psi0] + the state after
        every nout Strang steps (nt//nout*nout steps in total); r.psi is the final state."""
        self.build(dt=dt)
        dev = default_device()
        _lib.ensure_device(dev)
        nsteps = (nt // nout) * nout
        psi = _dev_c128(psi0, dev)
        nsnap = nt // nout
        snap = torch.empty((nsnap, self.nx, self.ny, self.ns), dtype=torch.complex128, device=dev) \
            if (nsnap and return_states) else None
        eVh = _dev_c128(self.exp_V_half, dev)
        eK = _dev_c128(self.exp_K, dev)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo2_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), self.nx, self.ny, self.ns,
                                         int(nsteps), int(nout), _lib.ptr(snap), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo2_run")
        r = ResultSPO2(dt=dt, psi0=psi0, Nt=nt, t0=t0, nout=nout)
        r.x = self.x
        r.y = self.y
        psilist = [psi0]
        if snap is not None:
            host = snap.cpu().numpy()
            psilist += [host[k] for k in range(nsnap)]
        r.psilist = psilist
        r.psi = psi.cpu().numpy()
        return r


class SPO3:
    """Drop-in for pyqed.wpd.SPO3 (wpd.py:1105-1432), linear coordinates."""

    def __init__(self, x, y, z, masses, nstates=2, coords='linear', G=None, abc=False):
        self.x, self.y, self.z = x, y, z
        self.X, self.Y, self.Z = meshgrid(x, y, z)
        self.nx, self.ny, self.nz = len(x), len(y), len(z)
        self.dx, self.dy, self.dz = interval(x), interval(y), interval(z)
        self.masses = masses
        self.kx = self.ky = self.kz = None
        self.dim = 3
        self.exp_V = self.exp_V_half = self.exp_K = None
        self.V = None
        self.G = G
        self.nstates = nstates
        self.coords = coords
        self.abc = abc

    def set_grid(self, x, y, z):
        self.x, self.y, self.z = x, y, z

    def set_masses(self, masses):
        self.masses = masses

    def setG(self, G):
        self.G = G

    def set_DPES(self, surfaces, diabatic_couplings, eta=None):
        """wpd.py:1163-1200 (real array; couplings written symmetrically)."""
        ns = self.nstates
        v = np.zeros([self.nx, self.ny, self.nz, ns, ns])
        for a in range(ns):
            v[:, :, :, a, a] = surfaces[a]
        for dc in diabatic_couplings:
            a, b = dc[0][:]
            v[:, :, :, a, b] = v[:, :, :, b, a] = np.real(dc[1])
        self.V = v
        return v

    def build(self, dt, inertia=None):
        """wpd.py:1210-1340 (linear): exp_K on the 'ij' grid, exp(-i V dt/2) per point."""
        if self.coords != 'linear':
            raise NotImplementedError("only linear coordinates run on the GPU path")
        self.kx = 2. * np.pi * fftfreq(self.nx, self.dx)
        self.ky = 2. * np.pi * fftfreq(self.ny, self.dy)
        self.kz = 2. * np.pi * fftfreq(self.nz, self.dz)
        mx, my, mz = self.masses
        Kx, Ky, Kz = meshgrid(self.kx, self.ky, self.kz)
        self.exp_K = np.exp(-1j * (Kx ** 2 / 2. / mx + Ky ** 2 / 2. / my + Kz ** 2 / 2. / mz) * dt)
        if self.V is None:
            raise ValueError('The diabatic PES is not specified.')
        w, u = np.linalg.eigh(self.V)
        ud = np.conj(np.swapaxes(u, -1, -2))
        self.exp_V = (u * np.exp(-1j * w * dt)[..., None, :]) @ ud
        self.exp_V_half = (u * np.exp(-1j * w * dt / 2)[..., None, :]) @ ud

    def run(self, psi0, e_ops=[], dt=0.01, nt=1, t0=0., nout=1, return_states=True):
        """wpd.py:1349-1411: nt//nout*nout Strang steps; psilist = state after every nout steps
        (psi0 NOT included, as the reference); r.psi the final state."""
        self.build(dt=dt)
        dev = default_device()
        _lib.ensure_device(dev)
        nsteps = (nt // nout) * nout
        nsnap = nt // nout
        psi = _dev_c128(psi0, dev)
        shape = (self.nx, self.ny, self.nz, self.nstates)
        snap = torch.empty((nsnap,) + shape, dtype=torch.complex128, device=dev) if nsnap else None
        eVh = _dev_c128(self.exp_V_half, dev)
        eK = _dev_c128(self.exp_K, dev)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo3_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), self.nx, self.ny, self.nz,
                                         self.nstates, int(nsteps), int(nout), _lib.ptr(snap), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo3_run")
        r = Result(dt=dt, psi0=psi0, Nt=nt, t0=t0, nout=nout)
        if snap is not None:
            host = snap.cpu().numpy()
            r.psilist = [host[k] for k in range(nsnap)]
        r.psi = psi.cpu().numpy()
        return r
