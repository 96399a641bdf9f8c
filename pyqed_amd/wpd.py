"""Split-operator wavepacket dynamics on MI355X (drop-in for pyqed/wpd.py SPO, SPO2).

Setup: grids and exp_K on the host like the reference's build (wpd.py:217-223, 496-625);
the per-point propagators exp(-i V dt), exp(-i V dt/2) on the device (qd_spo_expv: closed form for
ns <= 2, a matrix exponential up to ns = 256).
Every propagation step runs in libqdyn (qd_spo1d_run / qd_spo2_run_ex / qd_spo3_run).
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.fftpack import fftfreq

from . import _lib
from ._util import default_device
from .mol import Result

DEVICE_EXPM_MAX_NS = 1024   # qd_spo_expv / qd_spo_expm: work matrices in LDS to ns = 50, in device scratch above

pi = np.pi



def _check_finite(v):
    """The reference builds the point propagators with eigh / eig (wpd.py:585-623, 960-985), which raise LinAlgError on
    inf / NaN potentials; the device exponential would only produce NaN, so the same error is raised up front."""
    if not np.all(np.isfinite(v)):
        raise np.linalg.LinAlgError("Array must not contain infs or NaNs")

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
        xAve = np.real_if_close(xAve)  # wpd.py:150-151
        yAve = np.real_if_close(yAve)
        self.xAve = [xAve, yAve]
        np.savez('xAve', xAve, yAve)  # wpd.py:159 writes xAve.npz in the CWD
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


class _PointPropagators:
    """exp_V / exp_V_half of a Hermitian diabatic potential, built on the device.

    The reference's build (wpd.py:585-623, SPO3 :1290-1330) loops over grid points calling eigh and
    forming U e^{-i w tau} U^+.  qd_spo_expv evaluates the same point propagators on the GPU (LAPACK
    conventions: lower triangle, real diagonal): in closed form for ns <= 2, as a scaling-and-squaring
    matrix exponential for 2 < ns <= 1024; they stay on the device for the run and are copied to the
    host only when exp_V / exp_V_half are read.  The eigen data (d2a = U, apes = w) are host eigh
    results computed on first access.  ns > 1024 builds on the host with a vectorised eigh.
    """
    _eV_dev = _eVh_dev = None
    _exp_V_host = _exp_V_half_host = None
    _d2a = _apes = None
    _eig_pending = False

    @property
    def exp_V(self):
        if self._exp_V_host is None and self._eV_dev is not None:
            self._exp_V_host = self._eV_dev.cpu().numpy()
        return self._exp_V_host

    @exp_V.setter
    def exp_V(self, a):
        self._exp_V_host, self._eV_dev = a, None

    @property
    def exp_V_half(self):
        if self._exp_V_half_host is None and self._eVh_dev is not None:
            self._exp_V_half_host = self._eVh_dev.cpu().numpy()
        return self._exp_V_half_host

    @exp_V_half.setter
    def exp_V_half(self, a):
        self._exp_V_half_host, self._eVh_dev = a, None

    def _host_eig(self):
        v = self._pot()
        w, u = np.linalg.eigh(v)          # ascending eigenvalues per point (phys.sort order)
        self._d2a = u
        self._apes = None if np.iscomplexobj(v) else w
        self._eig_pending = False
        return w, u

    @property
    def d2a(self):
        if self._eig_pending:
            self._host_eig()
        return self._d2a

    @d2a.setter
    def d2a(self, u):
        self._d2a = u

    @property
    def apes(self):
        if self._eig_pending:
            self._host_eig()
        return self._apes

    @apes.setter
    def apes(self, w):
        self._apes = w

    def _build_point_ops(self, dt):
        v = self._pot()
        ns = v.shape[-1]
        _check_finite(v)
        if ns > DEVICE_EXPM_MAX_NS:   # beyond the device exponential's cap (qd_spo_expv): host eigh, as the reference
            w, u = self._host_eig()
            ud = np.conj(np.swapaxes(u, -1, -2))
            self.exp_V = (u * np.exp(-1j * w * dt)[..., None, :]) @ ud
            self.exp_V_half = (u * np.exp(-1j * w * dt / 2)[..., None, :]) @ ud
            return
        dev = default_device()
        _lib.ensure_device(dev)
        cplx = np.iscomplexobj(v)
        vd = torch.from_numpy(np.ascontiguousarray(v, dtype=complex if cplx else float)).to(dev)
        eV = torch.empty(v.shape, dtype=torch.complex128, device=dev)
        eVh = torch.empty_like(eV)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo_expv(vd.data_ptr(), int(cplx), int(v.size // (ns * ns)), ns, float(dt),
                                         eV.data_ptr(), eVh.data_ptr(), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo_expv")
        self.exp_V, self.exp_V_half = None, None
        self._eV_dev, self._eVh_dev = eV, eVh
        self._d2a = self._apes = None
        self._eig_pending = True

    def _point_ops_dev(self, dev, need_full=False):
        eVh = self._eVh_dev if self._eVh_dev is not None else _dev_c128(self.exp_V_half, dev)
        eV = None
        if need_full:
            eV = self._eV_dev if self._eV_dev is not None else _dev_c128(self.exp_V, dev)
        return eV, eVh


class SPO2(_PointPropagators):
    """Drop-in for pyqed.wpd.SPO2 (wpd.py:379-887), linear and Jacobi coordinates."""

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

    def _pot(self):
        return self.v

    def build(self, dt, inertia=None):
        """wpd.py:496-625: the kinetic propagator (linear: exp_K on the 'ij' k-grid; jacobi:
        exp_Kx and exp_Ky[i, ky] = exp(-i ky^2 / (2 I(x_i)) dt) with I = masses[1]) and the per-point
        U e^{-i w tau} U^+ (device build, _PointPropagators)."""
        nx, ny = self.nx, self.ny
        self.kx = 2. * np.pi * fftfreq(nx, interval(self.x))
        self.ky = 2. * np.pi * fftfreq(ny, interval(self.y))
        self._build_keo(dt)
        if self.v is None:
            raise ValueError('The diabatic PES is not specified.')
        self._build_point_ops(dt)

    def _build_keo(self, dt):
        if self.coords == 'linear':
            mx, my = self.masses
            Kx, Ky = meshgrid(self.kx, self.ky)
            self.exp_K = np.exp(-1j * (Kx ** 2 / 2. / mx + Ky ** 2 / 2. / my) * dt)
        elif self.coords == 'jacobi':
            mx = self.masses[0]
            self.exp_Kx = np.exp(-1j * self.kx ** 2 / 2. / mx * dt)
            Iinv = 1. / self.masses[1](self.x)  # y is the angle
            self.exp_Ky = np.exp(-1j * np.outer(Iinv, self.ky ** 2 / 2.) * dt)
        else:
            raise ValueError(f"unknown coordinates {self.coords!r}")

    def _propagate(self, psi0, dt, nt, nout, merged):
        """GPU run (qd_spo2_run_ex): Strang steps V/2 K V/2 with a snapshot after every nout
        steps (merged=False), or the merged V/2, [K V]..., K, V/2 structure (merged=True).
        Returns (final psi, list of snapshots)."""
        dev = default_device()
        _lib.ensure_device(dev)
        nsteps = (nt // nout) * nout
        psi = _dev_c128(psi0, dev)
        nsnap = nt // nout
        snap = torch.empty((nsnap, self.nx, self.ny, self.ns), dtype=torch.complex128, device=dev) if nsnap else None
        eV, eVh = self._point_ops_dev(dev, need_full=merged)
        if self.coords == 'jacobi':
            eK = _dev_c128(np.broadcast_to(self.exp_Kx[:, None], (self.nx, self.ny)), dev)
            eKy = _dev_c128(self.exp_Ky, dev)
        else:
            eK = _dev_c128(self.exp_K, dev)
            eKy = None
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo2_run_ex(psi.data_ptr(), eVh.data_ptr(), _lib.ptr(eV), eK.data_ptr(), _lib.ptr(eKy),
                                            self.nx, self.ny, self.ns, int(nsteps), int(nout), _lib.ptr(snap),
                                            _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo2_run_ex")
        states = []
        if snap is not None:
            host = snap.cpu().numpy()
            states = [host[k] for k in range(nsnap)]
        return psi.cpu().numpy(), states

    def run_batch(self, psi0s, dt=0.01, nt=1, nout=1, device=None):
        """Extension: B independent wavepackets psi0s [B, nx, ny, ns] on one potential, Strang steps as
        run(return_states=True) for each (qd_spo2_run_batch: one launch per pass for the whole batch).
        Returns (final states [B, nx, ny, ns], snapshots [B, nt//nout, nx, ny, ns]) as device tensors.
        Jacobi coordinates run the _KEO_jacobi step structure (qd_spo2_run_ex) member by member."""
        self.build(dt=dt)
        dev = device or default_device()
        _lib.ensure_device(dev)
        psi = psi0s if isinstance(psi0s, torch.Tensor) else _dev_c128(psi0s, dev)
        psi = psi.to(device=dev, dtype=torch.complex128).contiguous().clone()
        B = psi.shape[0]
        if tuple(psi.shape[1:]) != (self.nx, self.ny, self.ns):
            raise ValueError(f"psi0s must be [B, {self.nx}, {self.ny}, {self.ns}]")
        nsnap = nt // nout
        snap = torch.empty((B, nsnap, self.nx, self.ny, self.ns), dtype=torch.complex128, device=dev) if nsnap \
            else None
        _, eVh = self._point_ops_dev(dev, need_full=False)
        if self.coords == 'jacobi':
            eK = _dev_c128(np.broadcast_to(self.exp_Kx[:, None], (self.nx, self.ny)), dev)
            eKy = _dev_c128(self.exp_Ky, dev)
            with torch.cuda.device(dev):
                for b in range(B):
                    rc = _lib.load().qd_spo2_run_ex(psi[b].data_ptr(), eVh.data_ptr(), None, eK.data_ptr(),
                                                    eKy.data_ptr(), self.nx, self.ny, self.ns, int(nsnap * nout),
                                                    int(nout), snap[b].data_ptr() if nsnap else None,
                                                    _lib.stream_ptr(dev))
                    _lib.check(rc, "qd_spo2_run_ex")
            return psi, snap
        eK = _dev_c128(self.exp_K, dev)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo2_run_batch(psi.data_ptr(), B, eVh.data_ptr(), eK.data_ptr(), self.nx, self.ny,
                                               self.ns, int(nsnap * nout), int(nout), _lib.ptr(snap),
                                               _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo2_run_batch")
        return psi, snap

    def run(self, psi0, e_ops=[], dt=0.01, nt=1, t0=0., nout=1, return_states=True):
        """wpd.py:692-758.  return_states=True: psilist = [psi0] + the state after every nout
        Strang steps (nt//nout*nout steps).  return_states=False: the merged-V arithmetic runs
        but, as in the reference, psilist is only [psi0].  r.psi is the final state (the
        reference leaves it unset)."""
        self.build(dt=dt)
        psi, states = self._propagate(psi0, dt, nt, nout, merged=not return_states)
        r = ResultSPO2(dt=dt, psi0=psi0, Nt=nt, t0=t0, nout=nout)
        r.x = self.x
        r.y = self.y
        r.psilist = [psi0] + (states if return_states else [])
        r.psi = psi
        return r


class SPO2NH(SPO2):
    """Drop-in for pyqed.wpd.SPO2NH (wpd.py:921-1081): complex (non-Hermitian) diabatic
    potential; exp_V = U_R e^{-i w dt} U_R^-1 from the right eigenvectors (nonherm.eig,
    nonherm.py:26-76, eigenvalues sorted by np.argsort)."""

    def __init__(self, x, y, *args, **kwargs):
        self.right_eigenstates = None
        super().__init__(x, y, *args, **kwargs)

    _ur = _ovlp = None

    def build(self, dt):
        """wpd.py:960-985.  exp_V = U_R e^{-i w dt} U_R^-1 is the matrix exponential exp(-i V dt); it is evaluated on
        the GPU (qd_spo_expm, scaling and squaring, no eigenvectors) for ns <= 1024.  The right eigenvectors and their
        overlap (right_eigenstates, ovlp_rr; nonherm.eig order, eigenvalues by argsort) are host eig results made
        on first access (position() reads ovlp_rr)."""
        nx, ny = self.nx, self.ny
        self.kx = 2. * np.pi * fftfreq(nx, interval(self.x))
        self.ky = 2. * np.pi * fftfreq(ny, interval(self.y))
        self._build_keo(dt)
        v = np.asarray(self.v, dtype=complex)
        self._ur = self._ovlp = None
        ns = v.shape[-1]
        _check_finite(v)
        if ns > DEVICE_EXPM_MAX_NS:
            ur = self.right_eigenstates
            w = self._w
            ul = np.linalg.inv(ur)
            self.exp_V = (ur * np.exp(-1j * w * dt)[..., None, :]) @ ul
            self.exp_V_half = (ur * np.exp(-1j * w * dt / 2)[..., None, :]) @ ul
            return
        dev = default_device()
        _lib.ensure_device(dev)
        vd = _dev_c128(v, dev)
        eV = torch.empty(v.shape, dtype=torch.complex128, device=dev)
        eVh = torch.empty_like(eV)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_spo_expm(vd.data_ptr(), 0, int(v.size // (ns * ns)), ns, float(dt), eV.data_ptr(),
                                         eVh.data_ptr(), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_spo_expm")
        self.exp_V, self.exp_V_half = None, None
        self._eV_dev, self._eVh_dev = eV, eVh

    def _host_eig_nh(self):
        w, ur = np.linalg.eig(np.asarray(self.v, dtype=complex))
        idx = np.argsort(w, axis=-1)
        self._w = np.take_along_axis(w, idx, axis=-1)
        self._ur = np.take_along_axis(ur, idx[..., None, :], axis=-1)
        self._ovlp = np.conj(np.swapaxes(self._ur, -1, -2)) @ self._ur

    @property
    def right_eigenstates(self):
        if self._ur is None and getattr(self, "v", None) is not None:
            self._host_eig_nh()
        return self._ur

    @right_eigenstates.setter
    def right_eigenstates(self, u):
        self._ur = u

    @property
    def ovlp_rr(self):
        if self._ovlp is None and getattr(self, "v", None) is not None:
            self._host_eig_nh()
        return self._ovlp

    def position(self, psilist):
        """wpd.py:997-1017 (no plot, no xAve.npz file)."""
        dx, dy = interval(self.x), interval(self.y)
        S = self.ovlp_rr
        xAve = [np.einsum('ijm, i, ijmn, ijn ->', psi.conj(), self.x, S, psi) * dx * dy for psi in psilist]
        yAve = [np.einsum('ijn, j, ijmn, ijn ->', psi.conj(), self.y, S, psi) * dx * dy for psi in psilist]
        self.xAve = [xAve, yAve]
        return xAve, yAve

    def run(self, psi0, e_ops=[], dt=0.01, nt=1, t0=0., nout=1, return_states=True):
        """wpd.py:1019-1077: Strang steps (return_states=True) or the merged structure
        (False); psilist = [psi0] + the state after every nout steps in both cases; r.psi set."""
        self.build(dt=dt)
        psi, states = self._propagate(psi0, dt, nt, nout, merged=not return_states)
        r = ResultSPO2(dt=dt, psi0=psi0, Nt=nt, t0=t0, nout=nout)
        r.x = self.x
        r.y = self.y
        r.psilist = [psi0] + states
        r.psi = psi
        return r


def axis_propagator(k, m, dt):
    """First column m_a = ifft(e_a) of the circulant kinetic propagator of one axis, M_a = F^-1 diag(e_a) F with
    e_a = exp(-i k^2/(2m) dt) (M_a[i][j] = m_a[(i - j) mod n]; M_a @ v = ifft(e_a * fft(v))): exp_K of linear
    coordinates (wpd.py:1255-1262) is the outer product of the axis factors, so fftn, * exp_K, ifftn (wpd.py:1418-1432)
    is M_x (x) M_y (x) M_z.  Host setup, like exp_K itself."""
    k = np.asarray(k, dtype=float)
    return np.ascontiguousarray(np.fft.ifft(np.exp(-1j * k * k / 2. / m * dt)))


class SPO3(_PointPropagators):
    """Drop-in for pyqed.wpd.SPO3 (wpd.py:1105-1432), linear coordinates.

    kinetic_path: "auto" takes the separable kinetic step (qd_spo3_run_axes) when every axis has at most AXES_MAX_N
    points and there are one or two states: 64^3 as three register-FFT passes of F^-1 diag(e_a / n) F (22 us per
    64^3 x 2 step against 26 on the four passes of the 3-D exp_K), every other such grid as three per-axis mode
    products on the MFMAs (60^3 x 2: 31 us against 52 on the mixed-radix FFT passes; profiles/r06/spo/);
    larger grids or more states the FFT passes (qd_spo3_run).  "axes" / "fft" force one (tests).
    """

    AXES_MAX_N = 64
    kinetic_path = "auto"

    def _use_axes(self):
        dims = (self.nx, self.ny, self.nz)
        fits = max(dims) <= self.AXES_MAX_N and self.nstates <= 2
        if self.kinetic_path == "axes":
            if not fits:
                raise ValueError(f"kinetic_path='axes' needs every axis <= {self.AXES_MAX_N} points and nstates <= 2")
            return True
        if self.kinetic_path == "fft":
            return False
        return fits

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
        """wpd.py:1210-1340 (linear): exp_K on the 'ij' grid, exp(-i V dt/2) per point.
        coords='jacobi' is not a working path of the reference: its SPO3._KEO_jacobi (wpd.py:1434-1469) contracts the
        4-index wavefunction [nx, ny, nz, ns] with 'ij, ija -> ija' (the 2-D SPO2 form), which numpy rejects, and its
        build never forms a z kinetic factor; there is no step structure to reproduce, so it is refused here."""
        if self.coords == 'jacobi':
            raise NotImplementedError("SPO3 with coords='jacobi': the reference's _KEO_jacobi (wpd.py:1434-1469) is the "
                                      "2-D SPO2 operator applied to a 3-D grid and fails there; no 3-D Jacobi KEO exists")
        if self.coords != 'linear':
            raise ValueError(f"unknown coordinates {self.coords!r}")
        self.kx = 2. * np.pi * fftfreq(self.nx, self.dx)
        self.ky = 2. * np.pi * fftfreq(self.ny, self.dy)
        self.kz = 2. * np.pi * fftfreq(self.nz, self.dz)
        mx, my, mz = self.masses
        Kx, Ky, Kz = meshgrid(self.kx, self.ky, self.kz)
        self.exp_K = np.exp(-1j * (Kx ** 2 / 2. / mx + Ky ** 2 / 2. / my + Kz ** 2 / 2. / mz) * dt)
        if self.V is None:
            raise ValueError('The diabatic PES is not specified.')
        self._build_point_ops(dt)

    def _pot(self):
        return self.V

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
        _, eVh = self._point_ops_dev(dev)
        if self._use_axes():
            M = [_dev_c128(axis_propagator(k, m, dt), dev) for k, m in zip((self.kx, self.ky, self.kz), self.masses)]
            with torch.cuda.device(dev):
                rc = _lib.load().qd_spo3_run_axes(psi.data_ptr(), eVh.data_ptr(), *(m.data_ptr() for m in M),
                                                  self.nx, self.ny, self.nz, self.nstates, int(nsteps), int(nout),
                                                  _lib.ptr(snap), _lib.stream_ptr(dev))
            _lib.check(rc, "qd_spo3_run_axes")
        else:
            eK = _dev_c128(self.exp_K, dev)
            with torch.cuda.device(dev):
                rc = _lib.load().qd_spo3_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), self.nx, self.ny,
                                             self.nz, self.nstates, int(nsteps), int(nout), _lib.ptr(snap),
                                             _lib.stream_ptr(dev))
            _lib.check(rc, "qd_spo3_run")
        r = Result(dt=dt, psi0=psi0, Nt=nt, t0=t0, nout=nout)
        if snap is not None:
            host = snap.cpu().numpy()
            r.psilist = [host[k] for k in range(nsnap)]
        r.psi = psi.cpu().numpy()
        return r
