"""NumPy restatement of the split-operator propagators (test infrastructure only).

Follows:
  pyqed/wpd.py:191-273   SPO (1D): build (exp_V, exp_V_half, exp_K), run with the
                         reference's step structure V/2 ; (nt//nout-1)*nout x [K, V] ; K, V/2
  pyqed/wpd.py:496-625   SPO2.build (per-point eigh, sorted, U e^{-iw dt} U^+)
  pyqed/wpd.py:692-758   SPO2.run (return_states=True): nt//nout*nout Strang steps
                         V/2 . IFFT2 . exp_K . FFT2 . V/2, psilist incl. psi0
  pyqed/wpd.py:837-848   _KEO_linear (scipy.fftpack fft2/ifft2 over axes (0, 1))
  pyqed/wpd.py:850-887   _KEO_jacobi; wpd.py:540-553 its exp_Kx / exp_Ky
  pyqed/wpd.py:736-755   run(return_states=False): merged V
  pyqed/wpd.py:921-1077  SPO2NH (nonherm.eig, nonherm.py:26-76)
"""
import numpy as np
import scipy.linalg
from scipy.fftpack import fft, fft2, fftfreq, ifft, ifft2


def spo1d_ops(x, V, mass, dt):
    dx = x[1] - x[0]
    k = 2.0 * np.pi * fftfreq(len(x), dx)
    return np.exp(-1j * V * dt), np.exp(-1j * V * dt / 2.0), np.exp(-0.5j / mass * (k * k) * dt)


def spo1d_run(x, V, psi0, dt, nt, nout=1, mass=1.0):
    expV, expVh, expK = spo1d_ops(x, V, mass, dt)
    psi = expVh * psi0.copy()
    psilist = []
    for i in range(1, nt // nout):
        for _ in range(nout):
            psi = ifft(fft(psi) * expK)
            psi = expV * psi
        psilist.append(psi.copy())
    psi = ifft(fft(psi) * expK)
    psi = expVh * psi
    return psilist, psi


def spo2_build(x, y, v, masses, dt):
    nx, ny, ns = v.shape[0], v.shape[1], v.shape[2]
    kx = 2.0 * np.pi * fftfreq(nx, x[1] - x[0])
    ky = 2.0 * np.pi * fftfreq(ny, y[1] - y[0])
    Kx, Ky = np.meshgrid(kx, ky, indexing="ij")
    mx, my = masses
    exp_K = np.exp(-1j * (Kx ** 2 / 2. / mx + Ky ** 2 / 2. / my) * dt)
    exp_V_half = np.zeros(v.shape, dtype=complex)
    for i in range(nx):
        for j in range(ny):
            w, u = scipy.linalg.eigh(v[i, j])
            idx = np.argsort(w)
            w, u = w[idx], u[:, idx]
            exp_V_half[i, j] = u @ np.diag(np.exp(-1j * w * dt / 2)) @ u.conj().T
    return exp_V_half, exp_K


def spo2_run(exp_V_half, exp_K, psi0, nt, nout=1):
    psi = psi0.copy()
    psilist = [psi0]
    for _ in range(nt // nout):
        for _ in range(nout):
            psi = np.einsum("ijab,ijb->ija", exp_V_half, psi)
            psi = ifft2(np.einsum("ij,ija->ija", exp_K, fft2(psi, axes=(0, 1))), axes=(0, 1))
            psi = np.einsum("ijab,ijb->ija", exp_V_half, psi)
        psilist.append(psi.copy())
    return psilist


def spo3_run(exp_V_half, exp_K, psi0, nt, nout=1):
    """wpd.py:1349-1411 (return_states=True): psilist WITHOUT psi0, numpy fftn over axes (0,1,2)."""
    psi = psi0.copy()
    psilist = []
    for _ in range(nt // nout):
        for _ in range(nout):
            psi = np.einsum("ijkab,ijkb->ijka", exp_V_half, psi)
            psi = np.fft.ifftn(np.einsum("ijk,ijka->ijka", exp_K, np.fft.fftn(psi, axes=(0, 1, 2))), axes=(0, 1, 2))
            psi = np.einsum("ijkab,ijkb->ijka", exp_V_half, psi)
        psilist.append(psi.copy())
    return psilist, psi


def spo2nh_build(v, dt):
    """wpd.py:960-985 SPO2NH.build: exp_V = U_R e^{-i w dt} U_R^-1 per grid point, with
    nonherm.eig (nonherm.py:26-76): scipy eig, eigenvalues sorted by argsort, U_L = inv(U_R)."""
    import scipy.linalg
    nx, ny, ns = v.shape[0], v.shape[1], v.shape[2]
    eV = np.zeros((nx, ny, ns, ns), complex)
    eVh = np.zeros((nx, ny, ns, ns), complex)
    for i in range(nx):
        for j in range(ny):
            w, ur = scipy.linalg.eig(v[i, j])
            idx = np.argsort(w)
            w, ur = w[idx], ur[:, idx]
            ul = scipy.linalg.inv(ur)
            eV[i, j] = ur @ np.diagflat(np.exp(-1j * w * dt)) @ ul
            eVh[i, j] = ur @ np.diagflat(np.exp(-1j * w * dt / 2)) @ ul
    return eV, eVh


def spo2_merged_run(exp_V, exp_V_half, keo, psi0, nt, nout=1):
    """wpd.py:736-755 / 1054-1077 (return_states=False): V/2, nt//nout blocks of nout x [K, V]
    (state after each block recorded), then K, V/2.  Returns (psilist incl. psi0, final psi)."""
    psi = np.einsum("ijab,ijb->ija", exp_V_half, psi0)
    psilist = [psi0]
    for _ in range(nt // nout):
        for _ in range(nout):
            psi = keo(psi)
            psi = np.einsum("ijab,ijb->ija", exp_V, psi)
        psilist.append(psi.copy())
    psi = keo(psi)
    psi = np.einsum("ijab,ijb->ija", exp_V_half, psi)
    return psilist, psi


def keo_linear(exp_K):
    """wpd.py:837-848."""
    return lambda psi: ifft2(np.einsum("ij,ija->ija", exp_K, fft2(psi, axes=(0, 1))), axes=(0, 1))


def jacobi_ops(x, y, mx, inertia, dt):
    """wpd.py:540-553: exp_Kx[kx], exp_Ky[i, ky] = exp(-i ky^2 / (2 I(x_i)) dt)."""
    kx = 2.0 * np.pi * fftfreq(len(x), x[1] - x[0])
    ky = 2.0 * np.pi * fftfreq(len(y), y[1] - y[0])
    exp_Kx = np.exp(-1j * kx ** 2 / 2. / mx * dt)
    exp_Ky = np.exp(-1j * np.outer(1. / inertia(x), ky ** 2 / 2.) * dt)
    return exp_Kx, exp_Ky


def keo_jacobi(exp_Kx, exp_Ky):
    """wpd.py:850-887: fft along y, * exp_Ky, fft along x, * exp_Kx, ifft2."""
    def keo(psi):
        t = np.einsum("ij,ija->ija", exp_Ky, fft(psi, axis=1))
        t = np.einsum("i,ija->ija", exp_Kx, fft(t, axis=0))
        return ifft2(t, axes=(0, 1))
    return keo


def spo2_strang_run(exp_V_half, keo, psi0, nt, nout=1):
    """wpd.py:718-732 with any KEO: psilist = [psi0] + state after every nout steps."""
    psi = psi0.copy()
    psilist = [psi0]
    for _ in range(nt // nout):
        for _ in range(nout):
            psi = np.einsum("ijab,ijb->ija", exp_V_half, psi)
            psi = keo(psi)
            psi = np.einsum("ijab,ijb->ija", exp_V_half, psi)
        psilist.append(psi.copy())
    return psilist, psi
