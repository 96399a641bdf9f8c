"""Model builders shared by the arbitrary-grid SPO tests (the same seeded models tests/golden/make_golden.py runs
through the reference: spo2_model_rect, the spo3_24x20x18 potential, the spo1d_any harmonic well)."""
import numpy as np


def spo2_model_rect(nx, ny, ns=2, L=6.0):
    x = np.linspace(-L, L, nx)
    y = np.linspace(-L * 0.9, L * 0.9, ny)
    X, Y = np.meshgrid(x, y, indexing="ij")
    surfaces = [0.5 * ((X + 1 - a) ** 2 + Y ** 2) + 0.05 * a for a in range(ns)]
    couplings = [[[a, a + 1], 0.2 * X + 0.05 * Y] for a in range(ns - 1)]
    psi0 = np.zeros((nx, ny, ns), dtype=complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    return x, y, surfaces, couplings, psi0


def spo2_potential(surfaces, couplings, ns):
    """set_DPES's real potential array v[i, j, a, b] (wpd.py:436-484)."""
    nx, ny = surfaces[0].shape
    v = np.zeros((nx, ny, ns, ns))
    for a in range(ns):
        v[:, :, a, a] = surfaces[a]
    for (a, b), c in couplings:
        v[:, :, a, b] = np.real(c)
        v[:, :, b, a] = v[:, :, a, b]
    return v


def spo3_model():
    x, y, z = np.linspace(-6, 6, 24), np.linspace(-5, 5, 20), np.linspace(-5.5, 5.5, 18)
    X, Y, Z = np.meshgrid(x, y, z, indexing="ij")
    surfaces = [0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)]
    couplings = [[[0, 1], 0.2 * X]]
    psi0 = np.zeros((24, 20, 18, 2), dtype=complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 0.3j * Y) / np.pi ** 0.75
    return (x, y, z), [1.0, 1.2, 0.9], surfaces, couplings, psi0


def spo1d_model(n):
    x = np.linspace(-8, 8, n)
    psi0 = (np.exp(-(x + 2) ** 2 / 2 + 1j * 0.5 * x) / np.pi ** 0.25).astype(complex)
    return x, psi0
