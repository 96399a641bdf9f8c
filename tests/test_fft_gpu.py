"""pyqed.fft physical-unit transforms on the GPU (qd_fft_axis / qd_dft2) vs reference golden."""
import numpy as np
import pytest

from conftest import load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-12


def test_fft_ifft_1d():
    from pyqed_amd import fft as pf
    g = load_golden("fft_phys")
    G, w = pf.fft(g["a"], g["x"])
    assert relerr(G, g["fft_g"]) < TOL and np.allclose(w, g["fft_w"])
    G, w = pf.ifft(g["a"], g["x"])
    assert relerr(G, g["ifft_g"]) < TOL
    G, w = pf.fft(g["b"], g["x2"])           # n = 100: direct-DFT path
    assert relerr(G, g["fft100_g"]) < TOL


def test_fft_axis0_and_fft2_and_dft2():
    from pyqed_amd import fft as pf
    g = load_golden("fft_phys")
    G, w = pf.fft(g["M"], x=np.linspace(0, 3.1, 32), axis=0)
    assert relerr(G, g["fftax0_g"]) < TOL
    G, _ = pf.ifft(g["M"], x=np.linspace(0, 3.1, 32), axis=0)
    assert relerr(G, g["ifftax0_g"]) < TOL
    fx, fy, G = pf.fft2(g["M"][:, :32], dx=0.1, dy=0.2)
    assert relerr(G, g["fft2_g"]) < TOL and np.allclose(fy, g["fft2_fy"])
    assert relerr(pf.dft2(g["xs"], g["ys"], g["F"], g["kx"], g["ky"]), g["dft2"]) < TOL


def test_gaussian_known_answer():
    """Analytic check: FT of exp(-x^2/2) is sqrt(2 pi) exp(-w^2/2)."""
    from pyqed_amd import fft as pf
    x = np.linspace(-20, 20, 1024, endpoint=False)
    G, w = pf.fft(np.exp(-x ** 2 / 2), x)
    assert np.max(np.abs(G - np.sqrt(2 * np.pi) * np.exp(-w ** 2 / 2))) < 1e-11
