"""SPO3 kinetic step as three per-axis mode products on the MFMAs (qd_spo3_run_axes, spo_dense.hip) against the NumPy
fftn restatement of SPO3.run (oracle/spo.py, wpd.py:1349-1432) and the reference's own SPO3 fixture."""
import numpy as np
import pytest

from conftest import load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _model(dims, ns, seed=0):
    from pyqed_amd.wpd import SPO3
    ax = [np.linspace(-6, 6, n) for n in dims]
    X, Y, Z = np.meshgrid(*ax, indexing="ij")
    rng = np.random.default_rng(seed)
    psi0 = np.zeros(tuple(dims) + (ns,), dtype=complex)
    psi0[..., ns - 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 0.3j * Y) / np.pi ** 0.75
    psi0 += 0.05 * (rng.standard_normal(psi0.shape) + 1j * rng.standard_normal(psi0.shape))
    sol = SPO3(*ax, masses=[1.0, 1.3, 0.8], nstates=ns)
    sol.set_DPES([0.5 * ((X + (-1) ** a) ** 2 + Y ** 2 + Z ** 2) + 0.1 * a for a in range(ns)],
                 [[[a, a + 1], 0.2 * X] for a in range(ns - 1)])
    return sol, psi0


@pytest.mark.parametrize("dims,ns,nt,nout", [((64, 64, 64), 2, 4, 2), ((64, 64, 64), 1, 5, 2), ((60, 60, 60), 2, 3, 1),
                                             ((64, 48, 32), 1, 4, 4),
                                             ((17, 9, 33), 2, 5, 2), ((5, 7, 3), 2, 3, 1), ((2, 16, 40), 1, 2, 1),
                                             ((50, 3, 2), 2, 4, 3)])
def test_spo3_axes_matches_fftn_restatement(dims, ns, nt, nout, monkeypatch):
    """Every length in [1, 64] alike (the z pass's tile of whole points, column tiles crossing outer boundaries,
    padded K and rows, ragged last tiles), and 64^3 on the three separable register-FFT passes: snapshots and the
    final state against the fftn restatement, norm kept."""
    from oracle import spo as ospo
    from conftest import took
    sol, psi0 = _model(dims, ns)
    monkeypatch.setattr(type(sol), "kinetic_path", "axes")
    took("")
    r = sol.run(psi0=psi0, dt=0.1, nt=nt, nout=nout)
    hit, got = took("spo3_sep64" if tuple(dims) == (64, 64, 64) else "spo3_axes")
    assert hit, got
    ref, psi = ospo.spo3_run(sol.exp_V_half, sol.exp_K, psi0, nt, nout)
    assert len(r.psilist) == len(ref)
    assert relerr(np.array(r.psilist), np.array(ref)) < TOL
    assert relerr(r.psi, psi) < TOL
    assert abs(np.vdot(r.psi, r.psi).real / np.vdot(psi0, psi0).real - 1) < 1e-12


def test_spo3_axes_reference_fixture():
    """The reference's SPO3 on a 24 x 20 x 18 grid (tests/golden/make_golden.py: spo3_24x20x18): the default path of
    a grid that is not a power of two is the axis path."""
    from pyqed_amd import SPO3
    from spo_models import spo3_model
    from conftest import took
    g = load_golden("spo3_24x20x18")
    (x, y, z), masses, surfaces, couplings, psi0 = spo3_model()
    sol = SPO3(x, y, z, masses=masses, nstates=2)
    sol.set_DPES(surfaces, couplings)
    took("")
    r = sol.run(psi0=psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    assert took("spo3_axes")[0]
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL
    assert relerr(r.psi, g["psi"]) < TOL


def test_spo3_axes_long_run_matches_fft_passes():
    """400 Strang steps at 64^3 x 2: the separable entry point (three register-FFT passes at 64^3) against the four
    FFT passes of the 3-D exp_K (qd_spo3_run) on the same state."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.wpd import axis_propagator
    sol, psi0 = _model((64, 64, 64), 2)
    sol.build(0.05)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eVh, eK = t(sol.exp_V_half), t(sol.exp_K)
    M = [t(axis_propagator(k, m, 0.05)) for k, m in zip((sol.kx, sol.ky, sol.kz), sol.masses)]
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    a, b = t(psi0), t(psi0)
    _lib.check(lib.qd_spo3_run(a.data_ptr(), eVh.data_ptr(), eK.data_ptr(), 64, 64, 64, 2, 400, 400, None, st), "fft")
    _lib.check(lib.qd_spo3_run_axes(b.data_ptr(), eVh.data_ptr(), *(m.data_ptr() for m in M), 64, 64, 64, 2, 400,
                                    400, None, st), "axes")
    torch.cuda.synchronize()
    assert relerr(b.cpu().numpy(), a.cpu().numpy()) < 1e-10


def test_spo3_path_choice():
    """auto: every grid <= 64 per axis with one or two states takes the separable entry point (qd_spo3_run_axes);
    larger or many-state grids the FFT passes."""
    from pyqed_amd.wpd import SPO3
    pick = lambda dims, ns=2: SPO3(*[np.linspace(-1, 1, n) for n in dims], masses=[1, 1, 1], nstates=ns)._use_axes()
    assert pick((64, 64, 64)) and pick((32, 16, 64))
    assert pick((60, 60, 60)) and pick((64, 48, 32)) and pick((24, 20, 18), 1)
    assert not pick((96, 60, 60)) and not pick((60, 60, 60), 3)
