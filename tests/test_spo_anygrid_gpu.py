"""SPO / SPO2 / SPO3 on every grid the reference accepts: non-power-of-two lengths, prime
lengths (Bluestein axes), lines longer than the LDS plan (direct DFT axes), ns > 8 and the 1024 x 1024 x 2 grid
round 2 refused, all through the any-size engine (pyqed_amd/csrc/spo_gen.hip) against reference fixtures
(tests/golden/make_golden.py: spo2_20x20, spo2_96x80, spo2_67x45_ns3, spo2_12x10_ns9, spo2_1024, spo3_24x20x18,
spo1d_any).  fp64 with a different FFT factorisation than pocketfft: 1e-10 relative (L2)."""
import numpy as np
import pytest

from conftest import load_golden, relerr
from spo_models import spo1d_model, spo2_model_rect, spo3_model

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _spo2(name):
    from pyqed_amd import SPO2
    g = load_golden(name)
    nx, ny, ns = int(g["nx"]), int(g["ny"]), int(g["ns"])
    x, y, surfaces, couplings, psi0 = spo2_model_rect(nx, ny, ns)
    sol = SPO2(x, y, mass=[1.0, 1.3], nstates=ns)
    sol.set_DPES(surfaces, couplings)
    r = sol.run(psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    return g, r, x, y


@pytest.mark.parametrize("name", ["spo2_20x20", "spo2_96x80", "spo2_67x45_ns3", "spo2_12x10_ns9"])
def test_spo2_any_grid_matches_reference(name):
    g, r, x, y = _spo2(name)
    assert len(r.psilist) == int(g["n_psilist"])
    assert np.allclose(r.times, g["times"])
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL


@pytest.mark.parametrize("nx,ny,axes,layout", [(2579, 12, ("spo_axis_direct", "spo_axis_mixed"), "spo_layout_in_place"),
                                               (67, 45, ("spo_axis_bluestein", "spo_axis_mixed"), "spo_layout_alternating"),
                                               (96, 80, ("spo_axis_mixed",), "spo_layout_alternating")])
def test_spo2_axis_plans_and_layouts_match_oracle(nx, ny, axes, layout):
    """Each axis plan of the any-size engine, reached by its length: a prime line beyond the chirp-z plan (2579: the
    direct HBM DFT, in-place passes), a prime within it (67: Bluestein) and smooth lengths (mixed radix); the 2D
    alternating layouts wherever every axis is an LDS plan.  Strang runs against the oracle restatement (pinned to the
    reference at 32 x 32 and by the spo2_* fixtures)."""
    from oracle import spo as osp
    from pyqed_amd import SPO2
    from conftest import took
    x, y, surfaces, couplings, psi0 = spo2_model_rect(nx, ny, 2)
    sol = SPO2(x, y, mass=[1.0, 1.3], nstates=2)
    sol.set_DPES(surfaces, couplings)
    took("")
    r = sol.run(psi0, dt=0.05, nt=4, nout=2)
    got = took("")[1]
    for a in axes + (layout,):
        assert a in got, (a, got)
    pl, _ = osp.spo2_strang_run(sol.exp_V_half, osp.keo_linear(sol.exp_K), psi0, 4, 2)
    assert relerr(np.array(r.psilist), np.array(pl)) < TOL


def test_spo2_1024_matches_reference():
    g, r, x, y = _spo2("spo2_1024")
    psi = r.psilist[-1]
    assert relerr(psi[::16, ::16], g["psi_final_sample"]) < TOL
    assert relerr(psi[512], g["psi_final_row"]) < TOL
    assert relerr(psi[:, 1024 // 3], g["psi_final_col"]) < TOL
    dx, dy = x[1] - x[0], y[1] - y[0]
    pops = np.array([[np.vdot(p[:, :, k], p[:, :, k]).real * dx * dy for k in range(2)] for p in r.psilist])
    assert relerr(pops, g["populations"]) < TOL


def test_spo2_merged_and_jacobi_any_grid_match_oracle():
    """return_states=False (merged V, wpd.py:736-755) and coords='jacobi' (wpd.py:850-887) on a 30 x 22 grid
    against the oracle restatements (which tests/test_oracle_golden.py pins to the reference at 32 x 32)."""
    from oracle import spo as osp
    from pyqed_amd import SPO2
    x, y, surfaces, couplings, psi0 = spo2_model_rect(30, 22, 2)
    sol = SPO2(x, y, mass=[1.0, 1.3], nstates=2)
    sol.set_DPES(surfaces, couplings)
    r = sol.run(psi0, dt=0.05, nt=6, nout=2, return_states=False)
    keo = osp.keo_linear(sol.exp_K)
    _, fin = osp.spo2_merged_run(sol.exp_V, sol.exp_V_half, keo, psi0, 6, 2)
    assert relerr(r.psi, fin) < TOL
    solj = SPO2(x, y, mass=[1.0, lambda q: 1.5 + 0.2 * q ** 2], nstates=2, coords='jacobi')
    solj.set_DPES(surfaces, couplings)
    rj = solj.run(psi0, dt=0.05, nt=6, nout=3)
    pl, fin = osp.spo2_strang_run(solj.exp_V_half, osp.keo_jacobi(solj.exp_Kx, solj.exp_Ky), psi0, 6, 3)
    assert relerr(np.array(rj.psilist), np.array(pl)) < TOL


def test_spo3_any_grid_matches_reference(monkeypatch):
    """The mixed-radix FFT passes (spo_any); tests/test_spo3_axes_gpu.py runs the same fixture on the axis path."""
    from pyqed_amd import SPO3
    from conftest import took
    g = load_golden("spo3_24x20x18")
    (x, y, z), masses, surfaces, couplings, psi0 = spo3_model()
    sol = SPO3(x, y, z, masses=masses, nstates=2)
    sol.set_DPES(surfaces, couplings)
    monkeypatch.setattr(SPO3, "kinetic_path", "fft")
    took("")
    r = sol.run(psi0=psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    assert took("spo_any")[0]
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL
    assert relerr(r.psi, g["psi"]) < TOL


def test_spo1d_any_grid_matches_reference():
    """50, 97 (prime: Bluestein), 200, 2053 (prime, 4320-point chirp-z) and 6000 points (direct DFT)."""
    from pyqed_amd import SPO
    g = load_golden("spo1d_any")
    for n in g["sizes"]:
        n = int(n)
        x, psi0 = spo1d_model(n)
        sol = SPO(x, mass=1.0)
        sol.set_potential(lambda q: q ** 2 / 2)
        r = sol.run(psi0, dt=0.01, nt=int(g[f"n{n}_nt"]), nout=int(g[f"n{n}_nout"]))
        assert relerr(r.psi, g[f"n{n}_psi"]) < TOL, n
        if len(r.psilist):
            assert relerr(np.array(r.psilist), g[f"n{n}_psilist"]) < TOL, n


@pytest.mark.parametrize("n,path", [(6000, "spo1d_fourstep"), (2579, "spo1d_direct"), (97, "spo1d_bluestein"),
                                    (200, "spo1d_mixed")])
def test_spo1d_line_plans_match_oracle(n, path):
    """1D lines by plan: 6000 = 75 x 80 beyond the LDS plans (four-step FFT), the prime 2579 beyond the chirp-z plan
    (direct DFT), the prime 97 (Bluestein) and 200 (mixed radix), against the oracle's SPO.run restatement (wpd.py:
    225-273; the 6000-point line also against the reference fixture in test_spo1d_any_grid_matches_reference)."""
    from oracle import spo as osp
    from pyqed_amd import SPO
    from conftest import took
    x, psi0 = spo1d_model(n)
    sol = SPO(x, mass=1.0)
    sol.set_potential(lambda q: q ** 2 / 2)
    took("")
    r = sol.run(psi0, dt=0.01, nt=6, nout=2)
    hit, got = took(path)
    assert hit, got
    pl, fin = osp.spo1d_run(x, x ** 2 / 2, psi0, 0.01, 6, 2)
    assert relerr(r.psi, fin) < TOL
    assert relerr(np.array(r.psilist), np.array(pl)) < TOL


