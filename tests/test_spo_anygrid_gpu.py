"""SPO / SPO2 / SPO3 on every grid the reference accepts: non-power-of-two lengths, prime
lengths (Bluestein axes), lines longer than the LDS plan (direct DFT axes), ns > 8 and the 1024 x 1024 x 2 grid
round 2 refused, all through the any-size engine (pyqed_amd/csrc/spo_gen.hip) against reference fixtures
(tests/golden/make_golden.py: spo2_20x20, spo2_96x80, spo2_67x45_ns3, spo2_12x10_ns9, spo2_1024, spo3_24x20x18,
spo1d_any).  fp64 with a different FFT factorisation than pocketfft: 1e-10 relative (L2)."""
import os

import numpy as np
import pytest

from conftest import load_golden, relerr
from spo_models import spo1d_model, spo2_model_rect, spo3_model

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _spo2(name, env=None):
    from pyqed_amd import SPO2
    g = load_golden(name)
    nx, ny, ns = int(g["nx"]), int(g["ny"]), int(g["ns"])
    x, y, surfaces, couplings, psi0 = spo2_model_rect(nx, ny, ns)
    sol = SPO2(x, y, mass=[1.0, 1.3], nstates=ns)
    sol.set_DPES(surfaces, couplings)
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        r = sol.run(psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return g, r, x, y


@pytest.mark.parametrize("name", ["spo2_20x20", "spo2_96x80", "spo2_67x45_ns3", "spo2_12x10_ns9"])
def test_spo2_any_grid_matches_reference(name):
    g, r, x, y = _spo2(name)
    assert len(r.psilist) == int(g["n_psilist"])
    assert np.allclose(r.times, g["times"])
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL


@pytest.mark.parametrize("kind", ["1", "2"])
def test_spo2_forced_bluestein_and_direct_axes(kind):
    """Every axis forced onto the chirp-z plan (1) or the direct HBM DFT (2, unfused passes)."""
    g, r, x, y = _spo2("spo2_96x80", env={"QD_SPO_FORCE_KIND": kind})
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL


def test_spo2_1024_matches_reference():
    g, r, x, y = _spo2("spo2_1024")
    psi = r.psilist[-1]
    assert relerr(psi[::16, ::16], g["psi_final_sample"]) < TOL
    assert relerr(psi[512], g["psi_final_row"]) < TOL
    assert relerr(psi[:, 1024 // 3], g["psi_final_col"]) < TOL
    dx, dy = x[1] - x[0], y[1] - y[0]
    pops = np.array([[np.vdot(p[:, :, k], p[:, :, k]).real * dx * dy for k in range(2)] for p in r.psilist])
    assert relerr(pops, g["populations"]) < TOL


def test_spo2_pow2_through_generic_engine_matches_reference():
    """QD_SPO_GENERIC=1 sends a power-of-two grid (spo2_32) through the any-size engine too."""
    import os
    from pyqed_amd import SPO2
    g = load_golden("spo2_32")
    sol = SPO2(g["x"], g["y"], mass=list(g["masses"]), nstates=2)
    sol.set_DPES([g["v0"], g["v1"]], [[[0, 1], g["coupling"]]])
    os.environ["QD_SPO_GENERIC"] = "1"
    try:
        r = sol.run(g["psi0"], dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    finally:
        os.environ.pop("QD_SPO_GENERIC", None)
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL


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


def test_spo3_any_grid_matches_reference():
    from pyqed_amd import SPO3
    g = load_golden("spo3_24x20x18")
    (x, y, z), masses, surfaces, couplings, psi0 = spo3_model()
    sol = SPO3(x, y, z, masses=masses, nstates=2)
    sol.set_DPES(surfaces, couplings)
    r = sol.run(psi0=psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
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


def test_spo1d_long_line_direct_dft_matches_reference(monkeypatch):
    """The 6000-point line runs the four-step FFT by default (6000 = 75 x 80); QD_SPO_FORCE_KIND=2 sends it through the
    direct O(L^2) DFT instead — both against the reference fixture."""
    from pyqed_amd import SPO
    g = load_golden("spo1d_any")
    n = 6000
    x, psi0 = spo1d_model(n)
    monkeypatch.setenv("QD_SPO_FORCE_KIND", "2")
    sol = SPO(x, mass=1.0)
    sol.set_potential(lambda q: q ** 2 / 2)
    r = sol.run(psi0, dt=0.01, nt=int(g[f"n{n}_nt"]), nout=int(g[f"n{n}_nout"]))
    assert relerr(r.psi, g[f"n{n}_psi"]) < TOL


@pytest.mark.parametrize("name", ["spo2_96x80", "spo2_67x45_ns3"])
def test_spo2_alternating_layouts_bit_identical_to_in_place_passes(name, monkeypatch):
    """The 2D generic passes alternate [x][y][s] / [y][x][s] layouts (spo_gen.hip Exec::xpose): same FFT plans, same
    operations on the same line values, so the result equals the in-place passes (QD_SPO_XPOSE=0) bit for bit —
    Strang, merged-V and Jacobi step sequences — and the reference fixture."""
    from pyqed_amd import SPO2
    g, r1, x, y = _spo2(name)
    _, r0, _, _ = _spo2(name, env={"QD_SPO_XPOSE": "0"})
    assert np.array_equal(np.array(r1.psilist), np.array(r0.psilist))
    assert relerr(np.array(r1.psilist), g["psilist"]) < TOL
    xs, ys, surfaces, couplings, psi0 = spo2_model_rect(30, 22, 2)
    for kw, coords in (({"return_states": False}, "linear"), ({}, "jacobi")):
        mass = [1.0, 1.3] if coords == "linear" else [1.0, lambda q: 1.5 + 0.2 * q ** 2]
        out = []
        for xp in ("1", "0"):
            monkeypatch.setenv("QD_SPO_XPOSE", xp)
            sol = SPO2(xs, ys, mass=mass, nstates=2, coords=coords)
            sol.set_DPES(surfaces, couplings)
            out.append(sol.run(psi0, dt=0.05, nt=5, nout=2, **kw).psi)
        assert np.array_equal(out[0], out[1]), coords


def test_spo3_rotated_layouts_bit_identical_to_in_place_passes(monkeypatch):
    """3D grids can rotate their layouts (QD_SPO_XPOSE3=1, opt-in): [x][y][z] -> [x][z][y] -> [z][y][x] -> [x][z][y]
    -> [x][y][z] over a step's four passes (spo_gen.hip Exec::z3_pass), equal bit for bit to the in-place passes
    (QD_SPO_XPOSE3=0), Strang and merged V."""
    from pyqed_amd import SPO3
    g = load_golden("spo3_24x20x18")
    (x, y, z), masses, surfaces, couplings, psi0 = spo3_model()
    out = {}
    for xp in ("1", "0"):
        monkeypatch.setenv("QD_SPO_XPOSE3", xp)
        sol = SPO3(x, y, z, masses=masses, nstates=2)
        sol.set_DPES(surfaces, couplings)
        r = sol.run(psi0=psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
        rm = sol.run(psi0=psi0, dt=float(g["dt"]), nt=3, nout=1, return_states=False)
        out[xp] = (np.array(r.psilist), r.psi, rm.psi)
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(a, b)
    assert relerr(out["1"][0], g["psilist"]) < TOL
