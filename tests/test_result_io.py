"""Output formats: Result.dump / load_result (mol.py:146-179) and ResultSPO2.dump and its
population / position writers (wpd.py:57-178).  Host-only: the containers are plain Python objects."""
import os

import numpy as np
import pytest
from scipy.sparse import csr_matrix

from conftest import relerr


def test_result_times_convention():
    from pyqed_amd.mol import Result
    r = Result(dt=0.1, Nt=10, t0=0.5, nout=3)
    # mol.py:113: times = t0 + arange(Nt // nout + 1) * dt * nout
    assert np.allclose(r.times, 0.5 + np.arange(10 // 3 + 1) * 0.1 * 3)
    assert r.timesteps == r.nt == 10 and r.psilist == [] and r.psi is None and r.rholist is None


def test_result_dump_load_roundtrip(tmp_path):
    from pyqed_amd.mol import Result, load_result
    rng = np.random.default_rng(0)
    rho0 = rng.standard_normal((4, 4)) + 1j * rng.standard_normal((4, 4))
    r = Result(description="lindblad", rho0=rho0, dt=0.01, Nt=5, t0=0.2)
    r.observables = rng.standard_normal((6, 2)) + 1j * rng.standard_normal((6, 2))
    r.rholist = [csr_matrix(rng.standard_normal((4, 4))) for _ in range(5)]
    fname = os.path.join(tmp_path, "res.pkl")
    r.dump(fname)
    q = load_result(fname)
    assert isinstance(q, Result)
    assert q.description == "lindblad" and q.dt == 0.01 and q.nt == 5 and q.nout == 1
    assert np.array_equal(q.times, r.times)
    assert np.array_equal(q.observables, r.observables)
    assert np.array_equal(q.rho0, rho0)
    assert len(q.rholist) == 5
    assert all(abs(a - b).max() == 0 for a, b in zip(q.rholist, r.rholist))
    r.save(fname + "2")  # save == dump (mol.py:164-165)
    assert np.array_equal(load_result(fname + "2").observables, r.observables)


def _spo2_result():
    from pyqed_amd.wpd import ResultSPO2
    x = np.linspace(-3, 3, 16)
    y = np.linspace(-2, 2, 8)
    X, Y = np.meshgrid(x, y, indexing="ij")
    psi0 = np.zeros((16, 8, 2), complex)
    psi0[:, :, 0] = np.exp(-(X - 0.3) ** 2 - Y ** 2)
    psi1 = psi0.copy()
    psi1[:, :, 1] = 0.5j * np.exp(-X ** 2 - (Y + 0.2) ** 2)
    r = ResultSPO2(dt=0.05, psi0=psi0, Nt=4, t0=0.0, nout=2)
    r.x, r.y = x, y
    r.psilist = [psi0, psi1, psi1 * np.exp(0.3j)]
    r.psi = r.psilist[-1]
    return r


def test_result_spo2_population_position_and_dump(tmp_path, monkeypatch):
    from pyqed_amd.mol import load_result
    from pyqed_amd.wpd import ResultSPO2
    monkeypatch.chdir(tmp_path)
    r = _spo2_result()
    assert r.nstates == 2
    dx, dy = r.x[1] - r.x[0], r.y[1] - r.y[0]
    p = r.get_population(fname="pop")
    want = np.array([[np.vdot(psi[:, :, n], psi[:, :, n]).real * dx * dy for n in range(2)] for psi in r.psilist])
    assert relerr(p, want) < 1e-14
    assert np.array_equal(np.load("pop.npz")["arr_0"], p)  # np.savez(fname, p), wpd.py:117-119
    xa, ya = r.position()
    assert np.isrealobj(xa) and np.isrealobj(ya)  # np.real_if_close, wpd.py:150-151
    f = np.load("xAve.npz")                         # np.savez('xAve', xAve, yAve), wpd.py:159
    assert np.array_equal(f["arr_0"], xa) and np.array_equal(f["arr_1"], ya)
    r.dump("spo2.pkl")
    q = load_result("spo2.pkl")
    assert isinstance(q, ResultSPO2)
    assert np.array_equal(q.x, r.x) and np.array_equal(q.y, r.y)
    assert all(np.array_equal(a, b) for a, b in zip(q.psilist, r.psilist))
    assert np.array_equal(q.psi, r.psi) and np.array_equal(q.population, p)
    assert np.array_equal(q.times, r.times)


@pytest.mark.gpu
def test_spo2_run_result_dump_roundtrip(tmp_path):
    """A ResultSPO2 produced by the GPU SPO2.run survives dump / load_result bit for bit."""
    from pyqed_amd import SPO2
    from pyqed_amd.mol import load_result
    x = np.linspace(-4, 4, 32)
    y = np.linspace(-4, 4, 32)
    X, Y = np.meshgrid(x, y, indexing="ij")
    sol = SPO2(x, y, mass=[1, 1], nstates=2)
    sol.set_DPES([0.5 * (X ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
    psi0 = np.zeros((32, 32, 2), complex)
    psi0[:, :, 0] = np.exp(-(X + 0.5) ** 2 - Y ** 2)
    r = sol.run(psi0, dt=0.05, nt=6, nout=2)
    fname = os.path.join(tmp_path, "r.pkl")
    r.dump(fname)
    q = load_result(fname)
    assert len(q.psilist) == len(r.psilist) == 6 // 2 + 1
    assert all(np.array_equal(a, b) for a, b in zip(q.psilist, r.psilist))
    assert np.array_equal(q.times, r.times)
