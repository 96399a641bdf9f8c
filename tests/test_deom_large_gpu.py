"""DEOM / HEOM hierarchies beyond round 2's caps: ns > 16 system levels and more than 8
coupling modes run on the tiled stage kernel (deom.hip deom_stage_tile_kernel), the Euler HEOM chain on any ns,
all against the oracle restatements (oracle/deom.py run -> heom/deom.py:641-766, 1072-1114; oracle/heom.py ->
HEOM/heom.py:275-347, oqs.py:1808-1875), which tests/test_oracle_golden.py pins to the reference."""
import numpy as np
import pytest
import sympy as sp

from conftest import relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _model(ns, L, nbath=1, npsd=2, pulsed=True, seed=0):
    from pyqed_amd.deom import Bath, DEOMSolver
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (a + a.conj().T) / 2 / np.sqrt(ns)
    w = sp.symbols(r"\omega", real=True)
    spectra = [2 * 0.3 * (1 + 0.1 * i) * w / ((1 + 0.1 * i) ** 2 + w ** 2) for i in range(nbath)]
    mode = [i for i in range(nbath) for _ in range(1 + npsd)]
    bath = Bath(spectra, w, [1.0] * nbath, [npsd] * nbath, mode)
    Q = np.array([np.diag(np.cos(np.arange(ns) + i)).astype(complex) + 0.05 * np.roll(np.eye(ns), i + 1, 1)
                  for i in range(nbath)])
    Q = (Q + np.conj(np.swapaxes(Q, 1, 2))) / 2
    sdip = (np.roll(np.eye(ns), 1, 1) + np.roll(np.eye(ns), -1, 1)).astype(complex)
    fs = (lambda t: 0.3 * np.sin(2 * t)) if pulsed else None
    fc = (lambda t: 0.1 * np.cos(t)) if pulsed else None
    cdip = 0.5 * Q if pulsed else None
    sol = DEOMSolver(H, sdip if pulsed else None, bath, Q, cdip, fs, fc, L)
    rho0 = np.zeros((ns, ns), complex)
    rho0[0, 0] = 1
    return sol, bath, H, Q, sdip, cdip, fs, fc, rho0


def _check(ns, L, nbath=1, npsd=2, nt=5, dt=0.01, path=None):
    from oracle import deom as od
    from conftest import took
    sol, bath, H, Q, sdip, cdip, fs, fc, rho0 = _model(ns, L, nbath, npsd)
    P1 = np.diag(np.linspace(1, 0, ns)).astype(complex)
    took("")
    t, tr = sol.run(rho0.copy(), dt, nt, P1)
    if path:
        hit, got = took(path)
        assert hit, got
    _, tr_ref, ados_ref = od.run(H, sdip, fs, Q, cdip, fc, (bath.etal, bath.etar, bath.etaa, bath.expn), L, rho0, dt,
                                 nt, P1, mode=bath.mode)
    assert relerr(np.asarray(tr), tr_ref) < TOL
    assert relerr(sol.ddos, ados_ref) < TOL


@pytest.mark.parametrize("ns,L", [(24, 3), (40, 2), (17, 2), (33, 2)])
def test_deom_large_ns_matches_oracle(ns, L):
    """ns = 17 / 24 / 33 / 40 (K = 3 Pade terms, driven H(t) and Q(t)): 16 x 16 MFMA tiles in 2 x 2 blocks with
    ragged edges (deom_stage_tmfma_kernel)."""
    _check(ns, L, path="deom_tmfma")


def test_deom_ten_modes_matches_oracle():
    """Ten coupling operators (ten Drude baths, npsd = 0: K = 10, nmod = 10 > round 2's 8), ns = 3, L = 2: the VALU
    tile kernel (deom_stage_tile_kernel)."""
    _check(3, 2, nbath=10, npsd=0, path="deom_tile")


def test_deom_element_kernel_matches_oracle():
    """ns = 3 with two baths of npsd = 4 (K = 10 > 8: no lane-group kernel; nmod = 2 <= 8): the element-per-thread
    stage kernel (deom_stage_kernel)."""
    _check(3, 2, nbath=2, npsd=4, path="deom_element")


@pytest.mark.parametrize("ns", [20, 33])
def test_heom_chains_large_ns_match_oracle(ns):
    """HEOM/heom.py RK4 chain (DEOM kernel, tiled at ns > 16) and the oqs.py Euler sweep (any ns) at ns = 20 / 33."""
    import pyqed_amd.heom as hh
    import pyqed_amd.oqs as oqs
    from oracle import heom as oh
    rng = np.random.default_rng(ns)
    a = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (a + a.conj().T) / 2 / np.sqrt(ns)
    Q = np.diag(np.linspace(-1, 1, ns)).astype(complex)
    rho0 = np.zeros((ns, ns), complex)
    rho0[0, 0] = 1
    E = [Q, np.eye(ns, k=1) + np.eye(ns, k=-1)]
    kw = dict(temperature=2.0, cutoff=1.0, reorganization=0.1, nado=5)
    for mod, ref in ((hh, oh.chain_rk4), (oqs, oh.chain_euler)):
        sol = mod.HEOMSolver(H, c_ops=[Q], e_ops=E)
        got = sol.run(rho0=rho0.copy(), dt=0.01, nt=12, **kw)
        want = ref(H, Q, rho0, E, kw["temperature"], kw["cutoff"], kw["reorganization"], kw["nado"], 0.01, 12)
        assert relerr(got, want) < TOL, mod.__name__
