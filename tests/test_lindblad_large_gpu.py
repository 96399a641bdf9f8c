"""Lindblad / Redfield beyond round 2's caps: N > 1024 (split path), more than 16 collapse
operators and observables, many drive terms — against the oracle (oracle/lindblad.py, the restatement of
oqs._lindblad / liouvillian, oqs.py:697-714, 1596-1696, pinned to the reference in tests/test_oracle_golden.py)."""
import numpy as np
import pytest

from conftest import relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


def test_lindblad_n1100_matches_oracle():
    """N = 1100 (padded to 1152; round 2 refused N > 1024), one collapse operator, 2 RK4 steps, 2 density matrices."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import lindblad_rk4
    N, steps, dt = 1100, 2, 1e-2
    H, cs = olb.synthetic_lindblad(N, nc=1)
    rho0 = olb.random_pure_states(2, N, seed=3)
    ref = olb.lindblad_batch(H, cs, rho0, dt, steps)
    dev = torch.device("cuda", 0)
    rho = torch.from_numpy(rho0.copy()).to(dev)
    lindblad_rk4(torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev), rho, dt, steps)
    assert relerr(rho.cpu().numpy(), ref) < TOL


def test_lindblad_many_collapse_ops_and_observables_match_oracle():
    """LindbladSolver.run with 20 collapse operators and 20 observables (N = 40, 8 steps): observables including t0
    and the final state (oqs._lindblad contract) against the oracle's csr-free restatement."""
    from oracle import lindblad as olb
    from pyqed_amd import LindbladSolver
    N, nc, ne, Nt, dt = 40, 20, 20, 8, 5e-3
    rng = np.random.default_rng(20)
    H, _ = olb.synthetic_lindblad(N, nc=1)
    cs = [0.05 * (rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))) / np.sqrt(N) for _ in range(nc)]
    es = []
    for _ in range(ne):
        a = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
        es.append((a + a.conj().T) / 2)
    rho0 = olb.random_pure_states(1, N, seed=4)[0]
    obs_ref, rholist_ref, rho_ref = olb.lindblad(H, rho0, cs, es, Nt, dt)
    r = LindbladSolver(H, cs).run(rho0, dt=dt, Nt=Nt, e_ops=es)
    assert r.observables.shape == (Nt + 1, ne)
    assert relerr(r.observables, obs_ref) < TOL
    last = r.rholist[-1]
    assert relerr(last.toarray() if hasattr(last, "toarray") else np.asarray(last), rho_ref) < TOL


@pytest.mark.parametrize("N,nc,B,herm", [(64, 40, 4, None), (24, 256, 2, None), (24, 256, 2, False),
                                         (100, 120, 2, None), (100, 120, 20, True)])
def test_glf_many_pairs_batch_matches_oracle(N, nc, B, herm):
    """qd_lindblad_rk4 with up to 256 collapse operators (the kernels' LDS segment tables; round 2 capped them at 16,
    early round 3 at 64): the persistent kernels (N = 24, Hermitian and general), the split-K path (N = 100, B = 2)
    and the Hermitian pair-block split path (N = 100, B = 20) against the oracle."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import lindblad_rk4
    steps, dt = 4, 5e-3
    rng = np.random.default_rng(40)
    H, _ = olb.synthetic_lindblad(N, nc=1)
    cs = np.array([0.3 / np.sqrt(nc) * (rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))) / np.sqrt(N)
                   for _ in range(nc)])
    rho0 = olb.random_pure_states(B, N, seed=5)
    ref = olb.lindblad_batch(H, list(cs), rho0, dt, steps)
    dev = torch.device("cuda", 0)
    rho = torch.from_numpy(rho0.copy()).to(dev)
    lindblad_rk4(torch.from_numpy(H).to(dev), torch.from_numpy(cs).to(dev), rho, dt, steps, hermitian=herm)
    assert relerr(rho.cpu().numpy(), ref) < TOL


def _jump_ops(N, rng, scale=0.05):
    """every |i><j| transition (i != j) with a random rate: N(N - 1) collapse operators (a thermal Lindbladian)."""
    cs = []
    for i in range(N):
        for j in range(N):
            if i != j:
                c = np.zeros((N, N), complex)
                c[i, j] = np.sqrt(scale * rng.uniform(0.1, 1.0) / N)
                cs.append(c)
    return np.array(cs)


@pytest.mark.parametrize("N,nc,B,herm", [(24, 552, 2, False), (24, 552, 3, True), (64, 300, 4, None),
                                         (64, 300, 2, True), (100, 300, 2, None), (100, 300, 2, True)])
def test_lindblad_more_collapse_ops_than_lds_table(N, nc, B, herm):
    """More collapse operators than the kernels' LDS segment table (MAX_NC = 256; round 3 refused the rest,
    VERDICT r03 missing #2): the persistent kernels' CHUNK instantiations (glf_chunk.hip), general and Hermitian,
    Np = 32 / 64 / 128, against the oracle's sum over the whole list (oqs.py:697-714).  N = 24 runs every |i><j|
    jump operator (552)."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import lindblad_rk4
    steps, dt = 3, 5e-3
    rng = np.random.default_rng(41)
    H, _ = olb.synthetic_lindblad(N, nc=1)
    if nc == N * (N - 1):
        cs = _jump_ops(N, rng)
    else:
        cs = np.array([0.3 / np.sqrt(nc) * (rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
                       / np.sqrt(N) for _ in range(nc)])
    rho0 = olb.random_pure_states(B, N, seed=6)
    ref = olb.lindblad_batch(H, list(cs), rho0, dt, steps)
    dev = torch.device("cuda", 0)
    rho = torch.from_numpy(rho0.copy()).to(dev)
    lindblad_rk4(torch.from_numpy(H).to(dev), torch.from_numpy(cs).to(dev), rho, dt, steps, hermitian=herm)
    assert relerr(rho.cpu().numpy(), ref) < TOL
    # trace is conserved by every Lindbladian
    tr = np.einsum("bii->b", rho.cpu().numpy())
    assert np.max(np.abs(tr - 1.0)) < 1e-12
