"""TDSE RK4 (qd_tdse_rk4) behind SESolver / Mol.run vs reference golden vectors."""
import numpy as np
import pytest

from conftest import load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-11


@pytest.mark.parametrize("tag", ["a", "b"])
def test_sesolver_and_mol_run(tag):
    from pyqed_amd.mol import Mol, SESolver
    g = load_golden("sesolver")
    H, E, psi0 = g[f"{tag}_H"], list(g[f"{tag}_E"]), g[f"{tag}_psi0"]
    Nt, nout, dt = int(g[f"{tag}_Nt"]), int(g[f"{tag}_nout"]), float(g[f"{tag}_dt"])
    r = SESolver(H).run(psi0=psi0, dt=dt, Nt=Nt, e_ops=E, nout=nout)
    assert r.observables.shape == g[f"{tag}_obs"].shape
    assert relerr(r.observables, g[f"{tag}_obs"]) < TOL
    assert len(r.psilist) == len(g[f"{tag}_psilist"])
    assert relerr(np.array(r.psilist), g[f"{tag}_psilist"]) < TOL
    assert np.allclose(r.times, g[f"{tag}_times"])
    r2 = Mol(H).run(psi0=psi0, dt=dt, e_ops=E, nt=Nt, nout=nout)
    assert relerr(r2.observables, g[f"{tag}_obs"]) < TOL


def test_tdse_batch_norm_large():
    import torch
    from pyqed_amd.mol import tdse_rk4
    rng = np.random.default_rng(3)
    N, B = 1024, 3
    A = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = (A + A.conj().T) / 2 / np.sqrt(N)
    psi0 = rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))
    psi0 /= np.linalg.norm(psi0, axis=1, keepdims=True)
    dev = torch.device("cuda", 0)
    psi = torch.from_numpy(psi0.copy()).to(dev)
    tdse_rk4(torch.from_numpy(H).to(dev), psi, 0.01, 50)
    out = psi.cpu().numpy()
    # exact propagator
    w, U = np.linalg.eigh(H)
    ref = (U @ (np.exp(-1j * w * 0.5)[:, None] * (U.conj().T @ psi0.T))).T
    assert relerr(out, ref) < 1e-8          # RK4 truncation at dt = 0.01, |H| ~ 2
    assert np.max(np.abs(np.linalg.norm(out, axis=1) - 1)) < 1e-9
