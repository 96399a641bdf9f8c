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


def _pulse(p):
    from pyqed_amd.optics import Pulse
    return Pulse(omegac=p[0], tau=p[1], tc=p[2], amplitude=p[3])


def test_driven_sesolver_single_pulse():
    """SESolver.run(pulse=..., edip=2D) -> driven_dynamics (mol.py:1430-1456, 1862-1958)."""
    from scipy.sparse import issparse
    from pyqed_amd.mol import SESolver
    g = load_golden("tdse_driven")
    r = SESolver(g["a_H"]).run(psi0=g["a_psi0"], dt=float(g["a_dt"]), Nt=int(g["a_Nt"]), e_ops=list(g["a_E"]),
                               nout=int(g["a_nout"]), edip=g["a_d"], pulse=_pulse(g["a_pulse"]))
    assert r.observables.shape == g["a_obs"].shape
    assert relerr(r.observables, g["a_obs"]) < TOL
    assert relerr(r.psi, g["a_psit"]) < TOL
    assert all(issparse(x) for x in r.psilist[1:])  # csr columns, as the reference's sparse psi
    got = np.array([np.asarray(x.toarray() if issparse(x) else x).reshape(-1) for x in r.psilist])
    assert relerr(got, g["a_psilist"]) < TOL


def test_driven_sesolver_vector_dipole():
    """SESolver.run(edip=[N, N, 3], pulse with a vector field .E) -> mol._driven_dynamics (mol.py:1441-1445,
    1772-1859): the three dipole components are the drives of qd_tdse_driven_rk4; psilist holds only the block
    states (csr), observables include t0."""
    from scipy.sparse import issparse
    from pyqed_amd.mol import SESolver
    g = load_golden("tdse_driven3d")
    fp = g["field"]

    class VPulse:
        def E(self, t):
            amp, om, tc, tau = fp[:, 0], fp[:, 1], fp[:, 2], fp[:, 3]
            return amp * np.cos(om * t) * np.exp(-((t - tc) / tau) ** 2)

    r = SESolver(g["H"]).run(psi0=g["psi0"], dt=float(g["dt"]), Nt=int(g["Nt"]), e_ops=list(g["E"]),
                             nout=int(g["nout"]), edip=g["edip"], pulse=VPulse())
    assert r.observables.shape == g["obs"].shape
    assert relerr(r.observables, g["obs"]) < TOL
    assert relerr(r.psi, g["psit"]) < TOL
    assert len(r.psilist) == len(g["psilist"]) and all(issparse(x) for x in r.psilist)
    got = np.array([np.asarray(x.toarray()).reshape(-1) for x in r.psilist])
    assert relerr(got, g["psilist"]) < TOL


def test_driven_mol_two_pulses():
    """Mol.run(pulse=[p1, p2]) with self.edip a list of dipoles, t0 != 0 (mol.py:660-675)."""
    from pyqed_amd.mol import Mol
    g = load_golden("tdse_driven")
    pulses = [_pulse(p) for p in g["b_pulse"]]
    r = Mol(g["b_H"], edip=list(g["b_d"])).run(psi0=g["b_psi0"], dt=float(g["b_dt"]), e_ops=list(g["b_E"]),
                                                 nt=int(g["b_Nt"]), nout=int(g["b_nout"]), t0=float(g["b_t0"]),
                                                 pulse=pulses)
    assert relerr(r.observables, g["b_obs"]) < TOL
    assert relerr(r.psi, g["b_psit"]) < TOL
    got = np.array([np.asarray(x.toarray() if hasattr(x, "toarray") else x).reshape(-1) for x in r.psilist])
    assert relerr(got, g["b_psilist"]) < TOL


@pytest.mark.parametrize("N,B", [(40, 3), (512, 64)])
def test_driven_batch_vs_oracle(N, B):
    """Batched driven kernel vs the oracle for several wavefunctions, nout > 1; (512, 64) takes the MFMA GEMM
    stage path of the driven run."""
    import torch
    from oracle import tdse as ot
    from pyqed_amd.mol import tdse_driven_rk4
    rng = np.random.default_rng(5)
    nout, nblk, dt = 4, 6, 0.03
    A = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H0 = (A + A.conj().T) / 2 / np.sqrt(N)
    Hd = np.array([np.diag(np.arange(N) / N).astype(complex)])
    f = ot.gaussian_efield(1.0, 0.5, 0.3, 0.5)
    fvals = np.array([[f(k * dt * nout)] for k in range(nblk)], dtype=complex)
    psi0 = rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))
    psi0 /= np.linalg.norm(psi0, axis=1, keepdims=True)
    dev = torch.device("cuda", 0)
    psi = torch.from_numpy(psi0.copy()).to(dev)
    E = torch.from_numpy(np.array([H0])).to(dev)
    snap, obs = tdse_driven_rk4(torch.from_numpy(H0).to(dev), torch.from_numpy(Hd).to(dev), fvals, psi, dt, nout,
                                e_ops=E)
    for b in range(B):
        o, psit, _ = ot.driven_dynamics(H0, [(Hd[0], f)], psi0[b], dt, (nblk + 1) * nout, [H0], nout)
        assert relerr(obs[b].cpu().numpy(), o) < TOL
        assert relerr(snap[b].cpu().numpy(), psit[:, 1:].T) < TOL


@pytest.mark.parametrize("N,B,save_every,path", [(300, 1, 2, "tdse_rows"), (2500, 2, 3, "tdse_rows"),
                                                  (1024, 64, 5, "tdse_gemm"), (600, 130, 2, "tdse_gemm"),
                                                  (1024, 8, 2, "tdse_rows")])
def test_tdse_row_and_gemm_paths_vs_oracle(N, B, save_every, path):
    """The row path (a wave per row and stage launch) and, where tdse.hip's dispatch takes it ((B >= 64 and N >= 512)
    or (B >= 128 and N >= 256)), the MFMA GEMM stages (padded [Bp][Np] state, split-K slabs): snapshots and
    observables (E_m = H, diag) against the oracle's RK4 (oracle.tdse restates mol.py:1603-1691); B = 64 / 130 and
    N = 600 exercise the GEMM's padding to multiples of 128."""
    import torch
    from oracle import tdse as otd
    from pyqed_amd.mol import tdse_rk4
    from conftest import took
    rng = np.random.default_rng(N + B)
    A = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = (A + A.conj().T) / 2 / np.sqrt(N)
    Ed = np.diag(np.linspace(0, 1, N)).astype(complex)
    psi0 = rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))
    psi0 /= np.linalg.norm(psi0, axis=1, keepdims=True)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    steps, dt = 6, 0.02
    took("")
    psi = t(psi0.copy())
    snap, obs = tdse_rk4(t(H), psi, dt, steps, save_every=save_every, e_ops=t(np.array([H, Ed])))
    hit, got = took(path)
    assert hit, got
    out = {"1": (psi.cpu().numpy(), snap.cpu().numpy(), obs.cpu().numpy())}
    psi, snap, obs = out["1"]
    ref = psi0[0].copy()
    for s in range(steps):
        ref = otd._rk4(ref, H, dt)
        if (s + 1) % save_every == 0:
            assert relerr(snap[0][(s + 1) // save_every - 1], ref) < 1e-12
    assert relerr(psi[0], ref) < 1e-12
    e0 = np.vdot(psi0[0], H @ psi0[0])
    assert abs(obs[0, 0, 0] - e0) < 1e-12 * max(1, abs(e0))
    assert np.allclose(np.linalg.norm(psi, axis=1), 1, atol=1e-10)
