"""Redfield propagation (GLF kernel), basis transforms and 2DES response kernels vs golden/oracle."""
import numpy as np
import pytest

from conftest import SPECTRA, load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.mark.parametrize("name", ["redfield_n4", "redfield_n6_k2"])
def test_redfield_evolve_matches_reference(name):
    from pyqed_amd import RedfieldSolver
    g = load_golden(name)
    nk = len(g["a_ops"])
    sol = RedfieldSolver(g["H"], c_ops=list(g["a_ops"]), spectra=[SPECTRA[str(g["spectrum"])]] * nk)
    R, evecs = sol.redfield_tensor()
    assert relerr(R.toarray(), g["R"]) < 1e-12
    r = sol.evolve(g["rho0"], dt=float(g["dt"]), Nt=int(g["Nt"]), e_ops=list(g["E"]))
    assert r.observables.shape == g["observables"].shape
    assert relerr(r.observables, g["observables"]) < TOL
    assert relerr(np.array(r.rholist), g["rholist"]) < TOL


def test_redfield_propagator_eom_and_gf_match_reference():
    """propagator(t, 'EOM') = phys.expm(R, t) (RK4 of the identity, oqs.py:185-200, phys.py:2049-2097) on the
    batched dense-superoperator kernel, gf(t, 'EOM') = -1j of it, and gf(t, 'eseries') = getG(1j R, t)
    (oqs.py:136-158, 465-508), against the reference's outputs; 'SOS' agrees with 'EOM' to the RK4 truncation error (3e-5 here)."""
    from pyqed_amd import RedfieldSolver
    g = load_golden("redfield_eom")
    sol = RedfieldSolver(g["H"], c_ops=list(g["a_ops"]), spectra=[SPECTRA[str(g["spectrum"])]])
    sol.redfield_tensor()
    t = g["t"]
    U = sol.propagator(t, method="EOM")
    assert U.shape == g["U_eom"].shape
    assert relerr(U, g["U_eom"]) < TOL
    assert relerr(sol.G, -1j * g["U_eom"]) < TOL
    assert relerr(sol.gf(t, method="EOM"), -1j * g["U_eom"]) < TOL
    assert relerr(sol.gf(t, method="eseries"), g["G_eseries"]) < 1e-9
    # the reference's gf never forwards `domain` to getG (time domain whatever is asked)
    assert relerr(sol.gf(t, method="eseries", domain="freq"), g["G_eseries"]) < 1e-9
    U_sos = sol.propagator(t, method="SOS")
    assert relerr(U_sos, g["U_eom"]) < 1e-4   # RK4 truncation at dt = 0.05
    with pytest.raises(NotImplementedError):
        sol.propagator(t, method="krylov")


def test_basis_transform_batched():
    import torch
    from pyqed_amd.oqs import basis_transform
    rng = np.random.default_rng(5)
    for N, B in [(5, 3), (40, 2), (130, 2)]:
        V = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))[0]
        A = rng.standard_normal((B, N, N)) + 1j * rng.standard_normal((B, N, N))
        dev = torch.device("cuda", 0)
        At = torch.from_numpy(A.copy()).to(dev)
        Vt = torch.from_numpy(V).to(dev)
        basis_transform(Vt, At, inverse=False)
        ref = np.einsum("ji,bjk,kl->bil", V.conj(), A, V)
        assert relerr(At.cpu().numpy(), ref) < 1e-13
        basis_transform(Vt, At, inverse=True)
        assert relerr(At.cpu().numpy(), A) < 1e-13


def test_propagator_and_cube_match_reference():
    from pyqed_amd import RedfieldSolver
    g = load_golden("corr4_3level")
    dip = g["dip"]
    for sig in ["lccc", "llll", "lrlr"]:
        sol = RedfieldSolver(g["H"], c_ops=[g["a_op"]], spectra=[SPECTRA["flat005"]])
        sol.redfield_tensor()
        sol.propagator(g["tau16"])
        cube = sol.correlation_4op_3t(g["rho0"], [dip] * 4, sig, g["tau16"])
        assert cube.shape == (16, 16, 16)
        assert relerr(cube, g["cube_" + sig]) < TOL, sig
    sol = RedfieldSolver(g["H"], c_ops=[g["a_op"]], spectra=[SPECTRA["flat005"]])
    sol.redfield_tensor()
    U = sol.propagator(g["tau64"])
    assert relerr(U[:, :, 7], g["U64_k7"]) < TOL
    cube = sol.correlation_4op_3t(g["rho0"], [dip] * 4, "lccc", g["tau64"])
    assert relerr(cube[:, 0, :], g["slice64_j0"]) < TOL
    assert relerr(cube[:, 5, :], g["slice64_j5"]) < TOL


def _ensemble_inputs(E_list, t2):
    from pyqed_amd.response import ensemble_factors, redfield_superop_batch, sos_eig
    from pyqed_amd.superoperator import operator_to_superoperator
    N = 3
    dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
    a = np.diag([0.0, 1.0, 2.0])
    rho0 = np.zeros((3, 3), complex); rho0[0, 0] = 1
    E = np.asarray(E_list)
    spec = np.full((len(E), N, N), 0.05)
    R = redfield_superop_batch(E, a, spec)
    lam, U1 = np.linalg.eig(R)
    U2 = np.linalg.inv(U1)
    ops = [operator_to_superoperator(dip, s).toarray() for s in "lccc"]
    return lam, ensemble_factors(lam, U1, U2, ops, rho0.flatten(), t2)


def test_ensemble_slice_matches_reference():
    from pyqed_amd.response import response2d_ensemble
    g = load_golden("corr4_ensemble")
    tau = g["tau"]
    j = int(g["j"])
    lam, (alpha, Mt, beta) = _ensemble_inputs(g["E"], tau[j])
    # member by member
    for m in range(len(g["E"])):
        S = response2d_ensemble(lam[m:m + 1], alpha[m:m + 1], Mt[m:m + 1], beta[m:m + 1], tau, tau)
        assert relerr(S.cpu().numpy(), g["slices"][m]) < TOL
    S = response2d_ensemble(lam, alpha, Mt, beta, tau, tau)
    assert relerr(S.cpu().numpy(), g["ens_sum"]) < TOL


def test_ensemble_large_linearity_and_shards():
    """Size-independent properties at bench scale: sum of shard results == full result,
    and a doubled ensemble gives twice the signal (linearity)."""
    import torch
    from pyqed_amd.response import response2d_ensemble
    rng = np.random.default_rng(7)
    M = 512
    E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((M, 3))
    t = 0.5 * np.arange(256)
    lam, (alpha, Mt, beta) = _ensemble_inputs(E, 0.0)
    full = response2d_ensemble(lam, alpha, Mt, beta, t, t)
    part = None
    for sl in [slice(0, 100), slice(100, 333), slice(333, M)]:
        part = response2d_ensemble(lam[sl], alpha[sl], Mt[sl], beta[sl], t, t, out=part, accumulate=part is not None)
    assert relerr(part.cpu().numpy(), full.cpu().numpy()) < 1e-13
    dbl = response2d_ensemble(np.concatenate([lam, lam]), np.concatenate([alpha, alpha]),
                              np.concatenate([Mt, Mt]), np.concatenate([beta, beta]), t, t)
    assert relerr(dbl.cpu().numpy(), 2 * full.cpu().numpy()) < 1e-13
    # spot-check a few members' exact slice against the closed form
    from oracle import redfield as orf
    m = 17
    X = alpha[m][None, :] * np.exp(np.outer(t, lam[m]))
    Y = beta[m][None, :] * np.exp(np.outer(t, lam[m]))
    ref = (-1j) ** 3 * X @ Mt[m] @ Y.T
    one = response2d_ensemble(lam[m:m + 1], alpha[m:m + 1], Mt[m:m + 1], beta[m:m + 1], t, t)
    assert relerr(one.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("M,grid", [(1000, "uniform"), (1001, "uniform"), (2048, "uniform"), (1000, "array")])
def test_ensemble_gemm64_matches_closed_form(M, grid):
    """The 64-block ensemble GEMM (operand loads two K-tiles ahead) against the closed form summed over every member:
    M = 1000 gives workgroups with odd and even K-tile counts, M = 1001 a K that is not a multiple of the K-tile; uniform
    grids build X and Z from exponential tables, an array grid from the time arrays."""
    from pyqed_amd.response import response2d_ensemble
    from conftest import took
    rng = np.random.default_rng(M)
    E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((M, 3))
    t = 0.5 * np.arange(256)
    lam, (alpha, Mt, beta) = _ensemble_inputs(E, 0.0)
    took("")
    import torch
    tg = t if grid == "uniform" else torch.from_numpy(t + 1e-3 * np.sin(np.arange(256))).cuda()
    got = response2d_ensemble(lam, alpha, Mt, beta, tg, t).cpu().numpy()
    hit, paths = took("ens_gemm64")
    assert hit, paths
    t3 = t if grid == "uniform" else tg.cpu().numpy()
    X = alpha[:, None, :] * np.exp(t3[None, :, None] * lam[:, None, :])     # [M][n3][K]
    Y = beta[:, None, :] * np.exp(t[None, :, None] * lam[:, None, :])       # [M][n1][K]
    ref = (-1j) ** 3 * np.einsum("mik,mkl,mjl->ij", X, Mt, Y, optimize=True)
    assert relerr(got, ref) < TOL


@pytest.mark.parametrize("name", ["redfield_n4", "redfield_n6_k2"])
def test_redfield_dense_superop_path(name):
    """Module-level _redfield(R, ...) (oqs.py:364-459) on the HBM-bound dense-superoperator kernel."""
    from pyqed_amd.oqs import _redfield
    g = load_golden(name)
    r = _redfield(g["R"], g["rho0"], evecs=g["evecs"], Nt=int(g["Nt"]), dt=float(g["dt"]), e_ops=list(g["E"]))
    assert relerr(r.observables, g["observables"]) < TOL
    assert relerr(np.array(r.rholist), g["rholist"]) < TOL


def test_superop_batch_vs_glf():
    """Dense L.vec(rho) (Lindblad superoperator, N=24, B=6 -> two groups of <=4) vs the GLF kernel."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import lindblad_rk4
    from pyqed_amd.oqs import superop_rk4
    from pyqed_amd.superoperator import liouvillian
    N, B = 24, 6
    H, cs = olb.synthetic_lindblad(N)
    L = liouvillian(H, cs).toarray()
    rho0 = olb.random_pure_states(B, N)
    dev = torch.device("cuda", 0)
    v = torch.from_numpy(rho0.reshape(B, N * N).copy()).to(dev)
    superop_rk4(torch.from_numpy(L).to(dev), v, 0.01, 20)
    rho = torch.from_numpy(rho0.copy()).to(dev)
    lindblad_rk4(torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev), rho, 0.01, 20)
    assert relerr(v.cpu().numpy().reshape(B, N, N), rho.cpu().numpy()) < 1e-12


@pytest.mark.parametrize("M,nL,n3,n1", [(3, 20, 70, 40), (5, 9, 130, 257)])
def test_ensemble_slice_formula_generic_sizes(M, nL, n3, n1):
    """Direct evaluation of S[i,k] = (-i)^3 sum_m sum_pq alpha_mp e^{lam_mp t3_i} Mt_mpq beta_mq e^{lam_mq t1_k}:
    nL > 16 takes the generic Z path; ragged n3/n1 exercise the block padding."""
    from pyqed_amd.response import response2d_ensemble
    rng = np.random.default_rng(nL)
    lam = -rng.uniform(0.01, 0.2, (M, nL)) + 1j * rng.uniform(-2, 2, (M, nL))
    alpha = rng.standard_normal((M, nL)) + 1j * rng.standard_normal((M, nL))
    beta = rng.standard_normal((M, nL)) + 1j * rng.standard_normal((M, nL))
    Mt = rng.standard_normal((M, nL, nL)) + 1j * rng.standard_normal((M, nL, nL))
    t3 = 0.3 * np.arange(n3)
    t1 = 0.25 * np.arange(n1)
    ref = np.zeros((n3, n1), complex)
    for m in range(M):
        X = alpha[m][None, :] * np.exp(np.outer(t3, lam[m]))
        Z = (Mt[m] * beta[m][None, :]) @ np.exp(np.outer(lam[m], t1))
        ref += X @ Z
    ref *= (-1j) ** 3
    S = response2d_ensemble(lam, alpha, Mt, beta, t3, t1).cpu().numpy()
    assert relerr(S, ref) < 1e-12


def test_ensemble_uniform_tables_vs_array_path():
    """Uniform host grids take the exponential-table operand build; device-tensor grids take the direct
    exponentials.  Same result to ~1e-14; a non-uniform grid stays on the array path."""
    import torch
    from pyqed_amd.response import _uniform, response2d_ensemble
    rng = np.random.default_rng(11)
    M, nL = 64, 9
    lam = -rng.uniform(0.01, 0.2, (M, nL)) + 1j * rng.uniform(-2, 2, (M, nL))
    alpha = rng.standard_normal((M, nL)) + 1j * rng.standard_normal((M, nL))
    beta = rng.standard_normal((M, nL)) + 1j * rng.standard_normal((M, nL))
    Mt = rng.standard_normal((M, nL, nL)) + 1j * rng.standard_normal((M, nL, nL))
    t = 0.5 * np.arange(200)
    assert _uniform(t) == (0.0, 0.5)
    dev = torch.device("cuda", 0)
    uni = response2d_ensemble(lam, alpha, Mt, beta, t, t).cpu().numpy()
    arr = response2d_ensemble(lam, alpha, Mt, beta, torch.from_numpy(t).to(dev), torch.from_numpy(t).to(dev))
    assert relerr(uni, arr.cpu().numpy()) < 1e-13
    tn = np.sort(rng.uniform(0, 60, 150))
    assert _uniform(tn) is None
    S = response2d_ensemble(lam[:3], alpha[:3], Mt[:3], beta[:3], tn, t).cpu().numpy()
    ref = sum((alpha[m][None, :] * np.exp(np.outer(tn, lam[m]))) @
              ((Mt[m] * beta[m][None, :]) @ np.exp(np.outer(lam[m], t))) for m in range(3)) * (-1j) ** 3
    assert relerr(S, ref) < 1e-12


def test_t2scan_matches_reference_cube():
    """Waiting-time scan, one member: out[j, i, k] == correlation_4op_3t cube[i, j, k] of the reference."""
    from pyqed_amd.response import eigen_factors, response2d_t2scan, sos_eig
    g = load_golden("corr4_3level")
    lam, U1, U2 = sos_eig(g["R"])
    tau = g["tau16"]
    for sig in ["lccc", "llll", "lrlr"]:
        alpha, B, C, beta = eigen_factors(lam, U1, U2, [g["dip"]] * 4, sig, g["rho0"])
        S = response2d_t2scan(lam[None], alpha[None], B[None], C[None], beta[None], tau, tau, tau).cpu().numpy()
        assert S.shape == (16, 16, 16)
        assert relerr(S.transpose(1, 0, 2), g["cube_" + sig]) < TOL, sig


@pytest.mark.parametrize("M,n3,n1", [(300, 200, 256), (7, 130, 40)])
def test_t2scan_equals_per_t2_ensemble(M, n3, n1):
    """Every waiting time of the scan equals the fixed-t2 ensemble slice (Mt built on the host); shard
    accumulation over members equals the full scan."""
    import torch
    from pyqed_amd.response import (ensemble_factors, ensemble_factors_bc, redfield_superop_batch,
                                    response2d_ensemble, response2d_t2scan)
    from pyqed_amd.superoperator import operator_to_superoperator
    rng = np.random.default_rng(M)
    E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((M, 3))
    R = redfield_superop_batch(E, np.diag([0.0, 1.0, 2.0]), np.full((M, 3, 3), 0.05))
    lam, U1 = np.linalg.eig(R)
    U2 = np.linalg.inv(U1)
    dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
    ops = [operator_to_superoperator(dip, s).toarray() for s in "lccc"]
    rho0v = np.zeros(9, complex); rho0v[0] = 1
    alpha, B, C, beta = ensemble_factors_bc(lam, U1, U2, ops, rho0v)
    t3, t1 = 0.5 * np.arange(n3), 0.4 * np.arange(n1)
    t2 = np.array([0.0, 1.3, 4.0, 25.0])
    scan = response2d_t2scan(lam, alpha, B, C, beta, t3, t2, t1).cpu().numpy()
    for j, tj in enumerate(t2):
        a2, Mt, b2 = ensemble_factors(lam, U1, U2, ops, rho0v, tj)
        ref = response2d_ensemble(lam, a2, Mt, b2, t3, t1).cpu().numpy()
        assert relerr(scan[j], ref) < 1e-12, j
    dev = torch.device("cuda", 0)
    part = torch.zeros((len(t2), n3, n1), dtype=torch.complex128, device=dev)
    cut = [0, M // 3, M]
    for lo, hi in zip(cut[:-1], cut[1:]):
        response2d_t2scan(lam[lo:hi], alpha[lo:hi], B[lo:hi], C[lo:hi], beta[lo:hi], t3, t2, t1, out=part,
                          accumulate=True)
    assert relerr(part.cpu().numpy(), scan) < 1e-13


def test_t2scan_prepared_operands_buckets():
    """T2Scan: operands once, waiting times applied in buckets == the one-shot scan."""
    from pyqed_amd.response import T2Scan, response2d_t2scan
    rng = np.random.default_rng(21)
    M, nL = 50, 9
    lam = -rng.uniform(0.01, 0.2, (M, nL)) + 1j * rng.uniform(-2, 2, (M, nL))
    alpha, beta = (rng.standard_normal((M, nL)) + 1j * rng.standard_normal((M, nL)) for _ in range(2))
    B, C = (rng.standard_normal((M, nL, nL)) + 1j * rng.standard_normal((M, nL, nL)) for _ in range(2))
    t3, t1, t2 = 0.5 * np.arange(140), 0.3 * np.arange(200), np.array([0.0, 0.7, 3.1, 9.0, 20.0])
    full = response2d_t2scan(lam, alpha, B, C, beta, t3, t2, t1).cpu().numpy()
    sc = T2Scan(lam, alpha, B, C, beta, t3, t1)
    parts = np.concatenate([sc.apply(t2[:2]).cpu().numpy(), sc.apply(t2[2:]).cpu().numpy()])
    assert relerr(parts, full) < 1e-14
    # closed form for one waiting time
    j = 3
    ref = sum((alpha[m][None, :] * np.exp(np.outer(t3, lam[m]))) @ (B[m] * np.exp(lam[m] * t2[j])[None, :]) @ C[m]
              @ (beta[m][:, None] * np.exp(np.outer(lam[m], t1))) for m in range(M)) * (-1j) ** 3
    assert relerr(full[j], ref) < 1e-12


@pytest.mark.parametrize("N,nk,B,spec", [(40, 1, 3, "flat005"), (128, 2, 4, "flat005"), (128, 1, 3, "tanh"),
                                         (64, 2, 2, "tanh")])
def test_redfield_hermitian_glf_matches_general(N, nk, B, spec):
    """qd_glf_rk4_herm (X + X^+, X = P rho + sum A rho Lam^+) == qd_glf_rk4 with the full (P, Q, pairs) form.  With a
    frequency-dependent spectrum (tanh) sum A rho Lam^+ is not Hermitian, so the Lindblad-only skip of its lower-left
    block must stay off (N = 128: 128-blocks)."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import RedfieldSolver
    from pyqed_amd.oqs import glf_rk4
    rng = np.random.default_rng(N + nk)
    a = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = (a + a.conj().T) / 2 / np.sqrt(N)
    a_ops = []
    for _ in range(nk):
        x = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
        a_ops.append(0.2 * (x + x.conj().T) / 2 / np.sqrt(N))
    sol = RedfieldSolver(H, c_ops=a_ops, spectra=[SPECTRA[spec]] * nk)
    sol.redfield_tensor()
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(np.asarray(x, complex))).to(dev)
    P, Q, Ls, Rs = sol.glf_terms()
    Ph, Lh, Wh = sol.glf_terms_herm()
    rho0 = olb.random_pure_states(B, N, seed=N)
    r1, r2 = t(rho0), t(rho0)
    glf_rk4(t(P), t(Q), t(Ls), t(Rs), r1, 0.02, 30)
    glf_rk4(t(Ph), None, t(Lh), t(Wh), r2, 0.02, 30, hermitian=True)
    a1, a2 = r1.cpu().numpy(), r2.cpu().numpy()
    assert relerr(a2, a1) < 1e-12
    assert np.array_equal(a2, np.conj(np.swapaxes(a2, -1, -2)))      # exactly Hermitian


def test_redfield_evolve_non_hermitian_input_general_path():
    """A non-Hermitian rho0 (e.g. a coherence C rho0 A of a response function) takes the general GLF kernel."""
    from oracle import redfield as orf
    from pyqed_amd import RedfieldSolver
    g = load_golden("redfield_n4")
    rng = np.random.default_rng(3)
    r0 = rng.standard_normal((4, 4)) + 1j * rng.standard_normal((4, 4))
    sol = RedfieldSolver(g["H"], c_ops=list(g["a_ops"]), spectra=[SPECTRA[str(g["spectrum"])]])
    R, evecs = sol.redfield_tensor()
    r = sol.evolve(r0, dt=float(g["dt"]), Nt=int(g["Nt"]), e_ops=list(g["E"]))
    obs, rholist = orf.redfield_evolve(R.toarray(), r0, evecs, int(g["Nt"]), float(g["dt"]), list(g["E"]))
    assert relerr(r.observables, obs) < TOL
    assert relerr(np.array(r.rholist), np.array(rholist)) < TOL


def test_redfield_return_result_false_writes_obs_dat(tmp_path, monkeypatch):
    """oqs._redfield(return_result=False) (oqs.py:406-431): 'obs.dat' holds one time stamp per step (t after
    the increment), the final vec(rho) is returned; any e_op fails as in the reference (obs_dm of a vector)."""
    from pyqed_amd.oqs import _redfield
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(4)
    N = 3
    R = 0.3 * (rng.standard_normal((N * N, N * N)) + 1j * rng.standard_normal((N * N, N * N)))
    rho0 = np.diag([1.0, 0.0, 0.0]).astype(complex)
    v = _redfield(R, rho0, Nt=7, dt=0.01, t0=0.5, return_result=False)
    full = _redfield(R, rho0, Nt=7, dt=0.01, t0=0.5)
    assert v.shape == (N * N,) and relerr(v.reshape(N, N), full.rholist[-1]) < 1e-13
    lines = open(tmp_path / "obs.dat").read().splitlines()
    t, ts = 0.5, []
    for _ in range(7):
        t += 0.01
        ts.append(f"{t} ")
    assert lines == ts
    with pytest.raises(ValueError):
        _redfield(R, rho0, Nt=2, dt=0.01, e_ops=[np.eye(N)], return_result=False)
