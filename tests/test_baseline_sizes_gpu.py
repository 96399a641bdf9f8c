"""Parity at the exact BASELINE.json sizes: the HIP path against reference outputs
generated at the benchmarked size (tests/golden/make_golden.py: redfield_n128, corr4_2des_256, spo2_256;
lindblad_n128_long and deom_run_bench_long are in test_lindblad_gpu.py / test_deom_gpu.py).  fp64 results with
a different summation order than the reference: 1e-10 relative (L2), inside north_star's 1e-8."""
import numpy as np
import pytest

from conftest import SPECTRA, load_golden, relerr

TOL = 1e-10


@pytest.mark.gpu
def test_redfield_n128_evolve_matches_reference():
    """Config d1, Redfield half: N = 128, 6 RK4 steps of RedfieldSolver.evolve (oqs.py:57-81, 364-459) against the
    reference's csr R . vec(rho) propagation (replaces the round-1 Hermitian-vs-general self-comparison)."""
    from pyqed_amd import RedfieldSolver
    g = load_golden("redfield_n128")
    sol = RedfieldSolver(g["H"], c_ops=[g["a_op"]], spectra=[SPECTRA[str(g["spectrum"])]])
    r = sol.evolve(g["rho0"], dt=float(g["dt"]), Nt=int(g["Nt"]), e_ops=list(g["E"]))
    assert r.observables.shape == g["observables"].shape
    assert relerr(r.observables, g["observables"]) < TOL
    assert relerr(r.rholist[-1], g["rho_final"]) < TOL


@pytest.mark.gpu
def test_lindblad_n128_b256_headline_dispatch_matches_oracle():
    """The benched headline instantiation itself: N = 128, n_c = 1, B = 256 pure states, the
    bench's seeded inputs and dt, auto dispatch (exactly Hermitian states -> the persistent Hermitian kernel
    lindblad_rk4_kernel<128, true, true>), 5 RK4 steps, against the oracle's RK4 of oqs.liouvillian (oqs.py:697-714,
    1596-1696) on a spread of the 256 matrices, first and last included."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import lindblad_rk4
    N, B, steps, dt = 128, 256, 5, 1e-3
    H, cs = olb.synthetic_lindblad(N, nc=1)
    rho0 = olb.random_pure_states(B, N, seed=2)
    sel = [0, 1, 63, 64, 127, 128, 200, 255]
    ref = olb.lindblad_batch(H, cs, rho0[sel], dt, steps)
    dev = torch.device("cuda", 0)
    rho = torch.from_numpy(rho0.copy()).to(dev)
    lindblad_rk4(torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev), rho, dt, steps)
    got = rho.cpu().numpy()
    assert relerr(got[sel], ref) < 1e-12
    assert np.array_equal(got, np.conj(np.swapaxes(got, 1, 2)))   # every stage exactly Hermitian


def test_redfield_n128_tensor_rows_match_reference():
    """Host setup at N = 128 (no GPU): rows of the reference's csr R (oqs.py:519-570) from this package's GLF
    operands, R[(a,b),(c,d)] = P[a,c] d_bd + d_ac Q[d,b] + sum_k L_k[a,c] R_k[d,b] (row-major vec, SURVEY §8
    conventions).  The eigenbasis comes from the same LAPACK eigh as the reference's, so the rows agree."""
    from pyqed_amd import RedfieldSolver
    g = load_golden("redfield_n128")
    sol = RedfieldSolver(g["H"], c_ops=[g["a_op"]], spectra=[SPECTRA[str(g["spectrum"])]])
    P, Q, Ls, Rs = sol.glf_terms()
    N = P.shape[0]
    assert relerr(np.abs(sol.evecs), np.abs(g["evecs"])) < 1e-12
    eye = np.eye(N)
    for row, want in zip(g["R_row_index"], g["R_rows"]):
        a, b = divmod(int(row), N)
        got = np.outer(P[a], eye[b]) + np.outer(eye[a], Q[:, b])
        for L, R in zip(Ls, Rs):
            got = got + np.outer(L[a], R[:, b])
        assert relerr(got.reshape(-1), want) < 1e-12, row


def _two_des_members(g):
    from pyqed_amd.response import ensemble_factors, redfield_superop_batch
    from pyqed_amd.superoperator import operator_to_superoperator
    dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
    a = np.diag([0.0, 1.0, 2.0])
    rho0 = np.zeros((3, 3), complex); rho0[0, 0] = 1
    E = g["E"]
    R = redfield_superop_batch(E, a, np.full((len(E), 3, 3), 0.05))
    lam, U1 = np.linalg.eig(R)
    U2 = np.linalg.inv(U1)
    ops = [operator_to_superoperator(dip, s).toarray() for s in "lccc"]
    return lam, U1, U2, ops, rho0


@pytest.mark.gpu
def test_2des_256_cube_slices_match_reference():
    """Config d5 grid (256 x 256, tau = 0.5 arange(256)): RedfieldSolver.correlation_4op_3t (oqs.py:268-357) on the
    GPU, (t3, t1) slices at t2 index 0 and 37, for the unperturbed ladder and two disorder members."""
    from pyqed_amd import RedfieldSolver
    g = load_golden("corr4_2des_256")
    tau = g["tau"]
    for m, E in enumerate(g["E"]):
        H = np.diag(E)
        dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
        rho0 = np.zeros((3, 3), complex); rho0[0, 0] = 1
        sol = RedfieldSolver(H, c_ops=[np.diag([0.0, 1.0, 2.0])], spectra=[SPECTRA["flat005"]])
        sol.redfield_tensor()
        sol.propagator(tau)
        cube = sol.correlation_4op_3t(rho0, [dip] * 4, "lccc", tau)
        assert cube.shape == (256, 256, 256)
        assert relerr(cube[:, 0, :], g[f"m{m}_j0"]) < TOL, m
        assert relerr(cube[:, 37, :], g[f"m{m}_j37"]) < TOL, m


@pytest.mark.gpu
@pytest.mark.parametrize("j", [0, 37])
def test_2des_256_ensemble_path_matches_reference(j):
    """The bench's product path (response2d_ensemble: pruned split-K MFMA GEMM over members, uniform-grid operand
    tables) at the benchmarked 256 x 256 grid, member by member and summed, against the reference's slices.
    Members 1 and 2 of the fixture are members 0 and 1 of bench.py's seeded ensemble (twodes_inputs, seed 3)."""
    from pyqed_amd.response import ensemble_factors, response2d_ensemble
    g = load_golden("corr4_2des_256")
    rng = np.random.default_rng(3)
    bench_E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((4, 3))
    assert np.array_equal(g["E"][1:], bench_E[:2])
    tau = g["tau"]
    lam, U1, U2, ops, rho0 = _two_des_members(g)
    alpha, Mt, beta = ensemble_factors(lam, U1, U2, ops, rho0.flatten(), tau[j])
    tot = 0
    for m in range(len(g["E"])):
        S = response2d_ensemble(lam[m:m + 1], alpha[m:m + 1], Mt[m:m + 1], beta[m:m + 1], tau, tau).cpu().numpy()
        assert relerr(S, g[f"m{m}_j{j}"]) < TOL, m
        tot = tot + g[f"m{m}_j{j}"]
    S = response2d_ensemble(lam, alpha, Mt, beta, tau, tau).cpu().numpy()
    assert relerr(S, tot) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("j", [0, 37])
def test_2des_bench_size_gemm128_path_matches_reference(j):
    """the benched instantiation itself (the 128-block split-K GEMM with the generated A operand,
    ens_gemm_kernel<128, xtab>, which only ensembles of >= 32k eigen-index columns reach) pinned to the reference: the
    fixture's three members, each repeated 21,846 times (65,538 members, the bench's size), summed by the GPU and
    divided by the repeat count, equal the sum of the reference's slices."""
    from pyqed_amd.response import ensemble_factors, response2d_ensemble
    from conftest import took
    g = load_golden("corr4_2des_256")
    tau = g["tau"]
    lam, U1, U2, ops, rho0 = _two_des_members(g)
    alpha, Mt, beta = ensemble_factors(lam, U1, U2, ops, rho0.flatten(), tau[j])
    R = 21846
    rep = lambda a: np.tile(a, (R,) + (1,) * (a.ndim - 1))
    took("")
    S = response2d_ensemble(rep(lam), rep(alpha), rep(Mt), rep(beta), tau, tau).cpu().numpy()
    hit, paths = took("ens_gemm128_xtab")
    assert hit, paths
    tot = sum(g[f"m{m}_j{j}"] for m in range(len(g["E"])))
    assert relerr(S / R, tot) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("j", [0, 37])
def test_2des_shard_size_gemm64_matches_reference(j):
    """The one-rank 1/8 shard of the bench ensemble (8,192+ members) takes the 64-block split-K GEMM (ens_gemm64, the
    path the bench's shard_1of8 line times): the fixture's three members repeated 2,731 times (8,193 members,
    K = 16,386 -- not a multiple of the 16-wide K-tile), summed by the GPU and divided by the repeat count, equal the
    sum of the reference's slices."""
    from pyqed_amd.response import ensemble_factors, response2d_ensemble
    from conftest import took
    g = load_golden("corr4_2des_256")
    tau = g["tau"]
    lam, U1, U2, ops, rho0 = _two_des_members(g)
    alpha, Mt, beta = ensemble_factors(lam, U1, U2, ops, rho0.flatten(), tau[j])
    R = 2731
    rep = lambda a: np.tile(a, (R,) + (1,) * (a.ndim - 1))
    took("")
    S = response2d_ensemble(rep(lam), rep(alpha), rep(Mt), rep(beta), tau, tau).cpu().numpy()
    hit, paths = took("ens_gemm64")
    assert hit, paths
    tot = sum(g[f"m{m}_j{j}"] for m in range(len(g["E"])))
    assert relerr(S / R, tot) < TOL


@pytest.mark.gpu
def test_spo2_256_matches_reference():
    """Config d2 (256 x 256 x 2, the bench potential, dt = 0.05): 20 Strang steps of SPO2.run (wpd.py:692-758)
    against the reference's final state and per-output populations."""
    from pyqed_amd import SPO2
    g = load_golden("spo2_256")
    n = int(g["n"])
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
    psi0 = np.zeros((n, n, 2), complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    r = sol.run(psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    assert len(r.psilist) == int(g["n_psilist"])
    assert np.allclose(r.times, g["times"])
    assert relerr(r.psilist[-1], g["psi_final"]) < TOL
    assert relerr(sol.exp_K[7], g["exp_K_row7"]) < 1e-13
    assert relerr(sol.exp_V_half[100], g["exp_V_half_row100"]) < 1e-13
    dx = x[1] - x[0]
    pops = np.array([[np.vdot(p[:, :, k], p[:, :, k]).real * dx * dx for k in range(2)] for p in r.psilist])
    assert relerr(pops, g["populations"]) < TOL


@pytest.mark.gpu
def test_redfield_n128_bench_kernel_batch256_matches_reference():
    """the bench's Redfield kernel itself (qd_glf_rk4_herm, persistent Hermitian kernel, B = 256,
    N = 128, bench.py bench_redfield) pinned to the reference fixture: member 0 is the fixture's rho0 in the H
    eigenbasis, members 1..255 seeded pure states.  Member 0's observables Tr(e~ rho~) and its back-transformed final
    state must equal RedfieldSolver.evolve's reference outputs (oqs.py:364-459); member 255 is checked against a
    dense NumPy restatement of the same RHS (X + X^+, X = P rho + sum A rho Lam^+) built with oracle.lindblad.rk4."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd import RedfieldSolver
    from pyqed_amd.oqs import glf_rk4
    g = load_golden("redfield_n128")
    sol = RedfieldSolver(g["H"], c_ops=[g["a_op"]], spectra=[SPECTRA[str(g["spectrum"])]])
    sol.redfield_tensor()
    P, Ls, Ws = sol.glf_terms_herm()
    V = sol.evecs.astype(complex)
    N, Nt, dt, B = 128, int(g["Nt"]), float(g["dt"]), 256
    r0 = V.conj().T @ g["rho0"] @ V
    r0 = 0.5 * (r0 + r0.conj().T)
    rho = np.concatenate([r0[None], olb.random_pure_states(B - 1, N, seed=11)])
    E = np.array([V.conj().T @ e @ V for e in g["E"]])
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(np.asarray(x, complex))).to(dev)
    rd = t(rho)
    obs, _ = glf_rk4(t(P), None, t(Ls), t(Ws), rd, dt, Nt, t(E), hermitian=True)
    assert relerr(obs[0, 1:].cpu().numpy(), g["observables"]) < TOL
    out = rd.cpu().numpy()
    assert relerr(V @ out[0] @ V.conj().T, g["rho_final"]) < TOL

    def rhs(r):
        X = P @ r + sum(a @ r @ w for a, w in zip(Ls, Ws))
        return X + X.conj().T

    ref = rho[-1].copy()
    for _ in range(Nt):
        ref = olb.rk4(ref, lambda r, *a: rhs(r), dt)
    assert relerr(out[-1], ref) < TOL


@pytest.mark.gpu
def test_2des_256_t2scan_matches_reference():
    """the bench's waiting-time scan (T2Scan operands + bucketed apply, bench.py
    bench_2des_t2scan) at the benchmarked 256 x 256 grid against the reference's correlation_4op_3t slices at
    t2 = tau[0] and tau[37] (corr4_2des_256), member by member and summed over members."""
    from pyqed_amd.response import T2Scan, ensemble_factors_bc, response2d_t2scan
    g = load_golden("corr4_2des_256")
    tau = g["tau"]
    lam, U1, U2, ops, rho0 = _two_des_members(g)
    alpha, Bm, Cm, beta = ensemble_factors_bc(lam, U1, U2, ops, rho0.flatten())
    t2 = np.array([tau[0], tau[37]])
    tot = 0
    for m in range(len(g["E"])):
        S = response2d_t2scan(lam[m:m + 1], alpha[m:m + 1], Bm[m:m + 1], Cm[m:m + 1], beta[m:m + 1], tau, t2,
                              tau).cpu().numpy()
        for k, j in enumerate((0, 37)):
            assert relerr(S[k], g[f"m{m}_j{j}"]) < TOL, (m, j)
        tot = tot + np.array([g[f"m{m}_j0"], g[f"m{m}_j37"]])
    sc = T2Scan(lam, alpha, Bm, Cm, beta, tau, tau)
    S = np.concatenate([sc.apply(t2[:1]).cpu().numpy(), sc.apply(t2[1:]).cpu().numpy()])
    assert relerr(S, tot) < TOL
