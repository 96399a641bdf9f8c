"""DEOM hierarchy kernel (qd_deom_rk4) vs reference golden vectors and the oracle."""
import numpy as np
import pytest
import sympy as sp

from conftest import load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _solver(g, pulses):
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    lam, gam, beta, npsd = float(g["lam"]), float(g["gam"]), float(g["beta"]), int(g["npsd"])
    bath = Bath([2 * lam * gam * w / (gam ** 2 + w ** 2)], w, [beta], [npsd], [0] * (1 + npsd))
    fs = (lambda t: 0.3 * np.sin(2 * t)) if pulses else (lambda t: 0)
    fc = (lambda t: 0.1 * np.cos(t)) if pulses else (lambda t: 0)
    return DEOMSolver(g["H"], g["sdip"], bath, g["Q"], g["cdip"], fs, fc, int(g["lmax"]))


@pytest.mark.parametrize("name", ["deom_run_small", "deom_run_pulsed", "deom_run_bench", "deom_run_bench_long"])
def test_deom_run_matches_reference(name):
    g = load_golden(name)
    pulses = bool(g["pulses"])
    sol = _solver(g, pulses)
    rho0 = np.zeros((2, 2), complex)
    rho0[0, 0] = 1
    p1 = np.array([[1, 0], [0, 0]], complex) if "trace_p1" in g else None
    t, saved = sol.run(rho0, float(g["dt"]), int(g["nt"]), p1)
    assert sol.nmax == int(g["nmax"])
    assert np.allclose(t, g["t_save"])
    if p1 is not None:
        assert relerr(saved, g["trace_p1"]) < TOL
    else:
        assert relerr(np.array(saved), g["rho_sys"]) < TOL
        # aliasing quirk of the reference: rho0 holds the final system density matrix
        assert relerr(rho0, g["rho_sys"][-1]) < TOL
    if "ado_final" in g:
        assert relerr(sol.ddos, g["ado_final"]) < TOL


def test_deom_batch_vs_oracle_and_trace():
    """Two independent hierarchies (different rho0), K=4, L=5, vs the NumPy restatement."""
    from oracle import deom as od
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [3], [0] * 4)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 5)
    r0 = np.zeros((2, 2, 2), complex)
    r0[0, 0, 0] = 1
    r0[1] = 0.5 * np.array([[1, 1], [1, 1]])
    t, saved = sol.run_batch(r0, 0.02, 25)
    for b in range(2):
        tt, ref, _ = od.run(sz + sx, np.zeros((2, 2)), lambda t: 0, np.array([sx]), np.zeros((1, 2, 2)),
                            lambda t: 0, (bath.etal, bath.etar, bath.etaa, bath.expn), 5, r0[b], 0.02, 25)
        assert relerr(saved[b], ref) < TOL
    tr = np.trace(saved, axis1=2, axis2=3)
    assert np.max(np.abs(tr - 1)) < 1e-12


def test_deom_bench_size_properties():
    """L=12, K=5 (6188 ADOs): trace of rho_0 conserved, hermiticity kept, 300 steps.
    dt = 0.002: explicit RK4 needs dt * L * max Re(expn) = dt * 12 * 57.8 < 2.8 (dt = 0.01 diverges,
    in the reference arithmetic as well)."""
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
    rho0 = np.zeros((2, 2), complex)
    rho0[0, 0] = 1
    t, saved = sol.run(rho0, 0.002, 300)
    saved = np.array(saved)
    assert sol.nmax == 6188
    assert np.max(np.abs(np.trace(saved, axis1=1, axis2=2) - 1)) < 1e-12
    assert np.max(np.abs(saved - np.conj(np.swapaxes(saved, 1, 2)))) < 1e-12


@pytest.mark.parametrize("ns,npsd,L", [(3, 3, 4), (5, 1, 3), (2, 8, 2)])
def test_deom_layouts_vs_oracle(ns, npsd, L):
    """ns = 3 / 5 exercise the lane-group kernel with padding lanes (groups of 16 / 32 lanes);
    npsd = 8 (K = 9 > 8) exercises the element-per-thread kernel."""
    from oracle import deom as od
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.4 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [npsd], [0] * (1 + npsd))
    rng = np.random.default_rng(ns)
    A = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (A + A.conj().T) / 4
    Q = np.diag(np.arange(ns, dtype=float)).astype(complex) + 0.2 * (np.eye(ns, k=1) + np.eye(ns, k=-1))
    psi = rng.standard_normal(ns) + 1j * rng.standard_normal(ns)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    sol = DEOMSolver(H, None, bath, np.array([Q]), None, None, None, L)
    dt, nt = 0.005, 12
    t, saved = sol.run_batch(rho0[None], dt, nt)
    tt, ref, _ = od.run(H, np.zeros((ns, ns)), lambda t: 0, np.array([Q]), np.zeros((1, ns, ns)), lambda t: 0,
                        (bath.etal, bath.etar, bath.etaa, bath.expn), L, rho0, dt, nt)
    assert relerr(saved[0], ref) < TOL


def test_deom_correlation_4op_3t_matches_reference(tmp_path, monkeypatch):
    """DEOMSolver.correlation_4op_3t (heom/deom.py:1127-1209): host P / eig, GPU (w_x, w_y) grid."""
    from pyqed_amd.deom import Bath, DEOMSolver
    g = load_golden("deom_corr4")
    sx = g["Q"][0]
    sz = np.diag([1.0, -1.0]).astype(complex)
    bath = Bath.__new__(Bath)
    bath.etal, bath.etar, bath.etaa, bath.expn = g["etal"], g["etar"], g["etaa"], g["expn"]
    bath.mode = np.zeros(len(g["expn"]), dtype=np.int64)
    sol = DEOMSolver(g["H"], np.zeros((2, 2), complex), bath, g["Q"], np.zeros((1, 2, 2), complex),
                     lambda t: 0, lambda t: 0, int(g["lmax"]))
    T, wx, wy = float(g["T"]), g["wx"], g["wy"]
    for lcr in ["llll", "lrlr", "lccc"]:
        cw = sol.correlation_4op_3t(sx, sx, sx, sx, g["rho0"], T, wx, wy, lcr=lcr)
        assert cw.shape == (len(wx), len(wy))
        assert relerr(cw, g["cw_" + lcr]) < 1e-10, lcr
    assert relerr(sol.propgator, g["propagator"]) < 1e-14
    monkeypatch.chdir(tmp_path)
    cw = sol.correlation_4op_3t(sz, sx, sx, sz, g["rho0"], T, wx, wy, if_full=False, lcr="llll", if_save=True)
    # The eigenvalue cut keeps V[:, sel] and pinv(V)[sel, :] of a non-normal P: the result inherits the
    # conditioning of LAPACK's eig (another host's OpenBLAS kernels move it by ~1e-8 relative, the
    # reference's own output included).  Against the oracle on THIS host's eig the GPU grid is exact.
    assert relerr(cw, g["cw_cut_llll"]) < 1e-7
    from oracle import deom as od
    ref_here = od.correlation_4op_3t(sol.propgator, sol.nmax, 2, [sz, sx, sx, sz], g["rho0"], T, wx, wy,
                                     if_full=False)
    assert relerr(cw, ref_here) < 1e-10
    sol2 = DEOMSolver(g["H"], None, bath, g["Q"], None, None, None, int(g["lmax"]))
    cw2 = sol2.correlation_4op_3t(sz, sx, sx, sz, g["rho0"], T, wx, wy, if_full=False, if_load=True)
    assert relerr(cw2, cw) < 1e-12


def test_resolvent_grid2d_ragged_sizes():
    """qd_resolvent_grid2d against its closed form at sizes that exercise every padding path."""
    import torch
    from pyqed_amd import _lib
    rng = np.random.default_rng(4)
    dev = torch.device("cuda", 0)
    for n, nx, ny in [(7, 5, 3), (140, 129, 300), (300, 64, 130)]:
        lam = -rng.uniform(0.05, 2, n) + 1j * rng.uniform(-5, 5, n)
        a, v = (rng.standard_normal(n) + 1j * rng.standard_normal(n) for _ in range(2))
        M = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        wx, wy = np.linspace(-4, 4, nx), np.linspace(-3, 6, ny)
        X = a[None, :] / (-lam[None, :] - 1j * wx[:, None])
        Z = v[:, None] / (-lam[:, None] - 1j * wy[None, :])
        ref = X @ M @ Z
        t = lambda x, dt=torch.complex128: torch.from_numpy(np.ascontiguousarray(x)).to(device=dev, dtype=dt)
        out = torch.empty((nx, ny), dtype=torch.complex128, device=dev)
        args = [t(a), t(M), t(v), t(lam)]
        wxt, wyt = t(wx, torch.float64), t(wy, torch.float64)
        rc = _lib.load().qd_resolvent_grid2d(*(x.data_ptr() for x in args), n, wxt.data_ptr(), nx, wyt.data_ptr(),
                                             ny, out.data_ptr(), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_resolvent_grid2d")
        assert relerr(out.cpu().numpy(), ref) < 1e-12, (n, nx, ny)


@pytest.mark.parametrize("ns,B,pulse", [(2, 19, False), (2, 16, True), (3, 5, False)])
def test_deom_ado_major_batch_layout(ns, B, pulse):
    """Batches stored ADO-major ([nmax][B], qd_deom_rk4_ado_major: one ADO of 16 hierarchies per wave) vs the
    hierarchy-major layout and the oracle: per-hierarchy rho_0 histories, final ADOs, traces; a ragged batch
    (19: waves straddle two ADOs), a pulsed system / coupling, and ns = 3 (16-lane groups with padding)."""
    from oracle import deom as od
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [3], [0] * 4)
    rng = np.random.default_rng(B)
    A = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (A + A.conj().T) / 4
    Q = np.diag(np.arange(ns, dtype=float)).astype(complex) + 0.2 * (np.eye(ns, k=1) + np.eye(ns, k=-1))
    dip = 0.3 * (np.eye(ns, k=1) + np.eye(ns, k=-1)).astype(complex)
    f = (lambda t: np.exp(-((t - 0.05) / 0.02) ** 2) * np.cos(3 * t)) if pulse else None
    psi = rng.standard_normal((B, ns)) + 1j * rng.standard_normal((B, ns))
    psi /= np.linalg.norm(psi, axis=1, keepdims=True)
    rho0 = np.einsum("bi,bj->bij", psi, psi.conj())
    dt, nt, L = 0.005, 10, 5
    out = {}
    for mode, layout in (("1", "ado_major"), ("0", "element_major")):
        sol = DEOMSolver(H, dip if pulse else None, bath, np.array([Q]), None, f, None, L)
        sol.layout = layout
        t, saved = sol.run_batch(rho0, dt, nt)
        out[mode] = (saved, sol.ddos)
    assert relerr(out["1"][0], out["0"][0]) < 1e-13 and relerr(out["1"][1], out["0"][1]) < 1e-13
    for b in (0, B - 1):
        tt, ref, _ = od.run(H, dip if pulse else np.zeros((ns, ns)), f if pulse else (lambda t: 0), np.array([Q]),
                            np.zeros((1, ns, ns)), lambda t: 0, (bath.etal, bath.etar, bath.etaa, bath.expn), L,
                            rho0[b], dt, nt)
        assert relerr(out["1"][0][b], ref) < TOL, b


@pytest.mark.parametrize("ns,B,npsd", [(2, 16, 3), (2, 1, 3), (3, 8, 3), (2, 32, 4), (2, 24, 3), (2, 128, 4)])
def test_deom_xcd_block_classes(ns, B, npsd):
    """Hierarchies dealt to the 8 XCD block classes (whenever 8 | B) in both batch layouts, against the flat numbering
    (B = 1) and the oracle (heom/deom.py:1072-1114): every member's history and final ADOs agree across the layouts
    at 1e-13 and the last member matches the oracle.  ns = 2 ADO-major classes of 16k hierarchies (B = 128: classes
    of 16) run the wave-uniform kernel with scalar table loads; the others the per-lane group kernels."""
    from oracle import deom as od
    from pyqed_amd.deom import Bath, DEOMSolver
    from conftest import took
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [npsd], [0] * (npsd + 1))
    rng = np.random.default_rng(7 + B)
    A = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (A + A.conj().T) / 4
    Q = np.diag(np.arange(ns, dtype=float)).astype(complex) + 0.2 * (np.eye(ns, k=1) + np.eye(ns, k=-1))
    psi = rng.standard_normal((B, ns)) + 1j * rng.standard_normal((B, ns))
    psi /= np.linalg.norm(psi, axis=1, keepdims=True)
    rho0 = np.einsum("bi,bj->bij", psi, psi.conj())
    dt, nt, L = 0.005, 8, 6
    out = {}
    took("")
    for layout in ("element_major", "ado_major"):
        sol = DEOMSolver(H, None, bath, np.array([Q]), None, None, None, L)
        sol.layout = layout
        _, saved = sol.run_batch(rho0, dt, nt)
        out[layout] = (np.array(saved), sol.ddos.copy())
    if (ns, B) == (2, 128):
        assert took("deom_grp4_uniform")[0]
    assert relerr(out["ado_major"][0], out["element_major"][0]) < 1e-13
    assert relerr(out["ado_major"][1], out["element_major"][1]) < 1e-13
    tt, ref, _ = od.run(H, np.zeros((ns, ns)), lambda t: 0, np.array([Q]), np.zeros((1, ns, ns)), lambda t: 0,
                        (bath.etal, bath.etar, bath.etaa, bath.expn), L, rho0[B - 1], dt, nt)
    assert relerr(out["ado_major"][0][B - 1], ref) < TOL


def _multi_mode_model(ns, nmod, npsd, L, seed=3):
    from pyqed_amd.deom import Bath, DEOMSolver
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (A + A.conj().T) / 2 / np.sqrt(ns)
    Qs = []
    for m in range(nmod):
        B = rng.standard_normal((ns, ns))
        Qs.append(((B + B.T) / 2 / np.sqrt(ns)).astype(complex))
    w = sp.symbols(r"\omega", real=True)
    spes = [2 * lam * gam * w / (gam ** 2 + w ** 2) for lam, gam in [(0.4, 1.0), (0.2, 2.0)][:nmod]]
    mode = [m for m in range(nmod) for _ in range(1 + npsd)]
    bath = Bath(spes, w, [1.0] * nmod, [npsd] * nmod, mode)
    sdip = np.diag(np.linspace(0, 1, ns)).astype(complex)
    fs = lambda t: 0.2 * np.cos(3 * t)
    fc = lambda t: 0.05 * np.sin(t)
    cdip = np.array([0.3 * q for q in Qs])
    sol = DEOMSolver(H, sdip, bath, np.array(Qs), cdip, fs, fc, L)
    rho0 = np.zeros((ns, ns), complex)
    rho0[0, 0] = 1
    return sol, bath, H, np.array(Qs), sdip, cdip, fs, fc, rho0, mode


@pytest.mark.parametrize("ns,nmod,npsd,L", [(16, 1, 1, 3), (12, 2, 1, 2), (9, 1, 2, 3), (16, 2, 0, 3)])
def test_deom_mfma16_matches_oracle(ns, nmod, npsd, L):
    """The MFMA tile kernel (9 <= ns <= 16: two 16 x 16(1+nmod) x 16 complex GEMMs per ADO on v_mfma_f64_16x16x4_f64,
    zero padding to 16) for 1 and 2 bath modes with driven H(t), Q(t): against the oracle (oracle.deom.run restates
    DEOMSolver.run, heom/deom.py:1072-1114)."""
    from oracle import deom as od
    from conftest import took
    sol, bath, H, Qs, sdip, cdip, fs, fc, rho0, mode = _multi_mode_model(ns, nmod, npsd, L)
    nt, dt = 4, 0.02
    P1 = np.eye(ns, dtype=complex)[::-1]
    _, tr_ref, ados_ref = od.run(H, sdip, fs, Qs, cdip, fc, (bath.etal, bath.etar, bath.etaa, bath.expn), L, rho0,
                                 dt, nt, P1, mode=mode)
    took("")
    t, tr = sol.run_batch(rho0[None], dt, nt, P1)
    assert took("deom_mfma16")[0]
    assert relerr(tr[0], tr_ref) < TOL
    assert relerr(sol.ddos[0], ados_ref) < TOL


@pytest.mark.parametrize("ns,npsd,L,nbands", [(2, 4, 12, 8), (2, 1, 5, 3), (12, 1, 4, 4), (16, 2, 3, 2)])
def test_deom_tier_bands_loopback_matches_single(ns, npsd, L, nbands):
    """Tier-banded sharding on the GPU (pyqed_amd.deom_shard, qd_deom_stage + qd_gather_rows, all bands in one
    process with device-side halo copies): Tr(p1 rho_0) and the final hierarchy equal the single-process
    qd_deom_rk4 run (same kernels per ADO).  (2, 4, 12, 8) is the bench hierarchy (6188 ADOs) over 8 bands."""
    from pyqed_amd.deom_shard import ShardedDEOM
    if ns == 2:
        g = {"H": np.array([[1, 1], [1, -1]], complex), "Q": np.array([[[0, 1], [1, 0]]], complex),
             "sdip": np.array([[0, 1], [1, 0]], complex), "cdip": np.array([np.diag([1.0, -1.0]).astype(complex)]),
             "lam": 0.5, "gam": 1.0, "beta": 1.0, "npsd": npsd, "lmax": L}
        sol = _solver(g, True)
        rho0 = np.zeros((2, 2), complex)
        rho0[0, 0] = 1
    else:
        sol, *_, rho0, _ = _multi_mode_model(ns, 1, npsd, L)
    nt, dt = 5, 0.005
    P1 = np.eye(ns, dtype=complex)[::-1].copy()
    sh = ShardedDEOM(sol, nbands=nbands, loopback=True)
    t, tr = sh.run(rho0, dt, nt, P1)
    ados = sh.gather_ados()
    _, tr1 = sol.run_batch(rho0[None], dt, nt, P1)
    assert relerr(tr, tr1[0]) < 1e-13
    assert relerr(ados, sol.ddos[0]) < 1e-13


# the batched kernels of undriven ns = 2 hierarchies, each reached by its shape (the L = 6 cases of
# round 4 never reached the pipelined kernel): (B, npsd, L, layout, kernel path)
_BATCH_CASES = [
    (64, 4, 8, "ado_major", "deom_pipe_k5"),      # K = 5, 1287 ADOs: the pipelined persistent kernel, classes of 8
    (72, 4, 8, "ado_major", "deom_pipe_k5"),      # ragged classes of 9: the carry step of the class walk
    (64, 3, 11, "ado_major", "deom_pipe_k4"),     # K = 4, 1365 ADOs
    (64, 5, 7, "ado_major", "deom_pipe_k6"),      # K = 6, 1716 ADOs
    (64, 4, 6, "ado_major", "deom_grp4_w5"),      # 462 ADOs: below the pipelined kernel's lane count
    (64, 4, 6, "element_major", "deom_grp4_w5"),  # hierarchy-major layout
]


@pytest.mark.parametrize("B,npsd,L,layout,path", _BATCH_CASES)
def test_deom_batched_kernels_match_oracle(B, npsd, L, layout, path):
    """The batched stage kernels (Horner form, >= 64 hierarchies, 8 XCD block classes; VERDICT r03 weak #1, ADVICE r04
    medium): each case asserts the kernel its shape selects (qd_take_path), matches the oracle's RK4 (heom/deom.py:
    641-766, 1072-1114) at 1e-10 for the first and the last member, and agrees with the other layout at 1e-13."""
    from oracle import deom as od
    from pyqed_amd.deom import Bath, DEOMSolver
    from conftest import took
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [npsd], [0] * (npsd + 1))
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    rng = np.random.default_rng(B + npsd)
    psi = rng.standard_normal((B, 2)) + 1j * rng.standard_normal((B, 2))
    psi /= np.linalg.norm(psi, axis=1, keepdims=True)
    rho0 = np.einsum("bi,bj->bij", psi, psi.conj())
    dt, nt = 0.005, 3
    out = {}
    for lay in (layout, "element_major" if layout == "ado_major" else "ado_major"):
        sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, L)
        sol.layout = lay
        took("")
        _, saved = sol.run_batch(rho0, dt, nt)
        hit, got = took(path)
        if lay == layout:
            assert sol.nind == npsd + 1
            assert hit, got
        out[lay] = (np.array(saved), sol.ddos.copy())
    a, b = out.values()
    assert relerr(a[0], b[0]) < 1e-13 and relerr(a[1], b[1]) < 1e-13
    for m in (0, B - 1):
        _, ref, _ = od.run(sz + sx, np.zeros((2, 2)), lambda t: 0, np.array([sx]), np.zeros((1, 2, 2)),
                           lambda t: 0, (bath.etal, bath.etar, bath.etaa, bath.expn), L, rho0[m], dt, nt)
        assert relerr(out[layout][0][m], ref) < TOL, m


def test_deom_batched_pipe_kernel_bench_hierarchy_matches_reference():
    """64 hierarchies of the bench hierarchy (L = 12, K = 5: 6188 ADOs each, the bench's [nmax][B][2][2] layout and
    XCD dealing: the pipelined kernel) for the reference fixture's 3 steps: member 0 starts from the fixture's |0><0|
    and its Tr(p1 rho_0) equals deom_run_bench (the reference's own run) at 1e-10; every member agrees with the
    hierarchy-major layout (the five-waves kernel) at 1e-13."""
    from conftest import took
    g = load_golden("deom_run_bench")
    B = 64
    rng = np.random.default_rng(64)
    psi = rng.standard_normal((B, 2)) + 1j * rng.standard_normal((B, 2))
    psi /= np.linalg.norm(psi, axis=1, keepdims=True)
    rho0 = np.einsum("bi,bj->bij", psi, psi.conj())
    rho0[0] = np.array([[1, 0], [0, 0]], complex)
    p1 = np.array([[1, 0], [0, 0]], complex)
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    lam, gam, beta = float(g["lam"]), float(g["gam"]), float(g["beta"])
    out = {}
    for layout, path in (("ado_major", "deom_pipe_k5"), ("element_major", "deom_grp4_w5")):
        # the fixture's pulses are zero, so the undriven solver (Horner-form stages) runs the same equations of motion
        # as the reference's H + 0 * sdip
        bath = Bath([2 * lam * gam * w / (gam ** 2 + w ** 2)], w, [beta], [int(g["npsd"])], [0] * (1 + int(g["npsd"])))
        sol = DEOMSolver(g["H"], None, bath, g["Q"], None, None, None, int(g["lmax"]))
        sol.layout = layout
        took("")
        t, tr = sol.run_batch(rho0, float(g["dt"]), int(g["nt"]), p1)
        assert took(path)[0], layout
        out[layout] = (np.array(tr), sol.ddos.copy())
    assert sol.nmax == 6188
    assert relerr(out["ado_major"][0][0], g["trace_p1"]) < TOL
    assert relerr(out["ado_major"][0], out["element_major"][0]) < 1e-13
    assert relerr(out["ado_major"][1], out["element_major"][1]) < 1e-13


def test_gather_rows_bounds_checked():
    """qd_gather_rows (the tier bands' halo packing) never reads outside its source rows: an out-of-range index
    writes a NaN row, and check = 1 returns QD_EINVAL."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd._util import default_device
    dev = default_device()
    src = torch.arange(5 * 4, dtype=torch.float64, device=dev).to(torch.complex128).reshape(5, 4)
    dst = torch.zeros((3, 4), dtype=torch.complex128, device=dev)
    lib = _lib.load()
    idx = torch.tensor([4, 0, 2], dtype=torch.int32, device=dev)
    assert lib.qd_gather_rows(src.data_ptr(), 5, idx.data_ptr(), 3, 4, dst.data_ptr(), 1, _lib.stream_ptr(dev)) == 0
    assert torch.equal(dst, src[[4, 0, 2]])
    bad = torch.tensor([1, 5, -1], dtype=torch.int32, device=dev)
    rc = lib.qd_gather_rows(src.data_ptr(), 5, bad.data_ptr(), 3, 4, dst.data_ptr(), 1, _lib.stream_ptr(dev))
    assert rc == _lib.QD_EINVAL
    d = dst.cpu().numpy()
    assert np.array_equal(d[0], src[1].cpu().numpy()) and np.isnan(d[1:].real).all()
