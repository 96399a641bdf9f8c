"""qd_deom_rk4_banded (one hierarchy as one persistent launch over tier bands) against the per-stage launch
sequence (qd_deom_rk4: same arithmetic; bit-identical with one band, within 1e-13 with several -- the handed-off halo
rows carry their stage's parity in the lowest mantissa bit, deom.hip band_tag) and the NumPy restatement
(oracle/deom.py)."""
import numpy as np
import pytest
import sympy as sp

from conftest import relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _bath(npsd, nmod=1):
    from pyqed_amd.deom import Bath
    w = sp.symbols(r"\omega", real=True)
    return Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)] * nmod, w, [1.0] * nmod, [npsd] * nmod,
                [m for m in range(nmod) for _ in range(npsd + 1)])


def _run(sol, rho0, dt, nt, nbands, p1=None, status=True, calls=1, graph=False):
    """(rho_sys or trace, final ADOs) of one hierarchy: banded with `nbands` bands, or (None) the stage launches.
    status=False passes no status word (the asynchronous form with the stream-ordered fallback).  calls > 1 chains
    that many banded calls on the same ADOs; graph=True captures one banded call (no status word) into a HIP graph on
    a side stream and replays it `calls` times."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.deom import ado_coefficients
    from pyqed_amd._util import default_device
    dev = default_device()
    sol.check_()
    sol.init_()
    ns, K, nmax = sol.nsys, sol.nind, sol.nmax
    b = sol.bath
    coef, damp = ado_coefficients(sol.keys, np.asarray(b.etal), np.asarray(b.etar), np.asarray(b.etaa),
                                  np.asarray(b.expn), sol.lmax)
    c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
    ados = torch.zeros((nmax, ns, ns), dtype=torch.complex128, device=dev)
    ados[0] = c128(rho0)
    H = c128(sol.system)
    Q = c128(np.asarray(sol.coupling, dtype=complex).reshape(-1, ns, ns))
    nmod = Q.shape[0]
    Hdip, fs = sol._dip_values(sol.system_dipole, sol.pulse_system_func, nt, dt, (ns, ns))
    Qdip, fc = sol._dip_values(sol.coupling_dipole, sol.pulse_coupling_func, nt, dt, (nmod, ns, ns))
    Hd = c128(Hdip) if Hdip is not None else None
    Qd = c128(Qdip) if Qdip is not None else None
    fs = np.ascontiguousarray(fs) if fs is not None else None
    fc = np.ascontiguousarray(fc) if fc is not None else None
    rho_sys = torch.empty((nt + 1, ns, ns), dtype=torch.complex128, device=dev)
    p1_t = c128(np.asarray(p1, complex).reshape(1, ns, ns)) if p1 is not None else None
    trace = torch.empty((nt + 1, 1), dtype=torch.complex128, device=dev) if p1 is not None else None
    coef_t, damp_t, mode_t = c128(coef), c128(damp), i32(b.mode)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    fsp = fs.ctypes.data if fs is not None else None
    fcp = fc.ctypes.data if fc is not None else None
    if nbands is None:
        mi, pl = i32(sol._minus), i32(sol._plus)
        rc = lib.qd_deom_rk4(ados.data_ptr(), 1, nmax, K, ns, mi.data_ptr(), pl.data_ptr(), coef_t.data_ptr(),
                             damp_t.data_ptr(), mode_t.data_ptr(), nmod, H.data_ptr(), _lib.ptr(Hd), Q.data_ptr(),
                             _lib.ptr(Qd), fsp, fcp, dt, nt, rho_sys.data_ptr(), _lib.ptr(p1_t),
                             1 if p1 is not None else 0, _lib.ptr(trace), st)
        _lib.check(rc, "qd_deom_rk4")
    else:
        bt = sol.band_tables(dev, nbands)
        assert bt is not None and bt.nbands == min(nbands, nmax)
        stat = torch.zeros(1, dtype=torch.int32, device=dev) if status and not graph else None

        def call(stream):
            rc = lib.qd_deom_rk4_banded(ados.data_ptr(), nmax, K, ns, *bt.args(), coef_t.data_ptr(),
                                        damp_t.data_ptr(), mode_t.data_ptr(), nmod, H.data_ptr(), _lib.ptr(Hd),
                                        Q.data_ptr(), _lib.ptr(Qd), fsp, fcp, dt, nt, rho_sys.data_ptr(),
                                        _lib.ptr(p1_t), 1 if p1 is not None else 0, _lib.ptr(trace), _lib.ptr(stat),
                                        stream)
            _lib.check(rc, "qd_deom_rk4_banded")
        if graph:
            side = torch.cuda.Stream(dev)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                call(side.cuda_stream)
            for _ in range(calls):
                g.replay()
        else:
            for _ in range(calls):
                call(st)
        torch.cuda.synchronize(dev)
        if stat is not None:
            assert int(stat.item()) == 0
    torch.cuda.synchronize(dev)
    out = trace[:, 0] if p1 is not None else rho_sys
    return out.cpu().numpy(), ados.cpu().numpy()


def _spin_boson(L, npsd=4, pulses=False):
    from pyqed_amd.deom import DEOMSolver
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    if pulses:
        return DEOMSolver(sz + sx, 0.5 * sx, _bath(npsd), np.array([sx]), np.array([0.2 * sz]),
                          lambda t: 0.3 * np.sin(2 * t), lambda t: 0.1 * np.cos(t), L)
    return DEOMSolver(sz + sx, None, _bath(npsd), np.array([sx]), None, None, None, L)


HALO_TAG_TOL = 1e-13   # a halo value is off by at most one unit in its last place; it enters through dt x stencil


@pytest.mark.parametrize("L,nbands", [(5, 1), (5, 2), (5, 7), (12, 65), (12, 128), (12, 194), (12, 256)])
def test_banded_matches_stage_launches(L, nbands):
    """K = 5 at L = 5 (252 ADOs: one, two and seven bands) and the bench hierarchy (L = 12: 6188 ADOs, 65 to 256
    bands), 12 RK4 steps: bit-identical with one band (no halo), within HALO_TAG_TOL with several."""
    sol = _spin_boson(L)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    ref, ref_ados = _run(sol, rho0, 0.002, 12, None)
    got, got_ados = _run(sol, rho0, 0.002, 12, nbands)
    if nbands == 1:
        assert np.array_equal(got, ref)
        assert np.array_equal(got_ados, ref_ados)
    else:
        assert relerr(got, ref) < HALO_TAG_TOL
        assert relerr(got_ados, ref_ados) < HALO_TAG_TOL


LONG_RUN_TOL = 1e-11   # 2000 steps x 4 stages of at most one ulp entering through dt x stencil (measured ~1e-13)


def test_banded_long_run_matches_stage_launches():
    """the data-as-flag halo tag changes a handed-off value by at most one ulp per stage, so the banded
    launch and the stage launches drift apart with the step count.  The bench hierarchy (L = 12, 6188 ADOs) over 256
    bands for 2000 RK4 steps (a production-length run) stays within LONG_RUN_TOL of the stage launches, for the
    reduced density matrix at every step and for the final ADOs."""
    sol = _spin_boson(12)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    ref, ref_ados = _run(sol, rho0, 0.002, 2000, None)
    got, got_ados = _run(sol, rho0, 0.002, 2000, 256)
    err = max(relerr(got, ref), relerr(got_ados, ref_ados))
    print(f"banded vs stage launches, 2000 steps: {err:.3e}")
    assert err < LONG_RUN_TOL


def test_banded_pulsed_trace_matches_oracle():
    """Driven H(t) = H + f_s(t) Hdip, Q(t) = Q + f_c(t) Qdip, Tr(p1 rho_0), against the oracle."""
    from oracle import deom as od
    sol = _spin_boson(5, npsd=3, pulses=True)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    p1 = np.diag([1.0, 0.0]).astype(complex)
    got, _ = _run(sol, rho0, 0.01, 30, 9, p1=p1)
    b = sol.bath
    _, ref_rho, _ = od.run(sol.system, sol.system_dipole, sol.pulse_system_func, np.array(sol.coupling),
                           np.array(sol.coupling_dipole), sol.pulse_coupling_func,
                           (b.etal, b.etar, b.etaa, b.expn), 5, rho0, 0.01, 30)
    ref = np.einsum("ij,tji->t", p1, ref_rho)
    assert relerr(got, ref) < TOL
    ref2, _ = _run(sol, rho0, 0.01, 30, None, p1=p1)
    assert relerr(got, ref2) < HALO_TAG_TOL


@pytest.mark.parametrize("ns,nmod", [(3, 1), (4, 2)])
def test_banded_ns3_ns4_matches_stage_launches_and_oracle(ns, nmod):
    """16 lanes per ADO (ns = 3, 4), two bath modes (K = 8: the KMAX = 8 instantiation)."""
    from oracle import deom as od
    from pyqed_amd.deom import DEOMSolver
    rng = np.random.default_rng(ns)
    A = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (A + A.conj().T) / 4
    Qs = []
    for _ in range(nmod):
        B = rng.standard_normal((ns, ns))
        Qs.append((B + B.T) / 4)
    npsd = 3
    sol = DEOMSolver(H, None, _bath(npsd, nmod), np.array(Qs, dtype=complex), None, None, None, 4)
    rho0 = np.zeros((ns, ns), complex)
    rho0[0, 0] = 1
    got, got_ados = _run(sol, rho0, 0.01, 15, 11)
    ref, ref_ados = _run(sol, rho0, 0.01, 15, None)
    # same formula as the 16-lane group kernel; the compilers' FMA contraction may differ in the last bit
    assert relerr(got, ref) < 1e-14
    assert relerr(got_ados, ref_ados) < 1e-14
    b = sol.bath
    _, orc, _ = od.run(H, np.zeros((ns, ns)), lambda t: 0, np.array(Qs, dtype=complex),
                       np.zeros((nmod, ns, ns)), lambda t: 0, (b.etal, b.etar, b.etaa, b.expn), 4, rho0, 0.01, 15,
                       mode=np.asarray(b.mode))
    assert relerr(got, orc) < TOL


def test_solver_run_takes_banded_path_and_attribute_disables_it():
    """DEOMSolver.run (B = 1) runs the banded launch by default; solver.banded = False gives the stage launches."""
    import torch
    from pyqed_amd._util import default_device
    from conftest import took
    sol = _spin_boson(8)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    took("")
    t, a = sol.run(rho0.copy(), 0.005, 20)
    assert took("deom_banded")[0]
    assert sol.band_tables(default_device()) is not None
    sol.banded = False
    assert sol.band_tables(default_device()) is None
    t2, b = sol.run(rho0.copy(), 0.005, 20)
    assert relerr(np.array(a), np.array(b)) < HALO_TAG_TOL
    torch.cuda.synchronize()


def test_banded_stretch_hierarchy_256_bands_matches_stage_launches():
    """The stretch hierarchy (npsd = 5, K = 6, L = 12: 18,564 ADOs) on 256 bands (the default there; the generic
    K <= 8 instantiation), 6 steps."""
    sol = _spin_boson(12, npsd=5)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    ref, ref_ados = _run(sol, rho0, 0.001, 6, None)
    got, got_ados = _run(sol, rho0, 0.001, 6, 256)
    assert relerr(got, ref) < HALO_TAG_TOL
    assert relerr(got_ados, ref_ados) < HALO_TAG_TOL


def test_solver_run_falls_back_to_stage_launches_after_band_timeout():
    """A hand-off timeout (status = 1, forced by the QD_OPT_FAKE_TIMEOUT test option after a real banded run has
    overwritten the ADOs) makes DEOMSolver.run restore the initial ADOs and re-run on the stage launches with a
    warning: the result equals the stage launches bit for bit."""
    import warnings
    from conftest import qd_option
    sol = _spin_boson(8)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    sol.banded = False
    _, ref = sol.run(rho0.copy(), 0.005, 20)
    ref_ddos = sol.ddos.copy()
    sol.banded = None
    with qd_option("fake_timeout", 1), warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        _, got = sol.run(rho0.copy(), 0.005, 20)
    assert any("timed out" in str(x.message) for x in w)
    assert sol.last_run_banded is False
    assert np.array_equal(np.array(got), np.array(ref))
    assert np.array_equal(sol.ddos, ref_ddos)
    _, again = sol.run(rho0.copy(), 0.005, 20)
    assert sol.last_run_banded is True
    assert relerr(np.array(again), np.array(ref)) < HALO_TAG_TOL


@pytest.mark.parametrize("pulsed", [False, True])
def test_banded_without_status_word_falls_back_on_device(pulsed):
    """qd_deom_rk4_banded without a status word stays asynchronous -- a hand-off timeout (forced by
    QD_OPT_FAKE_TIMEOUT after a real banded run) is repaired by the stream-ordered fallback queued behind the launch
    (one workgroup restores the saved ADOs and re-runs every stage on the element stencil, band tables mapped back to
    global rows): rho_sys at every step, the trace and the final ADOs equal the stage launches' within 1e-13, for the
    Horner form and for a driven (classic RK4) run; without the timeout the guard changes nothing."""
    from conftest import qd_option, took
    sol = _spin_boson(5, npsd=3, pulses=pulsed)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    ref, ref_ados = _run(sol, rho0, 0.01, 12, None)
    took("")
    with qd_option("fake_timeout", 1):
        got, got_ados = _run(sol, rho0, 0.01, 12, 9, status=False)
    assert "deom_banded_guarded" in took("")[1]
    assert relerr(got, ref) < 1e-13 and relerr(got_ados, ref_ados) < 1e-13
    plain, plain_ados = _run(sol, rho0, 0.01, 12, 9, status=False)
    banded, banded_ados = _run(sol, rho0, 0.01, 12, 9)
    assert np.array_equal(plain, banded) and np.array_equal(plain_ados, banded_ados)


def test_banded_call_without_status_returns_before_its_kernels_finish():
    """VERDICT r05 item 6 (SURVEY §8(b) threading): with no status word the banded call queues its launch and the
    guarded fallback and returns; a 2000-step call at the bench hierarchy (~17 ms of device time) returns to the host in
    a small fraction of it."""
    import time
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.deom import ado_coefficients
    sol = _spin_boson(12)
    sol.check_()
    sol.init_()
    dev = torch.device("cuda", 0)
    ns, K, nmax = sol.nsys, sol.nind, sol.nmax
    b = sol.bath
    coef, damp = ado_coefficients(sol.keys, np.asarray(b.etal), np.asarray(b.etar), np.asarray(b.etaa),
                                  np.asarray(b.expn), sol.lmax)
    c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
    ados = torch.zeros((nmax, ns, ns), dtype=torch.complex128, device=dev)
    ados[0, 0, 0] = 1
    H, Q = c128(sol.system), c128(np.asarray(sol.coupling, dtype=complex).reshape(-1, ns, ns))
    coef_t, damp_t, mode_t = c128(coef), c128(damp), i32(b.mode)
    bt = sol.band_tables(dev, 256)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)

    def call(nt):
        rc = lib.qd_deom_rk4_banded(ados.data_ptr(), nmax, K, ns, *bt.args(), coef_t.data_ptr(), damp_t.data_ptr(),
                                    mode_t.data_ptr(), Q.shape[0], H.data_ptr(), None, Q.data_ptr(), None, None, None,
                                    0.002, nt, None, None, 0, None, None, st)
        _lib.check(rc, "qd_deom_rk4_banded")

    call(5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call(2000)
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"host return {host * 1e3:.2f} ms of {total * 1e3:.2f} ms")
    assert host < 0.25 * total, (host, total)
    tr = torch.diagonal(ados[0]).sum().item()
    assert abs(tr - 1) < 1e-10


def test_banded_cooperative_and_plain_launch_agree():
    """The cooperative launch (default) and the plain launch (QD_OPT_COOP_LAUNCH = 0) give identical results (a band
    only ever consumes the tagged values, whatever the timing)."""
    from conftest import qd_option
    sol = _spin_boson(12)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    a, a_ados = _run(sol, rho0, 0.005, 5, 256)
    with qd_option("coop", 0):
        b, b_ados = _run(sol, rho0, 0.005, 5, 256)
    assert np.array_equal(a, b) and np.array_equal(a_ados, b_ados)


def test_band_table_cache_keyed_on_ns_and_modes():
    """band_tables' cache key includes ns and the mode count: a solver whose system size changes between
    runs re-plans instead of reusing stale, unchecked tables."""
    from pyqed_amd._util import default_device
    dev = default_device()
    sol = _spin_boson(5)
    sol.check_()
    sol.init_()
    t1 = sol.band_tables(dev, 4)
    assert sol._band_cache[0][-2:] == (2, 1)
    assert sol.band_tables(dev, 4) is t1


@pytest.mark.parametrize("pulsed", [False, True])
def test_banded_call_replays_from_a_graph(pulsed):
    """One banded call (16 bands, spin-boson L = 5) captured into a HIP graph and replayed three times equals three
    chained direct calls bit for bit: the call's
    scratch belongs to the graph (qd_runtime.hip capture_alloc), its fills are kernels, and the driven run's pulse
    values are uploaded at capture time."""
    sol = _spin_boson(5, npsd=3, pulses=pulsed)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    ref, ref_ados = _run(sol, rho0, 0.01, 12, 16, calls=3)
    out, ados = _run(sol, rho0, 0.01, 12, 16, calls=3, graph=True)
    assert np.array_equal(out, ref) and np.array_equal(ados, ref_ados)
