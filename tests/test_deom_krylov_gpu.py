"""Krylov form of DEOMSolver.correlation_4op_3t on the GPU (pyqed_amd/deom_krylov.py, qd_deom_apply): the stencil
operator P and its transposed-table form P^T against the assembled ADO Liouvillian (heom/deom.py:769-893), the
correlation against the reference fixture and the eigen form, and the bench hierarchy (L = 12, K = 5, n = 24,752,
whose dense P the reference cannot diagonalise) through the two orientations of the algorithm."""
import numpy as np
import pytest
import sympy as sp
import torch

from conftest import load_golden, relerr
from test_deom_krylov_cpu import _hierarchy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ns,npsd,L,nmod,B", [(2, 3, 4, 1, 1), (2, 3, 4, 1, 5), (3, 2, 3, 1, 2), (5, 1, 3, 1, 1),
                                              (2, 1, 4, 2, 3), (2, 8, 2, 1, 1)])
def test_deom_apply_is_the_generator_and_its_transpose(ns, npsd, L, nmod, B):
    from pyqed_amd import _lib
    from pyqed_amd.deom import ado_liouvillian
    from pyqed_amd.deom_krylov import DeomOperator, transposed_tables
    dev = torch.device("cuda", 0)
    sol, H, Q, coef, damp, mode = _hierarchy(ns, npsd, L, nmod)
    P = ado_liouvillian(sol.keys, sol._minus, sol._plus, coef, damp, H, Q, mode)
    mT, pT, cT = transposed_tables(sol._minus, sol._plus, coef)
    op = DeomOperator(dev, sol._minus, sol._plus, coef, damp, mode, H, Q, ns)
    opT = DeomOperator(dev, mT, pT, cT, damp, mode, H.T, np.swapaxes(Q, 1, 2), ns)
    rng = np.random.default_rng(7)
    x = rng.standard_normal((B, P.shape[0])) + 1j * rng.standard_normal((B, P.shape[0]))
    xd = torch.from_numpy(x).to(dev)
    y = torch.empty_like(xd)
    _lib.take_path()
    op.apply(xd, y, 0.75)
    torch.cuda.synchronize()
    assert "deom_apply" in _lib.take_path()
    assert relerr(y.cpu().numpy(), 0.75 * (x @ P.T)) < 1e-13
    opT.apply(xd, y, -2.0)
    assert relerr(y.cpu().numpy(), -2.0 * (x @ P)) < 1e-13


def test_taylor_graph_replay_equals_direct_substeps():
    """expv_taylor's graph form (one captured substep of 20 stencil launches and adds, replayed s times) equals the
    direct loop bit for bit and counts the same stencil launches; e^{PT} x against expm of the assembled P."""
    import scipy.linalg
    from pyqed_amd.deom import ado_liouvillian
    from pyqed_amd.deom_krylov import DeomOperator, expv_taylor
    dev = torch.device("cuda", 0)
    sol, H, Q, coef, damp, mode = _hierarchy(2, 3, 4, 1)
    P = ado_liouvillian(sol.keys, sol._minus, sol._plus, coef, damp, H, Q, mode)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((3, P.shape[0])) + 1j * rng.standard_normal((3, P.shape[0]))
    xd = torch.from_numpy(x).to(dev)
    ops = [DeomOperator(dev, sol._minus, sol._plus, coef, damp, mode, H, Q, 2) for _ in range(2)]
    T = 3.0 / ops[0].norm * 2.5   # several substeps
    yd, s1 = expv_taylor(ops[0], xd, T, graph=False)
    yg, s2 = expv_taylor(ops[1], xd, T, graph=True)
    torch.cuda.synchronize()
    assert s1 == s2 >= 2
    assert torch.equal(yd, yg)
    assert (ops[0].launches, ops[0].vec_applies) == (ops[1].launches, ops[1].vec_applies)
    assert relerr(yg.cpu().numpy(), x @ scipy.linalg.expm(P * T).T) < 1e-11


@pytest.mark.parametrize("k,S", [(1, 3), (7, 5), (300, 33), (2500, 2)])
def test_shifted_hessenberg_solve_matches_dense_solves(k, S):
    """qd_shifted_hessenberg_solve (one workgroup per shift, adjacent-row pivoting) against numpy.linalg.solve of every
    (-H_k - s I) y = beta e_1 and the host residual form (_shift_residuals), on a random Hessenberg matrix with a
    leading dimension wider than k."""
    from pyqed_amd.deom_krylov import _hess_solve_dev, _shift_residuals
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(k)
    m = k + 4
    H = np.triu(rng.standard_normal((m + 1, m)) + 1j * rng.standard_normal((m + 1, m)), -1)
    shifts = 1j * rng.uniform(-3, 3, S) + 0.2
    beta = 1.7
    Y, res = _hess_solve_dev(torch.from_numpy(H).to(dev), k, beta, shifts, True)
    Y = Y.cpu().numpy()
    for i, sft in enumerate(shifts):
        ref = np.linalg.solve(-H[:k, :k] - sft * np.eye(k), beta * np.eye(k)[:, 0])
        assert relerr(Y[i], ref) < 1e-10
    assert relerr(res.cpu().numpy(), _shift_residuals(H, k, beta, shifts)) < 1e-10
    _, res2 = _hess_solve_dev(torch.from_numpy(H).to(dev), k, beta, shifts, False)
    assert torch.equal(res, res2)


def _fixture_solver(g):
    from pyqed_amd.deom import Bath, DEOMSolver
    bath = Bath.__new__(Bath)
    bath.etal, bath.etar, bath.etaa, bath.expn = g["etal"], g["etar"], g["etaa"], g["expn"]
    bath.mode = np.zeros(len(g["expn"]), dtype=np.int64)
    return DEOMSolver(g["H"], np.zeros((2, 2), complex), bath, g["Q"], np.zeros((1, 2, 2), complex),
                      lambda t: 0, lambda t: 0, int(g["lmax"]))


def test_krylov_corr4_matches_reference_fixture():
    """The reference's own outputs (tests/golden/deom_corr4.npz, eig of its 140 x 140 P) from the Krylov form."""
    g = load_golden("deom_corr4")
    sx = g["Q"][0]
    sol = _fixture_solver(g)
    sol.corr4_method = "krylov"
    for lcr in ["llll", "lrlr", "lccc"]:
        cw = sol.correlation_4op_3t(sx, sx, sx, sx, g["rho0"], float(g["T"]), g["wx"], g["wy"], lcr=lcr)
        assert sol.last_corr4["method"] == "krylov"
        assert relerr(cw, g["cw_" + lcr]) < 1e-9, lcr
    with pytest.raises(ValueError):
        sol.correlation_4op_3t(sx, sx, sx, sx, g["rho0"], 0.5, g["wx"], g["wy"], if_full=False)


def test_krylov_corr4_auto_above_threshold_matches_eigen_form():
    """n = nmax ns^2 = 1320 >= KRYLOV_MIN_DIM takes the Krylov form by default; the eigen form (host eig of the
    1320 x 1320 P, the reference's algorithm) agrees."""
    from pyqed_amd.deom import KRYLOV_MIN_DIM, Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [3], [0] * 4)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 7)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    wx = np.linspace(-4.1, 4.3, 12)
    wy = np.linspace(-3.7, 4.9, 10)
    c = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, 0.4, wx, wy, lcr="lccc")
    assert sol.last_corr4["method"] == "krylov" and sol.last_corr4["n"] == 1320 >= KRYLOV_MIN_DIM
    sol.corr4_method = "eig"
    ref = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, 0.4, wx, wy, lcr="lccc")
    assert sol.last_corr4["method"] == "eig"
    assert relerr(c, ref) < 1e-9


def test_krylov_corr4_bench_hierarchy_orientations_agree():
    """L = 12, K = 5 (6188 ADOs, n = 24,752): the reference would diagonalise a 9.8 GB P.  The Krylov form's two
    orientations (e^{PT} on the right-hand vectors when n_wy <= n_wx, e^{P^T T} on the left-hand ones otherwise)
    share only the resolvent solves' definition, not their arithmetic order: they agree to 1e-9."""
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    wx = np.linspace(-4.1, 4.3, 8)
    wy = np.linspace(-3.7, 4.9, 6)
    c1 = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, 0.2, wx, wy)
    info1 = dict(sol.last_corr4)
    assert info1["method"] == "krylov" and info1["n"] == 24752
    c2 = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, 0.2, wx, np.concatenate([wy, [5.3, 6.1, 7.7]]))
    assert np.all(np.isfinite(c1))
    assert relerr(c2[:, :len(wy)], c1) < 1e-9, (info1, sol.last_corr4)


class _DenseOpDev:
    """A dense P on the device standing in for DeomOperator (test infrastructure only)."""

    def __init__(self, P, norm):
        self.P = torch.from_numpy(np.ascontiguousarray(P)).to("cuda:0")
        self.n = P.shape[0]
        self.dev = torch.device("cuda", 0)
        self.norm = norm

    def apply(self, x, y, alpha=1.0):
        y.copy_((alpha * (self.P @ x.reshape(-1, self.n).T).T).reshape(y.shape))
        return y


def test_delayed_cgs2_arnoldi_matches_cgs2():
    """qd_arnoldi_dcgs2_step (two basis passes per step, the re-orthogonalisation folded into the next projection)
    against the four-pass CGS2 loop: the same solutions of the shifted systems, on a random dense P and on the DEOM
    stencil operator; exact breakdowns (P = 0; b an eigenvector) end the solve with the exact answer."""
    from pyqed_amd import deom_krylov as dk
    from pyqed_amd.deom_krylov import DeomOperator, shifted_krylov_solve
    rng = np.random.default_rng(5)
    n = 300
    P = (rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))) / 20 - 2.0 * np.eye(n)
    b = torch.from_numpy(rng.standard_normal(n) + 1j * rng.standard_normal(n)).to("cuda:0")
    shifts = 1j * np.linspace(-3, 3, 7) + 0.1
    ref = np.linalg.solve(-P[None] - shifts[:, None, None] * np.eye(n)[None], b.cpu().numpy()[None, :, None])[..., 0]
    sol, H, Q, coef, damp, mode = _hierarchy(2, 3, 4, 1)
    op = DeomOperator(torch.device("cuda", 0), sol._minus, sol._plus, coef, damp, mode, H, Q, 2)
    bd = torch.from_numpy(rng.standard_normal(op.n) + 0j).to("cuda:0")
    out = {}
    try:
        for flag in (False, True):
            dk.ARNOLDI_DCGS2 = flag
            X, k = shifted_krylov_solve(_DenseOpDev(P, 1.0), b, shifts)
            Xd, kd = shifted_krylov_solve(op, bd, shifts)
            out[flag] = (X.cpu().numpy(), k, Xd.cpu().numpy(), kd)
            assert relerr(out[flag][0], ref) < 1e-10, (flag, k)
        assert relerr(out[True][2], out[False][2]) < 1e-11
        assert abs(out[True][1] - out[False][1]) <= 10 and abs(out[True][3] - out[False][3]) <= 10
        m = 12
        bz = torch.from_numpy(rng.standard_normal(m) + 0j).to("cuda:0")
        X, k = shifted_krylov_solve(_DenseOpDev(np.zeros((m, m), complex), 1.0), bz, shifts)
        assert k == 1 and np.all(np.isfinite(X.cpu().numpy()))
        assert relerr(X.cpu().numpy(), -bz.cpu().numpy()[None, :] / shifts[:, None]) < 1e-14
        Pd = np.diag(np.arange(m, dtype=complex) - 2.5)
        e = torch.zeros(m, dtype=torch.complex128, device="cuda:0")
        e[3] = 2.0
        X, k = shifted_krylov_solve(_DenseOpDev(Pd, 10.0), e, shifts)
        assert k == 1
        assert relerr(X.cpu().numpy(), e.cpu().numpy()[None, :] / (-Pd[3, 3] - shifts)[:, None]) < 1e-14
    finally:
        dk.ARNOLDI_DCGS2 = True
