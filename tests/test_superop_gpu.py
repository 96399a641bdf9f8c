"""Dense Liouville-space path on the GPU (superop.hip): the device-built superoperators (qd_superop_lindblad,
qd_superop_from_glf) and the RK4 on vec(rho) (qd_superop_rk4: VALU GEMV for small batches, MFMA GEMM stages for
B >= 48) against the oracle's commutator-form RK4 and the reference's Redfield tensor at N = 128."""
import numpy as np
import pytest

from conftest import SPECTRA, load_golden, relerr

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.device("cuda", 0))


def test_lindblad_superop_builder_matches_host_kron():
    """qd_superop_lindblad == superoperator.liouvillian's host kron assembly (superoperator.py:29-58) and
    L vec(rho) == vec(oqs.liouvillian(rho)) (oracle, oqs.py:697-714), also for a non-Hermitian H."""
    from oracle import lindblad as olb
    from pyqed_amd.oqs import lindblad_superop
    from pyqed_amd.superoperator import liouvillian
    N = 9
    H, cs = olb.synthetic_lindblad(N, nc=2)
    rng = np.random.default_rng(3)
    Hn = H + 0.3 * (rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    for h in (H, Hn):
        L = lindblad_superop(_t(h), _t(np.array(cs))).cpu().numpy()
        Lh = liouvillian(h, list(cs))
        Lh = Lh.toarray() if hasattr(Lh, "toarray") else np.asarray(Lh)
        assert relerr(L, Lh) < 1e-14
        rho = olb.random_pure_states(1, N)[0] + 0.1j * rng.standard_normal((N, N))
        assert relerr(L @ rho.reshape(-1), olb.liouvillian(rho, h, cs).reshape(-1)) < 1e-13


@pytest.mark.parametrize("N,B", [(16, 1), (16, 5), (24, 11), (64, 1), (64, 3), (40, 50), (64, 64), (128, 1),
                                 (128, 64)])
def test_superop_rk4_matches_oracle(N, B, monkeypatch):
    """RK4 on vec(rho) with the device-built dense L vs the oracle's commutator-form RK4 (same linear ODE, same RK4:
    agreement to rounding).  B < 48: GEMV path (groups of <= 8 vectors); B >= 48: MFMA GEMM stages (N = 40 pads
    N^2 = 1600 to 1664); N = 128 is the BASELINE config d1 size (L = 4 GiB)."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd.oqs import lindblad_superop, superop_rk4
    H, cs = olb.synthetic_lindblad(N, nc=1)
    rho0 = olb.random_pure_states(B, N, seed=N + B)
    steps, dt = 3, 0.02
    L = lindblad_superop(_t(H), _t(np.array(cs)))
    v = _t(rho0.reshape(B, N * N))
    W = _t(np.eye(N, dtype=complex).reshape(1, N * N))  # vec(I^T): Tr(rho)
    obs, snap = superop_rk4(L, v, dt, steps, W, save_every=1)
    torch.cuda.synchronize()
    sel = sorted({0, B // 2, B - 1})
    ref = olb.lindblad_batch(H, cs, rho0[sel], dt, steps)
    got = v.cpu().numpy().reshape(B, N, N)[sel]
    assert relerr(got, ref) < TOL
    assert np.allclose(obs.cpu().numpy()[:, :, 0], 1.0, atol=1e-12)  # trace kept at every step
    s = snap.cpu().numpy()
    assert s.shape == (B, steps, N * N) and relerr(s[sel, -1].reshape(len(sel), N, N), ref) < TOL
    del L
    torch.cuda.empty_cache()


@pytest.mark.parametrize("B,path", [(8, "superop_gemv"), (64, "superop_gemm")])
def test_superop_gemm_and_gemv_paths_match_oracle(B, path):
    """Batches below 48 vectors run GEMV stages, from 48 the MFMA GEMM stages (qd_take_path): both against the
    oracle's Lindblad RK4 (oqs.py:697-714) on a spread of members."""
    import torch
    from oracle import lindblad as olb
    from pyqed_amd.oqs import lindblad_superop, superop_rk4
    from conftest import took
    N = 32
    H, cs = olb.synthetic_lindblad(N, nc=2)
    rho0 = olb.random_pure_states(B, N, seed=9)
    L = lindblad_superop(_t(H), _t(np.array(cs)))
    v = _t(rho0.reshape(B, N * N))
    took("")
    superop_rk4(L, v, 0.02, 4)
    hit, got = took(path)
    assert hit, got
    sel = [0, B // 2, B - 1]
    ref = olb.lindblad_batch(H, cs, rho0[sel], 0.02, 4)
    assert relerr(v.cpu().numpy().reshape(B, N, N)[sel], ref) < TOL


def test_redfield_superop_n128_matches_reference_tensor_and_evolution():
    """Config d1 Redfield at N = 128: the device-built R (qd_superop_from_glf on RedfieldSolver.glf_terms) equals the
    reference's csr R (oqs.py:519-570) on the fixture's rows, and 6 RK4 steps of R vec(rho~) (_redfield, oqs.py:
    364-459, on the HBM-bound GEMV) reproduce the reference's observables and final state."""
    import torch
    from pyqed_amd import RedfieldSolver
    from pyqed_amd.oqs import glf_superop, superop_rk4
    g = load_golden("redfield_n128")
    sol = RedfieldSolver(g["H"], c_ops=[g["a_op"]], spectra=[SPECTRA[str(g["spectrum"])]])
    P, Q, Ls, Rs = sol.glf_terms()
    N = P.shape[0]
    R = glf_superop(_t(P), _t(Q), _t(np.array(Ls)), _t(np.array(Rs)))
    rows = torch.from_numpy(g["R_row_index"]).to(R.device)
    assert relerr(R[rows].cpu().numpy(), g["R_rows"]) < 1e-12
    V = sol.evecs
    rho_eb = V.conj().T @ g["rho0"] @ V
    E_eb = np.array([V.conj().T @ e @ V for e in g["E"]])
    v = _t(rho_eb.reshape(1, N * N))
    W = _t(np.array([e.T.reshape(-1) for e in E_eb]))
    obs, _ = superop_rk4(R, v, float(g["dt"]), int(g["Nt"]), W)
    assert relerr(obs.cpu().numpy()[0, 1:], g["observables"]) < TOL
    fin = v.cpu().numpy().reshape(N, N)
    assert relerr(V @ fin @ V.conj().T, g["rho_final"]) < TOL
    del R
    torch.cuda.empty_cache()
