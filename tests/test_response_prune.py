"""Structural-zero pruning of the 2DES ensemble sums (pyqed_amd.response): the compact rectangular
operands reproduce the full eigen-form sum S[i,k] = (-i)^3 sum_m sum_pq alpha_mp e^{lam_mp t3_i} Mt_mpq
beta_mq e^{lam_mq t1_k} (oqs.py:268-357 at fixed t2).  Host tests check the compaction algebra with numpy;
GPU tests compare the pruned HIP path with the unpruned one and with the closed form."""
import numpy as np
import pytest
import torch

from conftest import relerr


def _closed_form(lam, alpha, Mt, beta, t3, t1):
    return sum((alpha[m][None, :] * np.exp(np.outer(t3, lam[m]))) @
               ((Mt[m] * beta[m][None, :]) @ np.exp(np.outer(lam[m], t1))) for m in range(len(lam))) * (-1j) ** 3


def _inputs(M, nL, zero_a, zero_b, seed, partial=()):
    rng = np.random.default_rng(seed)
    lam = -rng.uniform(0.01, 0.2, (M, nL)) + 1j * rng.uniform(-2, 2, (M, nL))
    alpha, beta = (rng.standard_normal((M, nL)) + 1j * rng.standard_normal((M, nL)) for _ in range(2))
    Mt = rng.standard_normal((M, nL, nL)) + 1j * rng.standard_normal((M, nL, nL))
    alpha[:, list(zero_a)] = 0
    beta[:, list(zero_b)] = 0
    for p in partial:                       # zero for some members only: must be kept
        alpha[: M // 2, p] = 0
    return lam, alpha, Mt, beta


def _ladder(M, seed=3):
    from pyqed_amd.response import ensemble_factors_bc, redfield_superop_batch
    from pyqed_amd.superoperator import operator_to_superoperator
    rng = np.random.default_rng(seed)
    E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((M, 3))
    R = redfield_superop_batch(E, np.diag([0.0, 1.0, 2.0]), np.full((M, 3, 3), 0.05))
    lam, U1 = np.linalg.eig(R)
    U2 = np.linalg.inv(U1)
    dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
    ops = [operator_to_superoperator(dip, s).toarray() for s in "lccc"]
    rho0v = np.zeros(9, complex); rho0v[0] = 1
    return (lam,) + ensemble_factors_bc(lam, U1, U2, ops, rho0v)


# ----------------------------------------------------------------------------- host (no GPU)
@pytest.mark.parametrize("zero_a,zero_b,swap", [((0, 2, 4, 6, 8), (0, 2, 4, 5, 6, 7, 8), True),
                                                ((0, 1, 2, 3, 4, 5, 8), (0, 2, 4), False)])
def test_fixed_t2_compaction_algebra(zero_a, zero_b, swap):
    """_prune_fixed_t2 on CPU tensors: the compact (possibly swapped) operands give the same sum."""
    from pyqed_amd.response import _prune_fixed_t2
    lam, alpha, Mt, beta = _inputs(6, 9, zero_a, zero_b, seed=len(zero_a))
    t3, t1 = 0.5 * np.arange(20), 0.3 * np.arange(13)
    T = lambda x: torch.from_numpy(x)
    sw, ax, lx, Mc, bz, lz = (x.numpy() if isinstance(x, torch.Tensor) else x
                              for x in _prune_fixed_t2(T(lam), T(alpha), T(Mt), T(beta)))
    assert sw == swap
    assert ax.shape[1] == min(9 - len(zero_a), 9 - len(zero_b))
    ga, gb = (t1, t3) if sw else (t3, t1)
    S = sum((ax[m][None, :] * np.exp(np.outer(ga, lx[m]))) @ ((Mc[m] * bz[m][None, :]) @ np.exp(np.outer(lz[m], gb)))
            for m in range(len(lam))) * (-1j) ** 3
    ref = _closed_form(lam, alpha, Mt, beta, t3, t1)
    assert relerr(S.T if sw else S, ref) < 1e-13


def test_t2_compaction_ladder_sets():
    """The 3-level ladder 'lccc' pathways keep p in {1,3,5,7}, r in {0,2,4,6}, q in {1,3} (exact zeros)."""
    from pyqed_amd.response import _prune_t2
    lam, alpha, B, C, beta = _ladder(16)
    T = lambda x: torch.from_numpy(x)
    ap, lp, Bc, lr, Cc, bq, lq = _prune_t2(T(lam), T(alpha), T(B), T(C), T(beta))
    assert (ap.shape[1], lr.shape[1], bq.shape[1]) == (4, 4, 2)
    t3, t1, t2 = 0.5 * np.arange(12), 0.4 * np.arange(9), 3.7
    full = sum((alpha[m][None, :] * np.exp(np.outer(t3, lam[m]))) @ (B[m] * np.exp(lam[m] * t2)[None, :]) @ C[m]
               @ (beta[m][:, None] * np.exp(np.outer(lam[m], t1))) for m in range(16))
    ap, lp, Bc, lr, Cc, bq, lq = (x.numpy() for x in (ap, lp, Bc, lr, Cc, bq, lq))
    comp = sum((ap[m][None, :] * np.exp(np.outer(t3, lp[m]))) @ (Bc[m] * np.exp(lr[m] * t2)[None, :]) @ Cc[m]
               @ (bq[m][:, None] * np.exp(np.outer(lq[m], t1))) for m in range(16))
    assert relerr(comp, full) < 1e-13


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("zero_a,zero_b,partial", [((0, 2, 4, 6, 8), (0, 2, 4, 5, 6, 7, 8), ()),
                                                   ((0, 1, 2, 3, 4, 5, 8), (0, 2, 4), ()),
                                                   ((0, 2), (1, 3, 5, 7), (4, 6)),
                                                   ((), (), ())])
@pytest.mark.parametrize("grids", ["uniform", "array", "mixed"])
def test_pruned_matches_unpruned_and_closed_form(zero_a, zero_b, partial, grids):
    from pyqed_amd.response import response2d_ensemble
    dev = torch.device("cuda", 0)
    M = 37
    lam, alpha, Mt, beta = _inputs(M, 9, zero_a, zero_b, seed=7 + len(zero_a), partial=partial)
    t3, t1 = 0.5 * np.arange(130), 0.3 * np.arange(200)
    if grids == "mixed":
        t3 = np.sort(np.random.default_rng(1).uniform(0, 60, 130))
    g3, g1 = (torch.from_numpy(t3).to(dev), torch.from_numpy(t1).to(dev)) if grids == "array" else (t3, t1)
    ref = _closed_form(lam, alpha, Mt, beta, t3, t1)
    full = response2d_ensemble(lam, alpha, Mt, beta, g3, g1, prune=False).cpu().numpy()
    pr = response2d_ensemble(lam, alpha, Mt, beta, g3, g1).cpu().numpy()
    assert relerr(full, ref) < 1e-12
    assert relerr(pr, ref) < 1e-12
    # accumulate into an existing grid (transposed reduce adds as well)
    acc = torch.from_numpy(full.copy()).to(dev)
    response2d_ensemble(lam, alpha, Mt, beta, g3, g1, out=acc, accumulate=True)
    assert relerr(acc.cpu().numpy(), 2 * ref) < 1e-12


@pytest.mark.gpu
def test_pruned_all_zero_and_cache_invalidation():
    from pyqed_amd.response import response2d_ensemble
    dev = torch.device("cuda", 0)
    lam, alpha, Mt, beta = _inputs(5, 9, range(9), (), seed=3)
    t = 0.5 * np.arange(64)
    out = torch.full((64, 64), 1 + 1j, dtype=torch.complex128, device=dev)
    response2d_ensemble(lam, alpha, Mt, beta, t, t, out=out, accumulate=True)
    assert np.all(out.cpu().numpy() == 1 + 1j)
    assert np.all(response2d_ensemble(lam, alpha, Mt, beta, t, t).cpu().numpy() == 0)
    # device inputs: an in-place change of alpha bumps its version, so the pruned form is rebuilt
    lam2, alpha2, Mt2, beta2 = _inputs(5, 9, (0, 2), (1,), seed=4)
    tens = [torch.from_numpy(x).to(dev) for x in (lam2, alpha2, Mt2, beta2)]
    a = response2d_ensemble(*tens, t, t).cpu().numpy()
    assert relerr(a, _closed_form(lam2, alpha2, Mt2, beta2, t, t)) < 1e-12
    alpha2[:, 0] = 0.5
    tens[1].copy_(torch.from_numpy(alpha2))
    b = response2d_ensemble(*tens, t, t).cpu().numpy()
    assert relerr(b, _closed_form(lam2, alpha2, Mt2, beta2, t, t)) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("M,n3,n1", [(200, 256, 256), (9, 70, 130)])
def test_t2scan_pruned_matches_unpruned(M, n3, n1):
    from pyqed_amd.response import T2Scan
    lam, alpha, B, C, beta = _ladder(M, seed=M)
    t3, t1, t2 = 0.5 * np.arange(n3), 0.4 * np.arange(n1), np.array([0.0, 2.0, 7.5])
    a = T2Scan(lam, alpha, B, C, beta, t3, t1)
    assert a.index_sizes == (4, 4, 2)
    pr = a.apply(t2).cpu().numpy()
    full = T2Scan(lam, alpha, B, C, beta, t3, t1, prune=False).apply(t2).cpu().numpy()
    assert relerr(pr, full) < 1e-12


@pytest.mark.gpu
def test_large_k_generated_x_operand():
    """K = 36k (no zero columns): the split plan takes 128-blocks, and the uniform t3 side is generated in
    the GEMM staging from the coarse/fine exponential tables (ens_xtab_kernel) instead of a materialised X.
    Checked against the closed form and against the array-grid path (materialised X, direct exponentials)."""
    from pyqed_amd.response import response2d_ensemble
    dev = torch.device("cuda", 0)
    M = 4000
    lam, alpha, Mt, beta = _inputs(M, 9, (), (), seed=5)
    lam = lam * 0.3
    t3, t1 = 0.5 * np.arange(200), 0.4 * np.arange(150)
    S = response2d_ensemble(lam, alpha, Mt, beta, t3, t1).cpu().numpy()
    ref = np.zeros((len(t3), len(t1)), complex)
    for lo in range(0, M, 500):
        sl = slice(lo, lo + 500)
        X = alpha[sl][:, None, :] * np.exp(t3[None, :, None] * lam[sl][:, None, :])          # [m, i, p]
        Z = np.einsum("mpq,mqk->mpk", Mt[sl], beta[sl][:, :, None] * np.exp(lam[sl][:, :, None] * t1[None, None, :]))
        ref += np.einsum("mip,mpk->ik", X, Z)
    ref *= (-1j) ** 3
    assert relerr(S, ref) < 1e-12
    arr = response2d_ensemble(lam, alpha, Mt, beta, torch.from_numpy(t3).to(dev), torch.from_numpy(t1).to(dev))
    assert relerr(arr.cpu().numpy(), S) < 1e-13
