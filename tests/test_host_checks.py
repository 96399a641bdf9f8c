"""Host-side logic of the Python layer that runs without a GPU: the cached Hermiticity check that lindblad_rk4 uses
to gate the Hermitian kernel (pyqed_amd/oqs.py)."""
import torch

from pyqed_amd.oqs import _is_hermitian_cached


def test_hermitian_check_cache_follows_the_tensor():
    a = torch.randn(6, 6, dtype=torch.complex128)
    h = a + a.conj().T
    assert _is_hermitian_cached(h) and _is_hermitian_cached(h)   # second call: cached
    h[0, 1] += 1.0                                                  # in place: _version bumps, the check reruns
    assert not _is_hermitian_cached(h)
    assert not _is_hermitian_cached(a)
    # a new tensor (possibly at a recycled id) is checked afresh
    for _ in range(5):
        b = torch.randn(6, 6, dtype=torch.complex128)
        assert not _is_hermitian_cached(b)
        del b
        c = torch.eye(6, dtype=torch.complex128)
        assert _is_hermitian_cached(c)
        del c


def test_hermitian_check_cache_follows_a_repointed_data():
    """swapping the storage under the same tensor object (h.data = ...) must not reuse a cached True."""
    a = torch.randn(6, 6, dtype=torch.complex128)
    h = a + a.conj().T
    assert _is_hermitian_cached(h)
    h.data = torch.randn(6, 6, dtype=torch.complex128)
    assert not _is_hermitian_cached(h)


def test_dyn_superop_probe_is_the_generator_and_refuses_nonlinear():
    """correlation_3p_1t's host probe of a general dyn(rho, H, c_ops) (VERDICT r04 missing #4): its matrix applied to
    row-major vec(rho) equals dyn(rho) for dense and scipy.sparse operators, and a nonlinear dyn raises."""
    import numpy as np
    import pytest
    from scipy.sparse import csr_matrix
    from oracle import lindblad as olb
    from pyqed_amd.correlation import _dyn_superop
    H, cs = olb.synthetic_lindblad(5, nc=1)
    rho = olb.random_pure_states(1, 5, seed=4)[0]
    for Hx, cx in ((H, cs), (csr_matrix(H), [csr_matrix(c) for c in cs])):
        L = _dyn_superop(olb.liouvillian, Hx, cx, 5)
        assert np.allclose(L @ rho.ravel(), olb.liouvillian(rho, H, cs).ravel(), rtol=1e-12, atol=1e-14)
    with pytest.raises(ValueError):
        _dyn_superop(lambda r, H, c: r @ r, H, cs, 5)
