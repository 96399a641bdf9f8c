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
