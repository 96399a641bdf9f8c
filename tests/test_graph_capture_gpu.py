"""Library calls captured into a HIP graph (torch.cuda.graph): scratch comes from stream-ordered allocations that
become the graph's own alloc / free nodes (qd_runtime.hip workspace), so a captured call neither waits on events
recorded outside the capture nor shares an arena slab with later uncaptured calls.  Replays equal direct calls."""
import numpy as np
import pytest
import torch

from conftest import relerr

pytestmark = pytest.mark.gpu


def _spo_inputs(dev, n=256, ns=2, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((n, n, ns, ns)) + 1j * rng.standard_normal((n, n, ns, ns))
    h = (a + np.conj(np.swapaxes(a, -1, -2))) / 4
    w, u = np.linalg.eigh(h)
    U = (u * np.exp(-0.5j * w)[..., None, :]) @ np.conj(np.swapaxes(u, -1, -2))
    K = np.exp(-1j * rng.uniform(0, 6, (n, n)))
    psi = rng.standard_normal((n, n, ns)) + 0j
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    return t(U), t(K), t(psi)


@pytest.mark.parametrize("n", [256, 200])
def test_spo2_call_replays_from_a_graph(n):
    """SPO2 Strang steps (power-of-two and any-grid engines, the latter with arena scratch) captured once and
    replayed twice: the state equals two direct calls."""
    from pyqed_amd import _lib
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    U, K, psi = _spo_inputs(dev, n)
    ref = psi.clone()
    s = torch.cuda.Stream(dev)

    def run(x):
        _lib.check(lib.qd_spo2_run_ex(x.data_ptr(), U.data_ptr(), None, K.data_ptr(), None, n, n, 2, 5, 5, None,
                                      s.cuda_stream), "qd_spo2_run_ex")
    with torch.cuda.stream(s):
        run(ref)
        run(ref)
    torch.cuda.synchronize()
    x = psi.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        run(x)
    x.copy_(psi)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert relerr(x.cpu().numpy(), ref.cpu().numpy()) < 1e-13


def test_lindblad_batch_replays_from_a_graph():
    """The persistent Lindblad kernel (256 matrices, Hermitian form) and its scratch inside a graph; uncaptured calls
    before and after the capture keep using the arena."""
    from oracle import lindblad as olb
    from pyqed_amd import _lib, lindblad_rk4
    dev = torch.device("cuda", 0)
    N, B = 32, 256
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht = torch.from_numpy(H).to(dev)
    Ct = torch.from_numpy(np.array(cs)).to(dev)
    rho0 = torch.from_numpy(olb.random_pure_states(B, N, seed=5)).to(dev)
    s = torch.cuda.Stream(dev)
    ref = rho0.clone()
    with torch.cuda.stream(s):
        lindblad_rk4(Ht, Ct, ref, 1e-2, 6, hermitian=True, stream=s.cuda_stream)
    torch.cuda.synchronize()
    x = rho0.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        lindblad_rk4(Ht, Ct, x, 1e-2, 3, hermitian=True, stream=s.cuda_stream)
    x.copy_(rho0)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert relerr(x.cpu().numpy(), ref.cpu().numpy()) < 1e-12
    y = rho0.clone()   # an uncaptured call after the capture
    lindblad_rk4(Ht, Ct, y, 1e-2, 6, hermitian=True)
    torch.cuda.synchronize()
    assert relerr(y.cpu().numpy(), ref.cpu().numpy()) < 1e-12
