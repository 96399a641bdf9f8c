"""Library calls captured into a HIP graph (torch.cuda.graph): a captured call's scratch is a buffer the graph owns
(qd_runtime.hip capture_alloc: released when the graph is destroyed), so it neither waits on events recorded outside
the capture nor shares an arena slab with uncaptured calls, and its fills are kernels, not memset nodes.  Replays
equal direct calls bit for bit, sequence after sequence."""
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


def _replays(g, x, x0, side, sequences=3, replays=2):
    """States after `replays` replays of g from x0, once per sequence: alternately on the current (null) stream and
    on the side stream, with no host sync between the copy and the replays."""
    outs = []
    for k in range(sequences):
        if k % 2:
            with torch.cuda.stream(side):
                x.copy_(x0)
                for _ in range(replays):
                    g.replay()
        else:
            x.copy_(x0)
            for _ in range(replays):
                g.replay()
        torch.cuda.synchronize()
        outs.append(x.clone())
    return outs


@pytest.mark.parametrize("path,herm", [("single", True), ("single", False), ("split", True), ("split", False),
                                       ("persistent", True), ("persistent", False)])
def test_lindblad_call_replays_repeat_bit_for_bit(path, herm):
    """One N = 128 trajectory captured on each Lindblad path (the single-trajectory hand-off launch, the split path's
    dependent launches with their arrival tickets, the persistent kernel): every sequence of two replays equals two
    direct calls bit for bit, sequence after sequence.  Round 6 found later sequences wrong on this ROCm while
    captured scratch came from stream-ordered graph allocations and the tickets / flags were set by memset nodes;
    captured scratch is now a buffer the graph owns and every fill is a kernel (qd_runtime.hip)."""
    from conftest import qd_option
    from oracle import lindblad as olb
    from pyqed_amd import _lib, lindblad_rk4
    dev = torch.device("cuda", 0)
    N = 128
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    r0 = torch.from_numpy(olb.random_pure_states(1, N, seed=12)).to(dev)
    s = torch.cuda.Stream(dev)
    with qd_option("glf_path", path):
        ref = r0.clone()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            for _ in range(2):
                lindblad_rk4(Ht, Ct, ref, 1e-3, 6, hermitian=herm, stream=s.cuda_stream)
        torch.cuda.synchronize()
        x = r0.clone()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        _lib.take_path()
        with torch.cuda.graph(g, stream=s):
            lindblad_rk4(Ht, Ct, x, 1e-3, 6, hermitian=herm, stream=s.cuda_stream)
        taken = _lib.take_path()
    assert ("glf_single" in taken) == (path == "single"), taken
    for k, out in enumerate(_replays(g, x, r0, s)):
        assert torch.equal(out, ref), (k, float((out - ref).abs().max()))


def test_graph_scratch_is_released_with_the_graph():
    """A captured call's scratch is owned by the graph: destroying the graph hands it back, and the next uncaptured
    call frees it (device memory returns to its level before the capture)."""
    import gc
    from oracle import lindblad as olb
    from pyqed_amd import lindblad_rk4
    dev = torch.device("cuda", 0)
    N, B = 128, 64
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    x = torch.from_numpy(olb.random_pure_states(B, N, seed=3)).to(dev)
    s = torch.cuda.Stream(dev)
    y = x.clone()
    lindblad_rk4(Ht, Ct, y, 1e-3, 2, hermitian=False)   # the arena's slab for this shape exists before the baseline
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(dev)[0]
    for _ in range(3):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            lindblad_rk4(Ht, Ct, x, 1e-3, 2, hermitian=False, stream=s.cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        held = free0 - torch.cuda.mem_get_info(dev)[0]
        assert held >= B * N * N * 16   # the graph holds at least one state-sized buffer
        del g
        gc.collect()
        lindblad_rk4(Ht, Ct, y, 1e-3, 2, hermitian=False)   # an uncaptured call frees what destroyed graphs released
        torch.cuda.synchronize()
        assert free0 - torch.cuda.mem_get_info(dev)[0] < 64 << 20


@pytest.mark.parametrize("n", [64, 60])
def test_spo3_separable_call_replays_from_a_graph(n):
    """qd_spo3_run_axes captured once (64^3: the separable register-FFT passes with their device-side axis factors;
    60^3: the MFMA axis products) and replayed twice equals two direct calls bit for bit."""
    from pyqed_amd import _lib
    from pyqed_amd.wpd import SPO3, axis_propagator
    dev = torch.device("cuda", 0)
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    sol = SPO3(x, x, x, masses=[1.0, 1.2, 0.9], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)], [[[0, 1], 0.2 * X]])
    sol.build(0.05)
    psi0 = np.zeros((n, n, n, 2), complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 0.3j * Y)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eVh = t(sol.exp_V_half)
    m = [t(axis_propagator(k, ma, 0.05)) for k, ma in zip((sol.kx, sol.ky, sol.kz), sol.masses)]
    lib = _lib.load()
    s = torch.cuda.Stream(dev)

    def run(psi):
        _lib.check(lib.qd_spo3_run_axes(psi.data_ptr(), eVh.data_ptr(), *(v.data_ptr() for v in m), n, n, n, 2, 3, 3,
                                        None, s.cuda_stream), "qd_spo3_run_axes")
    ref = t(psi0)
    with torch.cuda.stream(s):
        run(ref)
        run(ref)
    torch.cuda.synchronize()
    xg = t(psi0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        run(xg)
    for out in _replays(g, xg, t(psi0), s):
        assert torch.equal(out, ref)
