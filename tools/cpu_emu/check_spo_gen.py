"""Host check of spo_gen.hip through the flat-loop emulation (tools/cpu_emu/libemu_spo.so) against oracle/spo.py.
Debug tool: `python tools/cpu_emu/check_spo_gen.py` from the repo root after building libemu_spo.so."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from oracle import spo as osp  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libemu_spo.so"))
P = ctypes.c_void_p


def ptr(a):
    return None if a is None else a.ctypes.data_as(P)


def unitary_ops(shape, ns, rng):
    a = rng.standard_normal(shape + (ns, ns)) + 1j * rng.standard_normal(shape + (ns, ns))
    h = (a + np.conj(np.swapaxes(a, -1, -2))) / 4
    w, u = np.linalg.eigh(h)
    ud = np.conj(np.swapaxes(u, -1, -2))
    return (u * np.exp(-1j * w)[..., None, :]) @ ud, (u * np.exp(-0.5j * w)[..., None, :]) @ ud


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300)


def check_nd(dims, ns, nt=3, nout=1, merged=False, jacobi=False, seed=0):
    rng = np.random.default_rng(seed)
    shape = tuple(dims)
    eV, eVh = unitary_ops(shape, ns, rng)
    K = np.exp(-1j * rng.uniform(0, 6, shape))
    psi0 = rng.standard_normal(shape + (ns,)) + 1j * rng.standard_normal(shape + (ns,))
    psi = psi0.copy()
    nsnap = nt // nout
    snap = np.zeros((max(nsnap, 1),) + psi.shape, complex)
    Ky = None
    if jacobi:
        Kx = np.exp(-1j * rng.uniform(0, 6, dims[0]))
        Ky = np.exp(-1j * rng.uniform(0, 6, shape))
        K = np.ascontiguousarray(np.broadcast_to(Kx[:, None], shape))
    d = (ctypes.c_int * len(dims))(*dims)
    rc = lib.emu_spo_nd(ptr(psi), ptr(eVh), ptr(eV) if merged else None, ptr(K), ptr(Ky), d, len(dims), ns,
                        (nt // nout) * nout, nout, ptr(snap) if nsnap else None)
    assert rc == 0, rc
    if len(dims) == 3:
        states, fin = osp.spo3_run(eVh, K, psi0, nt, nout)
        ref_snaps = states
    else:
        keo = osp.keo_jacobi(K[:, 0], Ky) if jacobi else osp.keo_linear(K)
        if merged:
            states, fin = osp.spo2_merged_run(eV, eVh, keo, psi0, nt, nout)
        else:
            states, fin = osp.spo2_strang_run(eVh, keo, psi0, nt, nout)
        ref_snaps = states[1:]
    e1 = rel(psi, fin)
    e2 = max([rel(snap[k], ref_snaps[k]) for k in range(nsnap)] + [0])
    return e1, e2


def check_1d(nx, nt=5, nout=2, B=2, seed=0):
    rng = np.random.default_rng(seed)
    x = np.linspace(-8, 8, nx)
    V = 0.5 * x ** 2
    eV, eVh, eK = osp.spo1d_ops(x, V, 1.0, 0.01)
    psi0 = rng.standard_normal((B, nx)) + 1j * rng.standard_normal((B, nx))
    psi = psi0.copy()
    nsnap = max(nt // nout - 1, 0)
    snap = np.zeros((B, max(nsnap, 1), nx), complex)
    rc = lib.emu_spo1d(ptr(psi), ptr(eV), ptr(eVh), ptr(eK), nx, B, nt, nout, ptr(snap) if nsnap else None)
    assert rc == 0
    err = 0
    for b in range(B):
        sl, fin = osp.spo1d_run(x, V, psi0[b], 0.01, nt, nout)
        err = max(err, rel(psi[b], fin), *[rel(snap[b, k], sl[k]) for k in range(nsnap)])
    return err


if __name__ == "__main__":
    worst = 0
    for kind in ("0", "1", "2"):
        os.environ["QD_SPO_FORCE_KIND"] = kind
        cases = [((20, 20), 2), ((96, 80), 2), ((7, 11), 3), ((67, 5), 1), ((12, 10), 5), ((1, 9), 2)]
        for dims, ns in cases:
            e = check_nd(dims, ns)
            print("kind", kind, "2d", dims, ns, e)
            worst = max(worst, *e)
        for dims, ns in [((24, 20, 18), 2), ((5, 6, 7), 3)]:
            e = check_nd(dims, ns, nt=2)
            print("kind", kind, "3d", dims, ns, e)
            worst = max(worst, *e)
        e = check_nd((20, 30), 2, nt=4, nout=2, merged=True)
        print("kind", kind, "merged", e)
        worst = max(worst, *e)
        e = check_nd((18, 14), 2, nt=4, nout=2, jacobi=True)
        print("kind", kind, "jacobi", e)
        worst = max(worst, *e)
        for nx in (50, 97, 200, 127):
            e = check_1d(nx)
            print("kind", kind, "1d", nx, e)
            worst = max(worst, e)
    os.environ["QD_SPO_FORCE_KIND"] = "0"
    for nx in (2048, 6000, 2 * 2053):
        e = check_1d(nx, nt=3, nout=1, B=1)
        print("auto 1d", nx, e)
        worst = max(worst, e)
    print("WORST", worst)
