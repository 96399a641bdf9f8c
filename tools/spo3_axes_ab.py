"""SPO3 kinetic step: FFT passes (qd_spo3_run) against per-axis mode products on the MFMAs (qd_spo3_run_axes).

usage: python tools/spo3_axes_ab.py [steps] [sizes, comma separated]
Per grid (n^3 x 2, the examples/spo.py model): both entry points on the same device-resident state, HIP events over
`steps` Strang steps after a warm-up, the relative difference of the two results, and the per-point cost against 64^3.
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pyqed_amd import _lib  # noqa: E402
from pyqed_amd.wpd import SPO3, axis_propagator  # noqa: E402


def model(n, ns=2, dt=0.05):
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    sol = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=ns)
    sol.set_DPES([0.5 * ((X + (-1) ** a) ** 2 + Y ** 2 + Z ** 2) + 0.1 * a for a in range(ns)],
                 [[[a, a + 1], 0.2 * X] for a in range(ns - 1)])
    sol.build(dt)
    psi0 = np.zeros((n, n, n, ns), complex)
    psi0[..., ns - 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 0.3j * Y) / np.pi ** 0.75
    M = [axis_propagator(k, m, dt) for k, m in zip((sol.kx, sol.ky, sol.kz), sol.masses)]
    return sol, psi0, M


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    ref_us = None
    sizes = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 60, 48, 32]
    for n in sizes:
        sol, psi0, M = model(n)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        eVh, eK, Mt = t(sol.exp_V_half), t(sol.exp_K), [t(m) for m in M]
        out = {}
        for name in ("fft", "axes"):
            psi = t(psi0)

            def run(k):
                if name == "fft":
                    rc = lib.qd_spo3_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, n, 2, k, k, None, st)
                else:
                    rc = lib.qd_spo3_run_axes(psi.data_ptr(), eVh.data_ptr(), *(m.data_ptr() for m in Mt), n, n, n,
                                              2, k, k, None, st)
                _lib.check(rc, name)
            run(20)
            torch.cuda.synchronize()
            res = psi.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(steps)
            e1.record()
            torch.cuda.synchronize()
            out[name] = (e0.elapsed_time(e1) * 1e3 / steps, res)
        (tf, rf), (ta, ra) = out["fft"], out["axes"]
        diff = float((rf - ra).abs().max() / rf.abs().max())
        if ref_us is None:
            ref_us = tf * 64 ** 3 / n ** 3 if n != 64 else tf
        pp = lambda us: us / n ** 3 / (ref_us / 64 ** 3)
        print(f"{n}^3 x 2: fft {tf:7.2f} us/step ({pp(tf):.2f}x per point of 64^3 fft)   axes {ta:7.2f} us/step "
              f"({pp(ta):.2f}x)   max rel diff after 20 steps {diff:.2e}", flush=True)


if __name__ == "__main__":
    main()
