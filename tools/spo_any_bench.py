"""Strang steps/s of the split-operator passes on power-of-two vs other grids (device-resident state, HIP events):
SPO2 n x n x 2 (qd_spo2_run_ex), SPO3 n^3 x 2 (qd_spo3_run), SPO 1D (qd_spo1d_run).  Prints one JSON line per case
with the effective bytes rate of the pass structure (SPO2: 2 passes, psi in + out each, exp_V_half once, exp_K once)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
_lib.ensure_device(dev)
lib = _lib.load()
st = _lib.stream_ptr(dev)


def unit_ops(shape, ns, rng):
    a = rng.standard_normal(shape + (ns, ns)) + 1j * rng.standard_normal(shape + (ns, ns))
    h = (a + np.conj(np.swapaxes(a, -1, -2))) / 4
    w, u = np.linalg.eigh(h)
    return (u * np.exp(-0.5j * w)[..., None, :]) @ np.conj(np.swapaxes(u, -1, -2))


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def timed(fn, steps):
    fn(2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn(steps)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / steps


rng = np.random.default_rng(0)
mode = sys.argv[2] if len(sys.argv) > 2 else "all"   # "2d": SPO2 cases only; "3d": SPO3 cases only
cases2 = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "200,256,500,512,1000,1024".split(","))]
if mode == "3d":
    cases2 = []
for n in cases2:
    ns = 2
    U = t(unit_ops((n, n), ns, rng))
    K = t(np.exp(-1j * rng.uniform(0, 6, (n, n))))
    psi = t(rng.standard_normal((n, n, ns)) + 0j)

    def run(k):
        _lib.check(lib.qd_spo2_run_ex(psi.data_ptr(), U.data_ptr(), None, K.data_ptr(), None, n, n, ns, k, k, None,
                                      st), "qd_spo2_run_ex")

    sec = timed(run, 50)
    byts = 4 * n * n * ns * 16 + n * n * ns * ns * 16 + n * n * 16
    print(json.dumps({"case": f"spo2 {n}x{n}x2", "us_per_step": round(sec * 1e6, 2), "steps_per_s": round(1 / sec, 1),
                      "GBps": round(byts / sec / 1e9, 1)}), flush=True)
if len(sys.argv) > 2 and sys.argv[2] == "2d":
    sys.exit(0)
for n in (48, 60, 64, 96, 100, 128):
    ns = 2
    U = t(unit_ops((n, n, n), ns, rng))
    K = t(np.exp(-1j * rng.uniform(0, 6, (n, n, n))))
    psi = t(rng.standard_normal((n, n, n, ns)) + 0j)

    def run3(k):
        _lib.check(lib.qd_spo3_run(psi.data_ptr(), U.data_ptr(), K.data_ptr(), n, n, n, ns, k, k, None, st),
                   "qd_spo3_run")

    sec = timed(run3, 20)
    byts = 8 * n ** 3 * ns * 16 + n ** 3 * ns * ns * 16 + n ** 3 * 16
    print(json.dumps({"case": f"spo3 {n}^3x2", "us_per_step": round(sec * 1e6, 2), "steps_per_s": round(1 / sec, 1),
                      "GBps_4pass": round(byts / sec / 1e9, 1)}), flush=True)
for n in (() if mode == "3d" else (1000, 1024, 2048, 2053, 4096, 6000)):
    x = np.linspace(-8, 8, n)
    eV = t(np.exp(-1j * 0.01 * x ** 2 / 2))
    eVh = t(np.exp(-0.5j * 0.01 * x ** 2 / 2))
    eK = t(np.exp(-1j * rng.uniform(0, 6, n)))
    psi = t(rng.standard_normal((1, n)) + 0j)

    def run1(k):
        _lib.check(lib.qd_spo1d_run(psi.data_ptr(), eV.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, 1, k, 1, None, st),
                   "qd_spo1d_run")

    sec = timed(run1, 200)
    print(json.dumps({"case": f"spo1d {n}", "us_per_step": round(sec * 1e6, 2), "steps_per_s": round(1 / sec, 1)}),
          flush=True)
