"""SPO3 (qd_spo3_run) Strang steps/s at the examples/spo.py size (64^3 x 2) and 128^3 x 2, one wavefunction."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import _lib  # noqa: E402
from pyqed_amd.wpd import SPO3  # noqa: E402

dev = torch.device("cuda", 0)
for n in [int(v) for v in os.environ.get("SPO3_SIZES", "64,128").split(",")]:
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    sol = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)], [[[0, 1], 0.2 * X]])
    sol.build(0.05)
    psi0 = np.zeros((n, n, n, 2), complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2) / np.pi ** 0.75
    psi = torch.from_numpy(psi0).to(dev)
    eVh = torch.from_numpy(sol.exp_V_half).to(dev)
    eK = torch.from_numpy(sol.exp_K).to(dev)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    run = lambda k: _lib.check(lib.qd_spo3_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, n, 2, k, k, None,
                                               st), "qd_spo3_run")
    run(5)
    torch.cuda.synchronize()
    steps = 200
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    byts = (6 * n ** 3 * 2 + n ** 3 * 4 + n ** 3) * 16   # psi r+w in 3 passes, exp_V_half, exp_K
    print(json.dumps({"n": n, 
                      "steps_per_s": round(steps / el, 1), "us_per_step": round(el / steps * 1e6, 2),
                      "alg_GBs": round(byts * steps / el / 1e9, 1)}), flush=True)
