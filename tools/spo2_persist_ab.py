"""A/B of the single-wavefunction SPO2 run at 256 x 256 x 2 (bench config d2): the persistent launch
(spo2_persist_kernel) against the two-kernel loop (QD_SPO_PERSIST=0), alternating, HIP events around qd_spo2_run of
`steps` Strang steps after a >= 60 ms warm-up on the same work.  Prints one JSON line per (mode, round).
usage: python tools/spo2_persist_ab.py [steps] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pyqed_amd import _lib  # noqa: E402
from pyqed_amd.wpd import SPO2  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
n, dt = 256, 0.05
x = np.linspace(-6, 6, n)
X, Y = np.meshgrid(x, x, indexing="ij")
sol = SPO2(x, x, mass=[1.0, 1.0], nstates=2)
sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
sol.build(dt)
psi0 = np.zeros((n, n, 2), complex)
psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
psi = torch.from_numpy(psi0).to(dev)
eVh = torch.from_numpy(sol.exp_V_half).to(dev)
eK = torch.from_numpy(sol.exp_K).to(dev)
lib = _lib.load()
st = _lib.stream_ptr(dev)
stream = torch.cuda.current_stream(dev)
bytes_per_step = (4 * n * n * 2 + n * n * 4 + n * n) * 16


def run(k):
    _lib.check(lib.qd_spo2_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, 2, k, k, None, st), "qd_spo2_run")


for rnd in range(rounds):
    for mode in ("persist", "two_kernel"):
        if mode == "two_kernel":
            os.environ["QD_SPO_PERSIST"] = "0"
        else:
            os.environ.pop("QD_SPO_PERSIST", None)
        bench.ramp_warmup(lambda: run(10), dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(steps)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) * 1e3 / steps
        print(json.dumps({"mode": mode, "round": rnd, "steps": steps, "us_per_step": round(us, 3),
                          "steps_per_s": round(1e6 / us, 1),
                          "hbm_frac": round(bytes_per_step / (us * 1e-6) / 1e9 / bench.HBM_PEAK_GBS, 4)}), flush=True)
