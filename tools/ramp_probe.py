"""Clock ramp of a long MFMA-bound launch sequence: per-grid HIP-event times of the bench's fixed-t2 2DES grid
(65,536 members, 256 x 256) over 60 back-to-back grids from an idle GPU, then after 200 ms idle with bench.ramp_warmup
(synchronising every ~5 ms) ahead of 20 grids.  Prints one JSON line per phase.
usage: python tools/ramp_probe.py"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pyqed_amd.response import response2d_ensemble  # noqa: E402

dev = torch.device("cuda", 0)
if os.environ.get("RAMP_PRE_LINDBLAD") == "1":   # the bench's Lindblad legs first (their workspaces come and go)
    from pyqed_amd import lindblad_rk4
    H, cs = bench.synthetic_lindblad(128, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    rho = torch.from_numpy(bench.random_pure_states(256, 128, seed=2)).to(dev)
    for Bs in (1, 64):
        lindblad_rk4(Ht, Ct, rho[:Bs].clone(), 1e-3, 300)
    lindblad_rk4(Ht, Ct, rho, 1e-3, 25, hermitian=True)
    torch.cuda.synchronize()
    del rho
lam, alpha, Mt, beta = bench.twodes_inputs(65536)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
lam_t, alpha_t, Mt_t, beta_t = to(lam), to(alpha), to(Mt), to(beta)
t = 0.5 * np.arange(256)
out = torch.empty((256, 256), dtype=torch.complex128, device=dev)


def grid():
    response2d_ensemble(lam_t, alpha_t, Mt_t, beta_t, t, t, out=out, accumulate=False)


grid()
torch.cuda.synchronize()


def timeline(n):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record()
    for k in range(n):
        grid()
        ev[k + 1].record()
    torch.cuda.synchronize()
    return [round(ev[k].elapsed_time(ev[k + 1]), 4) for k in range(n)]


time.sleep(0.3)
print(json.dumps({"phase": "60 grids from idle", "ms_per_grid": timeline(60)}), flush=True)
time.sleep(0.2)
t0 = time.perf_counter()
bench.ramp_warmup(grid, dev)
wm = (time.perf_counter() - t0) * 1e3
print(json.dumps({"phase": f"20 grids after ramp_warmup ({wm:.0f} ms)", "ms_per_grid": timeline(20)}), flush=True)
time.sleep(0.2)
t0 = time.perf_counter()
bench.ramp_warmup(grid, dev, min_ms=200.0)
wm = (time.perf_counter() - t0) * 1e3
print(json.dumps({"phase": f"20 grids after ramp_warmup ({wm:.0f} ms)", "ms_per_grid": timeline(20)}), flush=True)
