"""Median HIP-event time per 2DES grid of the bench's fixed-t2 ensemble (65,536 members, 256 x 256) and of its 1/8
shard (8,192 members), 30 grids each after a 60 ms warm-up on the same work (per-grid events, then the mean of 30
grids under one event pair); for A/B runs of the library's
environment switches (one process per setting: several switches are read once per process).
usage: [ENV=...] python tools/ens_grid_time.py [label]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pyqed_amd.response import response2d_ensemble  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else ""
dev = torch.device("cuda", 0)
t = 0.5 * np.arange(256)
out = torch.empty((256, 256), dtype=torch.complex128, device=dev)
res = {"label": label}
for name, M in (("full", 65536), ("shard", 8192)):
    lam, alpha, Mt, beta = bench.twodes_inputs(M)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    args = [to(lam), to(alpha), to(Mt), to(beta)]

    def grid():
        response2d_ensemble(*args, t, t, out=out, accumulate=False)

    bench.ramp_warmup(grid, dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(31)]
    ev[0].record()
    for k in range(30):
        grid()
        ev[k + 1].record()
    torch.cuda.synchronize()
    ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(30)]
    res[name + "_ms_median"] = round(float(np.median(ms)), 4)
    # the same 30 grids with ONE event pair around them (no event packet between grids)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(30):
        grid()
    e1.record()
    torch.cuda.synchronize()
    res[name + "_ms_mean_no_grid_events"] = round(e0.elapsed_time(e1) / 30, 4)
    res[name + "_checksum"] = complex(out.sum().item()).__repr__()
print(json.dumps(res), flush=True)
