"""Per-launch fixed cost of the headline Lindblad launch (N = 128, n_c = 1, B = 256, Hermitian kernel): HIP-event
time of one lindblad_rk4 call of n steps, (a) after the GPU sat idle for `idle` ms, (b) queued right behind another
launch (no idle gap: the events then time the call alone on a busy GPU).  A fixed cost that appears only after idle
time is the clock ramp; one that appears in both is inside the call.
usage: python tools/lindblad_launch_overhead.py"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pyqed_amd import lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
N, B = 128, 256
H, cs = bench.synthetic_lindblad(N, nc=1)
Ht = torch.from_numpy(H).to(dev)
Ct = torch.from_numpy(np.array(cs)).to(dev)
rho = torch.from_numpy(bench.random_pure_states(B, N, seed=2)).to(dev)
lindblad_rk4(Ht, Ct, rho, 1e-3, 5, hermitian=True)
torch.cuda.synchronize()


def timed(n, idle_ms, busy_before):
    torch.cuda.synchronize()
    time.sleep(idle_ms / 1e3)
    if busy_before:
        lindblad_rk4(Ht, Ct, rho, 1e-3, 10, hermitian=True)   # queued work ahead of the timed call
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lindblad_rk4(Ht, Ct, rho, 1e-3, n, hermitian=True)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


for busy in (False, True):
    for idle in (0, 20, 200):
        for n in (1, 5, 20, 100):
            ms = min(timed(n, idle, busy) for _ in range(3))
            print(json.dumps({"busy_before": busy, "idle_ms": idle, "steps": n, "ms": round(ms, 3),
                              "ms_per_step": round(ms / n, 4)}), flush=True)
