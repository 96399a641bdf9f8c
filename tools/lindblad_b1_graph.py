"""One Lindblad trajectory (N = 128, n_c = 1, the split-K path: ~48 launches per RK4 step): host wall-clock of the
launch loop vs HIP-event time of the stream launches vs a captured HIP graph replay (torch.cuda.CUDAGraph around
the C-ABI call, workspaces warm before capture).  Tells whether the one-matrix path is bound by host launch
issue or by the GPU-side kernel boundaries."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import lindblad as olb  # noqa: E402  (seeded synthetic inputs only)
from pyqed_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
N = int(os.environ.get("LB_N", "128"))
H, cs = olb.synthetic_lindblad(N)
Ht = torch.from_numpy(H).to(dev)
Ct = torch.from_numpy(np.array(cs)).to(dev)
rho = torch.from_numpy(olb.random_pure_states(1, N)).to(dev)
s = torch.cuda.Stream(dev)


def run(k):
    rc = lib.qd_lindblad_rk4(Ht.data_ptr(), Ct.data_ptr(), 1, rho.data_ptr(), 1, N, 1e-3, k, None, 0, None, None, 0,
                             s.cuda_stream)
    _lib.check(rc, "qd_lindblad_rk4")


steps = 200
with torch.cuda.stream(s):
    run(steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    run(steps)
    t_host = time.perf_counter() - t0
    e1.record(s)
    torch.cuda.synchronize()
    t_stream = e0.elapsed_time(e1)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    run(steps)
g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s):
    e0.record(s)
    for _ in range(3):
        g.replay()
    e1.record(s)
torch.cuda.synchronize()
t_graph = e0.elapsed_time(e1) / 3
print(json.dumps({"N": N, "steps": steps, "host_issue_us_per_step": round(t_host / steps * 1e6, 2),
                  "stream_us_per_step": round(t_stream / steps * 1e3, 2),
                  "graph_us_per_step": round(t_graph / steps * 1e3, 2)}), flush=True)
