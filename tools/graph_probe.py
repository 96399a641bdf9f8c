"""Does a HIP graph shorten the per-kernel gaps of a launch-bound sequence?  SPO2 256 x 256 x 2 (qd_spo2_run_ex, two
kernels per Strang step): the same call issued directly and replayed from a captured graph (torch.cuda.CUDAGraph),
HIP events around K steps."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
lib = _lib.load()
n, ns, K = 256, 2, 200
rng = np.random.default_rng(0)
a = rng.standard_normal((n, n, ns, ns)) + 1j * rng.standard_normal((n, n, ns, ns))
h = (a + np.conj(np.swapaxes(a, -1, -2))) / 4
w, u = np.linalg.eigh(h)
U = torch.from_numpy((u * np.exp(-0.5j * w)[..., None, :]) @ np.conj(np.swapaxes(u, -1, -2))).to(dev)
Kx = torch.from_numpy(np.exp(-1j * rng.uniform(0, 6, (n, n)))).to(dev)
psi = torch.from_numpy(rng.standard_normal((n, n, ns)) + 0j).to(dev)
s = torch.cuda.Stream(dev)


def run(k, st):
    _lib.check(lib.qd_spo2_run_ex(psi.data_ptr(), U.data_ptr(), None, Kx.data_ptr(), None, n, n, ns, k, k, None, st),
               "qd_spo2_run_ex")


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        fn()
        e0.record(s)
        fn()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


with torch.cuda.stream(s):
    run(2, s.cuda_stream)
torch.cuda.synchronize()
direct = timed(lambda: run(K, s.cuda_stream))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    run(K, s.cuda_stream)
graph = timed(lambda: g.replay())
print(json.dumps({"case": "spo2 256x256x2", "steps": K, "us_per_step_direct": round(direct, 3),
                  "us_per_step_graph": round(graph, 3)}), flush=True)
