"""Stream launches vs a captured HIP graph (torch.cuda.CUDAGraph around the C-ABI call) for the launch-latency-bound
single-object paths: SPO2 256 x 256 x 2 (2 launches per Strang step) and DEOM L = 12, K = 5 (4 launches per RK4
step).  The library's workspaces are warm before capture (no allocation inside the captured region)."""
import json
import os
import sys

import numpy as np
import sympy as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()


def time_both(run, steps, label):
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        run(steps)                      # warm workspaces on this stream
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(steps)
        e1.record()
        torch.cuda.synchronize()
        t_stream = e0.elapsed_time(e1)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        run(steps)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    t_graph = e0.elapsed_time(e1) / 3
    print(json.dumps({"case": label, "steps": steps, "stream_us_per_step": round(t_stream / steps * 1e3, 3),
                      "graph_us_per_step": round(t_graph / steps * 1e3, 3)}), flush=True)


# SPO2 256 x 256 x 2
from pyqed_amd.wpd import SPO2  # noqa: E402
n = 256
x = np.linspace(-6, 6, n)
X, Y = np.meshgrid(x, x, indexing="ij")
sol = SPO2(x, x, mass=[1.0, 1.0], nstates=2)
sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
sol.build(0.05)
psi = torch.zeros((n, n, 2), dtype=torch.complex128, device=dev)
psi[:, :, 0] = torch.from_numpy(np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2) / np.sqrt(np.pi)).to(dev)
eVh = torch.from_numpy(sol.exp_V_half).to(dev)
eK = torch.from_numpy(sol.exp_K).to(dev)


def spo_run(k):
    _lib.check(lib.qd_spo2_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, 2, k, k, None,
                               torch.cuda.current_stream(dev).cuda_stream), "qd_spo2_run")


time_both(spo_run, 200, "spo2_256x256x2")

# DEOM 6188 ADOs
from pyqed_amd.deom import Bath, DEOMSolver, ado_coefficients  # noqa: E402
w = sp.symbols(r"\omega", real=True)
bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
sx = np.array([[0, 1], [1, 0]], complex)
sz = np.diag([1.0, -1.0]).astype(complex)
ds = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
ds.check_()
ds.init_()
coef, damp = ado_coefficients(ds.keys, np.asarray(bath.etal), np.asarray(bath.etar), np.asarray(bath.etaa),
                              np.asarray(bath.expn), ds.lmax)
c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
tabs = (i32(ds._minus), i32(ds._plus), c128(coef), c128(damp), i32(bath.mode))
H, Q = c128(sz + sx), c128(sx[None])
ados = torch.zeros((1, ds.nmax, 2, 2), dtype=torch.complex128, device=dev)
ados[0, 0, 0, 0] = 1
steps = 100
rho_sys = torch.empty((1, steps + 1, 2, 2), dtype=torch.complex128, device=dev)


def deom_run(k):
    _lib.check(lib.qd_deom_rk4(ados.data_ptr(), 1, ds.nmax, ds.nind, 2, *(t.data_ptr() for t in tabs), 1,
                               H.data_ptr(), None, Q.data_ptr(), None, None, None, 0.002, k, rho_sys.data_ptr(),
                               None, 0, None, torch.cuda.current_stream(dev).cuda_stream), "qd_deom_rk4")


time_both(deom_run, steps, "deom_6188")
