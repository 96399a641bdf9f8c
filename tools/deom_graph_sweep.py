"""DEOM one hierarchy (6188 ADOs): device time of a first call (graph capture inside) and a repeated call (cached
exec) for graph chunk sizes (QD_DEOM_GRAPH_STEPS, set by the caller) vs direct launches (QD_GRAPHS=0)."""
import json
import os
import sys
import time

import numpy as np
import sympy as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import _lib  # noqa: E402
from pyqed_amd.deom import Bath, DEOMSolver, ado_coefficients  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
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
for steps in (200, 1000):
    rho_sys = torch.empty((1, steps + 1, 2, 2), dtype=torch.complex128, device=dev)

    def run(k):
        _lib.check(lib.qd_deom_rk4(ados.data_ptr(), 1, ds.nmax, ds.nind, 2, *(t.data_ptr() for t in tabs), 1,
                                   H.data_ptr(), None, Q.data_ptr(), None, None, None, 0.002, k, rho_sys.data_ptr(),
                                   None, 0, None, torch.cuda.current_stream(dev).cuda_stream), "qd_deom_rk4")

    run(5)
    res = []
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(steps)
        e1.record()
        torch.cuda.synchronize()
        res.append((round(e0.elapsed_time(e1) / steps * 1e3, 3), round((time.perf_counter() - t0) / steps * 1e6, 3)))
    print(json.dumps({"steps": steps, "graphs": os.environ.get("QD_GRAPHS", "1"),
                      "chunk": os.environ.get("QD_DEOM_GRAPH_STEPS", "16"),
                      "first_call_us_per_step_event_wall": res[0], "repeat_us_per_step_event_wall": res[1]}),
          flush=True)
