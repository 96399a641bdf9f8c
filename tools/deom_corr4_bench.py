"""DEOMSolver.correlation_4op_3t at the bench hierarchy (L = 12, K = 5, n = 24,752) through the Krylov form: wall clock
per call and the Krylov / Taylor work (sol.last_corr4) for a few grid sizes and waiting times.  One JSON line per
case."""
import json
import os
import sys
import time

import numpy as np
import sympy as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd.deom import Bath, DEOMSolver  # noqa: E402

dev = torch.device("cuda", 0)
w = sp.symbols(r"\omega", real=True)
bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
sx = np.array([[0, 1], [1, 0]], complex)
sz = np.diag([1.0, -1.0]).astype(complex)
L = int(sys.argv[1]) if len(sys.argv) > 1 else 12
sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, L)
rho0 = np.array([[1, 0], [0, 0]], complex)
sol.correlation_4op_3t(sz, sx, sx, sz, rho0, 0.5, np.linspace(-4.1, 4.3, 4), np.linspace(-3.7, 4.9, 4), lcr="lccc")
for nw, T in ((32, 0.5), (64, 0.5), (128, 0.5), (64, 0.0), (64, 2.0)):
    wx = np.linspace(-4.1, 4.3, nw)
    wy = np.linspace(-3.7, 4.9, nw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, T, wx, wy, lcr="lccc")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"L": L, "nw": nw, "T": T, "seconds": round(el, 3), "points_per_s": round(nw * nw / el, 1),
                      "finite": bool(np.all(np.isfinite(c))), **sol.last_corr4}), flush=True)
