"""A/B of the device Arnoldi orthogonalisation in DEOMSolver.correlation_4op_3t at the bench hierarchy (L = 12,
K = 5, n = 24,752, 'lccc', T = 0.5, 64 x 64 grid): four-pass CGS2 (qd_cgs_project + GEMV updates) against the
delayed CGS2 step (qd_arnoldi_dcgs2_step, two passes).  Wall clock per call (best of 3), Krylov dimensions, and
the relative difference of the two correlation grids.  AB_ONLY_DCGS2=1: the delayed form only (for profiles)."""
import json
import os
import sys
import time

import numpy as np
import sympy as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import deom_krylov as dk  # noqa: E402
from pyqed_amd.deom import Bath, DEOMSolver  # noqa: E402

w = sp.symbols(r"\omega", real=True)
bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
sx = np.array([[0, 1], [1, 0]], complex)
sz = np.diag([1.0, -1.0]).astype(complex)
sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
rho0 = np.array([[1, 0], [0, 0]], complex)
wx = np.linspace(-4.1, 4.3, 64)
wy = np.linspace(-3.7, 4.9, 64)
res = {}
flags = (True,) if os.environ.get("AB_ONLY_DCGS2") else (False, True, False, True)
for flag in flags:
    dk.ARNOLDI_DCGS2 = flag
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, 0.5, wx, wy, lcr="lccc")
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    res[flag] = c
    print(json.dumps({"dcgs2": flag, "seconds": round(best, 4), "points_per_s": round(64 * 64 / best, 1),
                      **{k: v for k, v in sol.last_corr4.items() if not isinstance(v, np.ndarray)}}, default=str),
          flush=True)
if False in res:
    d = np.abs(res[True] - res[False]).max() / np.abs(res[False]).max()
    print(json.dumps({"relerr_dcgs2_vs_cgs2": float(d)}), flush=True)
