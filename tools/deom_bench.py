"""DEOM stage kernels timed by HIP events on device-resident state (no host transfers in the timed region): the
bench hierarchy (spin-boson, Drude, Pade npsd=4 -> K=5, L=12 -> 6188 ADOs, dt=0.002) at B hierarchies.
usage: python tools/deom_bench.py [B ...]   (env DEOM_LAYOUT = ado_major / element_major forces the layout)
One JSON line per B: RK4 steps/s, ADO-steps/s, and algorithmic HBM GB/s at 768 B per ADO-step."""
import json
import os
import sys

import numpy as np
import sympy as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd import _lib  # noqa: E402
from pyqed_amd.deom import Bath, DEOMSolver, ado_coefficients  # noqa: E402

dev = torch.device("cuda", 0)
w = sp.symbols(r"\omega", real=True)
bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
sx = np.array([[0, 1], [1, 0]], complex)
sz = np.diag([1.0, -1.0]).astype(complex)
sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
sol.check_()
sol.init_()
ns, K, nmax = 2, sol.nind, sol.nmax
coef, damp = ado_coefficients(sol.keys, np.asarray(bath.etal), np.asarray(bath.etar), np.asarray(bath.etaa),
                              np.asarray(bath.expn), sol.lmax)
c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
tabs = (i32(sol._minus), i32(sol._plus), c128(coef), c128(damp), i32(bath.mode))
H, Q = c128(sz + sx), c128(sx[None])
lib = _lib.load()
am_env = os.environ.get("DEOM_LAYOUT")
steps = int(os.environ.get("DEOM_STEPS", "100"))
for B in [int(a) for a in sys.argv[1:]] or [1, 64, 256]:
    ado_major = B >= 16 if am_env is None else am_env == "ado_major"
    fn = lib.qd_deom_rk4_ado_major if ado_major else lib.qd_deom_rk4
    shape = (nmax, B, ns, ns) if ado_major else (B, nmax, ns, ns)
    ados = torch.zeros(shape, dtype=torch.complex128, device=dev)
    (ados[0] if ado_major else ados[:, 0])[..., 0, 0] = 1
    rho_sys = torch.empty((B, steps + 1, ns, ns), dtype=torch.complex128, device=dev)

    def run(n):
        rc = fn(ados.data_ptr(), B, nmax, K, ns, *(t.data_ptr() for t in tabs), 1, H.data_ptr(), None, Q.data_ptr(),
                None, None, None, 0.002, n, rho_sys.data_ptr(), None, 0, None, _lib.stream_ptr(dev))
        _lib.check(rc, "qd_deom_rk4")

    run(5)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run(steps)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    sps = steps / ms * 1e3
    print(json.dumps({"B": B, "ado_major": ado_major, "path": _lib.take_path(),
                      "steps_per_s": round(sps, 1), "ado_steps_per_s": round(sps * nmax * B, 1),
                      "us_per_stage": round(ms * 1e3 / steps / 4, 2),
                      "algo_gbs": round(sps * nmax * B * 768 / 1e9, 1),
                      "trace_ok": bool(abs(torch.diagonal(rho_sys[:, -1], dim1=-2, dim2=-1).sum(-1) - 1).max() < 1e-10)}),
          flush=True)
