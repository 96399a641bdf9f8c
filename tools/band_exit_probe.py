"""Narrowing the `rocprofv3 --pmc` crash of the banded DEOM leg (profiles/r04/pmc_probe/):
the round-3 symptom reproduces as a SIGSEGV inside exit(), AFTER the bench printed its line and rocprofv3 wrote its
output and finalised.  This runs only the 8-band loopback run (ShardedDEOM) and then exits in one of several ways:

    python tools/band_exit_probe.py plain       return from main (normal exit)
    python tools/band_exit_probe.py shutdown    qd_shutdown() (trims libqdyn's stream-ordered memory pool) first
    python tools/band_exit_probe.py launches N  no DEOM: N tiny qd_gather_rows launches (dispatch-count probe)
    python tools/band_exit_probe.py persist     DEOMSolver.run only (the persistent banded kernel, qd_deom_rk4_banded)
    python tools/band_exit_probe.py both        DEOMSolver.run, then the 8-band loopback run
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
from pyqed_amd import _lib  # noqa: E402

if mode == "launches":
    n = int(sys.argv[2])
    src = torch.zeros((64, 4), dtype=torch.complex128, device=dev)
    dst = torch.zeros((8, 4), dtype=torch.complex128, device=dev)
    idx = torch.arange(8, dtype=torch.int32, device=dev)
    lib = _lib.load()
    for _ in range(n):
        _lib.check(lib.qd_gather_rows(src.data_ptr(), 64, idx.data_ptr(), 8, 4, dst.data_ptr(), 0,
                                      _lib.stream_ptr(dev)), "qd_gather_rows")
else:
    import sympy as sp
    from pyqed_amd.deom import Bath, DEOMSolver
    from pyqed_amd.deom_shard import ShardedDEOM
    w = sp.symbols(r"\omega", real=True)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
    r0 = np.zeros((2, 2), complex)
    r0[0, 0] = 1
    if mode in ("persist", "both"):
        _, rs = sol.run(r0.copy(), 0.002, 100)
        print("persistent banded: trace", float(np.trace(rs[-1]).real), "banded", sol.last_run_banded, flush=True)
    if mode != "persist":
        sh = ShardedDEOM(sol, nbands=8, loopback=True, device=dev, exchange="allgather")
        t, rs = sh.run(r0, 0.002, 40)
        print("loopback: trace", float(np.trace(rs[-1]).real), flush=True)
torch.cuda.synchronize(dev)
if mode == "shutdown":
    _lib.check(_lib.load().qd_shutdown(), "qd_shutdown")
print(f"{mode}: done", flush=True)
