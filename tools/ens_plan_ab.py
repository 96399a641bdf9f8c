"""HEAD's 2DES split plan against another build's (e.g. var/libqdyn_wg256.so: the pre-cc35caa
256-workgroup plan for the 64-block GEMM) IN ONE PROCESS: both libraries loaded side by side (ctypes), the same pruned
operands, the full grid (65,536 members) and the 1/8 shard (8,192) timed in alternation, 12 rounds of 20 grids each,
HIP events on one stream after a 60 ms warm-up; medians per library.
usage: python tools/ens_plan_ab.py var/libqdyn_wg256.so"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pyqed_amd import _lib  # noqa: E402
from pyqed_amd.response import _prune_fixed_t2  # noqa: E402

dev = torch.device("cuda", 0)
other = ctypes.CDLL(sys.argv[1])
head = _lib.load()
for L in (other,):
    f = L.qd_response2d_ensemble_rect
    f.restype = ctypes.c_int
    f.argtypes = head.qd_response2d_ensemble_rect.argtypes
libs = {"head": head, "other": other}
out = torch.empty((256, 256), dtype=torch.complex128, device=dev)
st = _lib.stream_ptr(dev)
res = {}
for name, M in (("full", 65536), ("shard", 8192)):
    lam, alpha, Mt, beta = bench.twodes_inputs(M)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    swap, ax, lx, Mc, bz, lz = _prune_fixed_t2(to(lam), to(alpha), to(Mt), to(beta))
    nx, nz = ax.shape[1], bz.shape[1]

    def grid(lib):
        rc = lib.qd_response2d_ensemble_rect(ax.data_ptr(), lx.data_ptr(), nx, Mc.data_ptr(), bz.data_ptr(),
                                             lz.data_ptr(), nz, M, None, 0.0, 0.5, 256, None, 0.0, 0.5, 256,
                                             int(swap), out.data_ptr(), 0, st)
        assert rc == 0, rc

    bench.ramp_warmup(lambda: (grid(head), grid(other)), dev)
    ms = {k: [] for k in libs}
    sums = {}
    for _ in range(12):
        for k, lib in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                grid(lib)
            e1.record()
            torch.cuda.synchronize()
            ms[k].append(e0.elapsed_time(e1) / 20)
            sums[k] = complex(out.sum().item())
    for k in libs:
        res[f"{name}_{k}_ms_median"] = round(float(np.median(ms[k])), 4)
        res[f"{name}_{k}_ms_min"] = round(float(np.min(ms[k])), 4)
    res[f"{name}_checksums_equal"] = abs(sums["head"] - sums["other"]) <= 1e-9 * abs(sums["head"])
print(json.dumps(res), flush=True)
