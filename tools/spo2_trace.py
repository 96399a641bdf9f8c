"""SPO2 256 x 256 x 2 single wavepacket (BASELINE configs[2]): diagnosis of the ~10 us Strang step.
  run:      python tools/spo2_trace.py run [steps]          -- warm-up, then `steps` steps in one qd_spo2_run call
  analyse:  python tools/spo2_trace.py analyse <kernel_trace.csv>
Under `rocprofv3 --kernel-trace --output-format csv`, `analyse` prints each kernel's median duration and the median gap
from one kernel's end to the next kernel's start (the dependent-launch gap) over the timed call's kernels."""
import csv
import os
import sys

import numpy as np


def run(steps):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pyqed_amd import _lib
    from pyqed_amd.wpd import SPO2
    dev = torch.device("cuda", 0)
    n, dt = 256, 0.05
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
    sol.build(dt)
    psi0 = np.zeros((n, n, 2), complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    psi = torch.from_numpy(psi0).to(dev)
    eVh = torch.from_numpy(sol.exp_V_half).to(dev)
    eK = torch.from_numpy(sol.exp_K).to(dev)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    for k in (20, 2000, steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(lib.qd_spo2_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, 2, k, k, None, st), "spo2")
        e1.record()
        torch.cuda.synchronize()
    print(f"{steps} steps: {e0.elapsed_time(e1) / steps * 1e3:.3f} us per step", flush=True)


def analyse(path, last=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if last:
        rows = rows[-last:]
    import re
    names = [re.sub(r"^.*::", "", r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0])
             for r in rows]
    t0 = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
    t1 = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
    for nm in sorted(set(names)):
        sel = [i for i, x in enumerate(names) if x == nm]
        print(f"{nm}: n={len(sel)} median_us={np.median((t1 - t0)[sel]) / 1e3:.3f}")
    gaps = (t0[1:] - t1[:-1]) / 1e3
    print(f"gap end->next start: median_us={np.median(gaps):.3f} p10={np.percentile(gaps, 10):.3f} "
          f"p90={np.percentile(gaps, 90):.3f}")
    per = (t1[-1] - t0[0]) / 1e3 / (len(rows) / 2)
    print(f"span per (row + col) pair: {per:.3f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 500)
    else:
        analyse(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
