"""Band-count sweep of the persistent tier-banded DEOM launch (qd_deom_rk4_banded) against the stage launches.

usage: python tools/deom_band_sweep.py [steps] [band counts, comma separated (bench hierarchy only)]
One hierarchy, device-resident state, HIP events (bench._deom_event_rate): the bench hierarchy (K = 5, L = 12,
6188 ADOs) and the stretch hierarchy (K = 6, L = 12, 18,564 ADOs)."""
import os
import sys

import numpy as np
import sympy as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _deom_event_rate  # noqa: E402
from pyqed_amd.deom import Bath, DEOMSolver  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    only = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else None
    dev = torch.device("cuda:0")
    w = sp.symbols(r"\omega", real=True)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    cases = ((4, 0.002, (65, 96, 128, 160, 192, 224, 256)), (5, 0.001, (128, 192, 256)))
    if only:
        cases = ((4, 0.002, only),)
    for npsd, dt, counts in cases:
        bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [npsd], [0] * (npsd + 1))
        sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
        sol.check_()
        sol.init_()
        r = _deom_event_rate(dev, sol, bath, sz + sx, sx[None], 1, steps, dt=dt, banded=False)
        print(f"nmax {sol.nmax}: stage launches {r:.0f} steps/s ({1e6 / r:.2f} us/step)", flush=True)
        for nb in counts:
            sol.bands = nb
            bt = sol.band_tables(dev)
            if bt is None:
                print(f"  {nb} bands: not eligible", flush=True)
                continue
            r = _deom_event_rate(dev, sol, bath, sz + sx, sx[None], 1, steps, dt=dt)
            print(f"  {bt.nbands} bands (own <= {bt.max_own}, rows <= {bt.max_loc}): {r:.0f} steps/s "
                  f"({1e6 / r:.2f} us/step)", flush=True)
        sol.bands = None


if __name__ == "__main__":
    main()
