"""Lindblad RK4 (N = 128 / 256, one Ginibre c_op) by batch size: persistent workgroup per matrix (Hermitian and
general kernels) vs the split path (a workgroup per BT x BT output block per phase, BT = 32 / 64 / 128).
Prints density-matrix steps/s per (N, B, mode)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import lindblad as olb  # noqa: E402  (input synthesis only)
from pyqed_amd import _lib, lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
Bs = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,4,16,32,64,128,256".split(","))]
for N in (128, 256):
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    for B in Bs:
        rho0 = torch.from_numpy(olb.random_pure_states(B, N)).to(dev)
        modes = [("herm-persistent", True, "persistent")] if N <= 128 else []
        modes += [("persistent", False, "persistent"), ("split", False, "split")]
        for mode, herm, path in modes:
            _lib.set_option(_lib.QD_OPT_GLF_PATH, _lib.GLF_PATHS[path])
            rho = rho0.clone()
            lindblad_rk4(Ht, Ct, rho, 1e-3, 2, hermitian=herm)
            torch.cuda.synchronize()
            steps = 20 if N == 128 else 5
            t0 = time.perf_counter()
            lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=herm)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(json.dumps({"N": N, "B": B, "mode": mode, "dm_steps_per_s": round(B * steps / el, 1),
                              "us_per_step": round(el / steps * 1e6, 1)}), flush=True)
