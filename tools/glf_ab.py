"""A/B helper: Lindblad RK4 rates (DM-steps/s, HIP events) of the default path at a few (N, B, hermitian) shapes,
with the dispatch path taken (qd_take_path).  Run once per library (QDYN_LIB) on the same box."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import random_pure_states, synthetic_lindblad  # noqa: E402
from pyqed_amd import _lib, lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cases = [(128, 64, None), (128, 128, None), (128, 16, False), (128, 64, False), (128, 4, False), (32, 256, None),
         (64, 64, None), (128, 256, None)]
for N, B, herm in cases:
    H, cs = synthetic_lindblad(N, nc=1)
    Ht = torch.from_numpy(H).to(dev)
    Ct = torch.from_numpy(np.array(cs)).to(dev)
    rho = torch.from_numpy(random_pure_states(B, N)).to(dev)
    lindblad_rk4(Ht, Ct, rho, 1e-3, 40, hermitian=herm)   # warm-up / clocks
    torch.cuda.synchronize()
    _lib.take_path()
    steps = max(20, 6000 // B)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=herm)
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / 1e3
    print(json.dumps({"N": N, "B": B, "herm": herm, "dm_steps_per_s": round(B * steps / sec, 1),
                      "path": _lib.take_path()}), flush=True)
