"""Hermitian single-trajectory launch (glf_single_herm_kernel) against the general single launch (hermitian=False) at
N = 128, B = 1 / 2, nc = 1 / 2: HIP-event rates on device-resident state after a 60 ms warm-up.  One JSON line per
case."""
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
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
for N, B, nc in [(128, 1, 1), (128, 2, 1), (128, 1, 2)]:
    H, cs = synthetic_lindblad(N, nc=nc)
    Ht = torch.from_numpy(H).to(dev)
    Ct = torch.from_numpy(np.array(cs)).to(dev)
    row = {"N": N, "B": B, "nc": nc}
    for herm in (True, False):
        rho = torch.from_numpy(random_pure_states(B, N)).to(dev)
        lindblad_rk4(Ht, Ct, rho, 1e-3, 300, hermitian=herm)   # warm-up (clocks)
        torch.cuda.synchronize()
        _lib.take_path()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=herm)
        e1.record()
        torch.cuda.synchronize()
        sec = e0.elapsed_time(e1) / 1e3
        r = rho.cpu().numpy()
        row["herm" if herm else "general"] = {
            "us_per_step": round(sec / steps * 1e6, 2), "dm_steps_per_s": round(B * steps / sec, 1),
            "path": _lib.take_path(), "hermitian_exact": bool(np.array_equal(r, np.conj(np.swapaxes(r, 1, 2))))}
    print(json.dumps(row), flush=True)
