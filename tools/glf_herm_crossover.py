"""Hermitian Lindblad (N = 128, n_c = 1) near the split / persistent crossover: DM-steps/s of both paths
(QD_OPT_GLF_PATH) for B in argv (default 160..256).  One JSON line per B."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import random_pure_states, synthetic_lindblad  # noqa: E402
from pyqed_amd import _lib, lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
Bs = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "160,192,208,224,240,256".split(","))]
H, cs = synthetic_lindblad(128, nc=1)
Ht = torch.from_numpy(H).to(dev)
Ct = torch.from_numpy(np.array(cs)).to(dev)
for B in Bs:
    row = {"B": B}
    for path in ("split", "persistent"):
        _lib.set_option(_lib.QD_OPT_GLF_PATH, _lib.GLF_PATHS[path])
        rho = torch.from_numpy(random_pure_states(B, 128)).to(dev)
        lindblad_rk4(Ht, Ct, rho, 1e-3, 20, hermitian=True)
        torch.cuda.synchronize()
        steps = 40
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=True)
        e1.record()
        torch.cuda.synchronize()
        row[path] = round(B * steps / (e0.elapsed_time(e1) / 1e3), 1)
    print(json.dumps(row), flush=True)
_lib.set_option(_lib.QD_OPT_GLF_PATH, 0)
