"""Few-trajectory Lindblad rates (device-resident state, HIP events): the one-launch single-trajectory kernel
(glf_single.hip, default) against the split path and the persistent batch kernel (QD_OPT_GLF_PATH), N = 128 / 64 / 32,
B = 1 .. the 256-workgroup cap.  Prints one JSON line per case."""
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
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cases = [(128, 1), (128, 2), (128, 4), (64, 1), (64, 16), (32, 1), (32, 4), (32, 16), (32, 32), (32, 64)]
for N, B in cases:
    H, cs = synthetic_lindblad(N, nc=1)
    Ht = torch.from_numpy(H).to(dev)
    Ct = torch.from_numpy(np.array(cs)).to(dev)
    row = {"N": N, "B": B}
    for mode in ("single", "split", "persistent"):
        if mode == "split" and N < 64:
            continue   # the general split path needs N_p >= 64
        _lib.set_option(_lib.QD_OPT_GLF_PATH, _lib.GLF_PATHS[mode])
        rho = torch.from_numpy(random_pure_states(B, N)).to(dev)
        lindblad_rk4(Ht, Ct, rho, 1e-3, 3, hermitian=False)
        torch.cuda.synchronize()
        _lib.take_path()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=False)
        e1.record()
        torch.cuda.synchronize()
        sec = e0.elapsed_time(e1) / 1e3
        row[mode] = {"us_per_step": round(sec / steps * 1e6, 2), "dm_steps_per_s": round(B * steps / sec, 1),
                     "path": _lib.take_path()}
    print(json.dumps(row), flush=True)
_lib.set_option(_lib.QD_OPT_GLF_PATH, 0)
