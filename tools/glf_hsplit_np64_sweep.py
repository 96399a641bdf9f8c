"""Hermitian Lindblad batches at N_p = 64 (N = 48, 64): the pair-block Hermitian split path (forced with
QD_GLF_HSPLIT_NP64=1) vs the persistent Hermitian kernel (QD_GLF_HSPLIT=0) vs the general split-K path
(hermitian=False), density-matrix steps/s by batch size (gate hsplit at N_p = 64 on this crossover)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import lindblad as olb  # noqa: E402  (input synthesis only)
from pyqed_amd import lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
for N in (48, 64):
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    for B in (16, 32, 64, 128, 192, 256):
        rho0 = torch.from_numpy(olb.random_pure_states(B, N)).to(dev)
        for mode, herm, env in (("hsplit", True, {"QD_GLF_HSPLIT_NP64": "1", "QD_GLF_HSPLIT": "1"}),
                                ("herm-persistent", True, {"QD_GLF_HSPLIT_NP64": "0", "QD_GLF_HSPLIT": "0"}),
                                ("general", False, {"QD_GLF_HSPLIT_NP64": "0", "QD_GLF_HSPLIT": "0"})):
            os.environ.update(env)
            rho = rho0.clone()
            lindblad_rk4(Ht, Ct, rho, 1e-3, 2, hermitian=herm)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lindblad_rk4(Ht, Ct, rho, 1e-3, 40, hermitian=herm)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"N": N, "B": B, "mode": mode,
                              "dm_steps_per_s": round(B * 40 / (e0.elapsed_time(e1) / 1e3), 1)}), flush=True)
