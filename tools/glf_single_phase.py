"""Phase clocks of the single-trajectory launches (QD_PHASE_TIMING build): N = 128, one matrix, nc = 1, the Hermitian
launch and the general one, 500 steps after a 300-step warm-up.
usage: QDYN_LIB=pyqed_amd/libqdyn_timing.so python tools/glf_single_phase.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import random_pure_states, synthetic_lindblad  # noqa: E402
from pyqed_amd import lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
H, cs = synthetic_lindblad(128, nc=1)
Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
for herm in (True, False):
    rho = torch.from_numpy(random_pure_states(1, 128)).to(dev)
    lindblad_rk4(Ht, Ct, rho, 1e-3, 300, hermitian=herm)
    torch.cuda.synchronize()
    print(f"--- herm={herm}", file=sys.stderr, flush=True)
    lindblad_rk4(Ht, Ct, rho, 1e-3, 500, hermitian=herm)
    torch.cuda.synchronize()
