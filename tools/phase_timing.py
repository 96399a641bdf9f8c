"""Per-phase clock breakdown of the persistent Lindblad kernel (QD_PHASE_TIMING diagnostics).
Run on the GPU box:  make -C pyqed_amd/csrc timing && QDYN_LIB=pyqed_amd/libqdyn_timing.so python tools/phase_timing.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import lindblad as olb  # noqa: E402  (input synthesis only)
from pyqed_amd import lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
for N, B in ((128, 256), (64, 256), (32, 256)):
    H, cs = olb.synthetic_lindblad(N)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    for herm in (True, False):
        rho = torch.from_numpy(olb.random_pure_states(B, N)).to(dev)
        lindblad_rk4(Ht, Ct, rho, 1e-3, 2, hermitian=herm)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lindblad_rk4(Ht, Ct, rho, 1e-3, 20, hermitian=herm)
        torch.cuda.synchronize()
        print(f"N={N} B={B} herm={herm}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us/step wall", flush=True)
