"""Counter target: the Lindblad B = 64 Hermitian split path (Y launch + pair launch, glf_split_pairs) for a few steps,
for rocprofv3 --pmc passes (tools: profiles/r05/lindblad/pair_pmc.txt)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import random_pure_states, synthetic_lindblad  # noqa: E402
from pyqed_amd import lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
H, cs = synthetic_lindblad(128, nc=1)
Ht = torch.from_numpy(H).to(dev)
Ct = torch.from_numpy(np.array(cs)).to(dev)
rho = torch.from_numpy(random_pure_states(64, 128)).to(dev)
lindblad_rk4(Ht, Ct, rho, 1e-3, 10)
torch.cuda.synchronize()
