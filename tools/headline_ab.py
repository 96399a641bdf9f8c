"""Headline Lindblad batch (N = 128, n_c = 1, 256 Hermitian density matrices, one 20-step launch per timed region):
DM-steps/s as the median of 5 regions, for comparing library builds (QDYN_LIB=... python tools/headline_ab.py)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import lindblad as olb  # noqa: E402
from pyqed_amd import lindblad_rk4  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N, B, steps = 128, 256, 20
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    rho = torch.from_numpy(olb.random_pure_states(B, N, seed=1)).to(dev)
    for _ in range(3):
        lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=True)
    torch.cuda.synchronize()
    rates = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=True)
        e1.record()
        torch.cuda.synchronize()
        rates.append(B * steps / (e0.elapsed_time(e1) / 1e3))
    print(f"median {np.median(rates):.0f} DM-steps/s  (min {min(rates):.0f}, max {max(rates):.0f})", flush=True)


if __name__ == "__main__":
    main()
