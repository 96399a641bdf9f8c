"""TDSE RK4 (qd_tdse_rk4) steps/s by N and batch: persistent workgroup per wavefunction vs the row-parallel path
(QD_TDSE_ROWS=0 / 1).  One JSON line per (N, B, path)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyqed_amd.mol import tdse_rk4  # noqa: E402

dev = torch.device("cuda", 0)
for N in (64, 256, 1024, 2048, 4096):
    rng = np.random.default_rng(N)
    A = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = torch.from_numpy((A + A.conj().T) / 2 / np.sqrt(N)).to(dev)
    for B in (1, 64, 256):
        for rows in ("0", "1"):
            if N > 2048 and rows == "0":
                continue
            os.environ["QD_TDSE_ROWS"] = rows
            psi = torch.randn(B, N, dtype=torch.complex128, device=dev)
            psi /= psi.abs().pow(2).sum(1, keepdim=True).sqrt()
            steps = 20 if (rows == "0" and N >= 1024) else 200
            tdse_rk4(H, psi, 1e-3, 2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tdse_rk4(H, psi, 1e-3, steps)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(json.dumps({"N": N, "B": B, "path": "rows" if rows == "1" else "persistent",
                              "steps_per_s": round(steps / el, 1),
                              "hbm_gbs_H": round(4 * N * N * 16 * steps / el / 1e9, 1)}), flush=True)
