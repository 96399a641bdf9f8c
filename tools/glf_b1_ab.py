"""Small-batch Lindblad split path A/B (general kernel, N = 128 unless given): one-tile-ahead vs whole-range
preloaded K tiles (QD_GLF_PRE) and split counts (QD_GLF_KS / QD_GLF_YS), event-timed on the launch stream,
variants alternated over several rounds.  Usage: glf_b1_ab.py "PRE,KS,YS;PRE,KS,YS;..." [B,...] [N]
(KS / YS = 0: the library's own choice).  Also checks every variant against the first one's result."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import lindblad as olb  # noqa: E402  (input synthesis only)
from pyqed_amd import lindblad_rk4  # noqa: E402

dev = torch.device("cuda", 0)
variants = [tuple(int(x) for x in v.split(",")) for v in sys.argv[1].split(";")]
Bs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 4]
N = int(sys.argv[3]) if len(sys.argv) > 3 else 128
H, cs = olb.synthetic_lindblad(N, nc=1)
Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
stream = torch.cuda.current_stream(dev)


def setenv(pre, ks, ys):
    os.environ["QD_GLF_PRE"] = str(pre)
    for k, v in (("QD_GLF_KS", ks), ("QD_GLF_YS", ys)):
        if v:
            os.environ[k] = str(v)
        else:
            os.environ.pop(k, None)


for B in Bs:
    rho0 = torch.from_numpy(olb.random_pure_states(B, N)).to(dev)
    ref = None
    res = {v: [] for v in variants}
    for rnd in range(3):
        for v in variants:
            setenv(*v)
            rho = rho0.clone()
            lindblad_rk4(Ht, Ct, rho, 1e-3, 2, hermitian=False)
            torch.cuda.synchronize()
            if rnd == 0:
                if ref is None:
                    ref = rho.clone()
                else:
                    err = float((rho - ref).abs().max() / ref.abs().max())
                    assert err < 1e-12, (v, err)
            steps = 200
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            lindblad_rk4(Ht, Ct, rho, 1e-3, steps, hermitian=False)
            e1.record(stream)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / steps)
    for v in variants:
        us = sorted(res[v])
        print(json.dumps({"N": N, "B": B, "pre": v[0], "ks": v[1], "ys": v[2], "us_per_step": [round(x, 2) for x in us],
                          "dm_steps_per_s_best": round(B * 1e6 / us[0], 1)}), flush=True)
