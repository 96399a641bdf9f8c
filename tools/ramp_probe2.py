import json, os, sys, time
import numpy as np, torch
sys.path.insert(0, '/root/repo')
import bench
from pyqed_amd.response import response2d_ensemble
dev = torch.device("cuda", 0)
lam, alpha, Mt, beta = bench.twodes_inputs(65536)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
lam_t, alpha_t, Mt_t, beta_t = to(lam), to(alpha), to(Mt), to(beta)
t = 0.5 * np.arange(256)
outs = [torch.empty((256, 256), dtype=torch.complex128, device=dev) for _ in range(2)]
def run(n, alt):
    ev=[torch.cuda.Event(enable_timing=True) for _ in range(n+1)]; host=[]
    ev[0].record()
    for k in range(n):
        h=time.perf_counter()
        response2d_ensemble(lam_t, alpha_t, Mt_t, beta_t, t, t, out=outs[k % 2 if alt else 0], accumulate=False)
        host.append(round((time.perf_counter()-h)*1e3,3))
        ev[k+1].record()
    torch.cuda.synchronize()
    return [round(ev[k].elapsed_time(ev[k+1]),3) for k in range(n)], host
run(3, False)
for alt in (False, True, False, True):
    bench.ramp_warmup(lambda: run(1, alt), dev)
    g,h=run(20, alt)
    print(json.dumps({"alt": alt, "grid_ms": g, "host_ms": h}), flush=True)
