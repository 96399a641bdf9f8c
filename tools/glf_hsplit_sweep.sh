# Hermitian pair-block split path vs the persistent Hermitian kernel across batch sizes (N = 128), 32- and 64-blocks
set -e
cat > /tmp/hs_sweep.py <<'PY'
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.getcwd())
from bench import synthetic_lindblad, random_pure_states
from pyqed_amd import lindblad_rk4
dev = torch.device("cuda", 0)
H, cs = synthetic_lindblad(128)
Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
for B in (64, 128, 160, 192, 224, 256):
    r = torch.from_numpy(random_pure_states(B, 128)).to(dev)
    lindblad_rk4(Ht, Ct, r, 1e-3, 2, hermitian=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); lindblad_rk4(Ht, Ct, r, 1e-3, 30, hermitian=True); e1.record(); torch.cuda.synchronize()
    print(json.dumps({"B": B, "dm_steps_per_s": round(B * 30 / (e0.elapsed_time(e1) / 1e3), 1)}), flush=True)
PY
QD_GLF_HSPLIT_MAX=100000 QD_GLF_HSPLIT_BT=32 python /tmp/hs_sweep.py | sed "s/^/hsplit32 /"
QD_GLF_HSPLIT_MAX=100000 QD_GLF_HSPLIT_BT=64 python /tmp/hs_sweep.py | sed "s/^/hsplit64 /"
QD_GLF_HSPLIT=0 python /tmp/hs_sweep.py | sed "s/^/persistent /"
