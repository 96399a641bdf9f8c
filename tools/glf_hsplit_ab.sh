# Lindblad N = 128 Hermitian batches of 16 / 64 / 128 matrices: pair-block split path (default) vs the persistent
# Hermitian kernel (QD_GLF_HSPLIT=0) vs the general split-K path (hermitian=False); event-timed, 2 rounds.
set -e
cat > /tmp/hs_bench.py <<'PY'
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.getcwd())
from bench import synthetic_lindblad, random_pure_states
from pyqed_amd import lindblad_rk4
dev = torch.device("cuda", 0)
H, cs = synthetic_lindblad(128)
Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
herm = None if os.environ.get("HS_GENERAL") is None else False
for B in (16, 64, 128):
    r = torch.from_numpy(random_pure_states(B, 128)).to(dev)
    lindblad_rk4(Ht, Ct, r, 1e-3, 2, hermitian=herm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); lindblad_rk4(Ht, Ct, r, 1e-3, 50, hermitian=herm); e1.record(); torch.cuda.synchronize()
    print(json.dumps({"B": B, "dm_steps_per_s": round(B * 50 / (e0.elapsed_time(e1) / 1e3), 1)}), flush=True)
PY
for rep in 1 2; do
  python /tmp/hs_bench.py | sed "s/^/hsplit /"
  QD_GLF_HSPLIT=0 python /tmp/hs_bench.py | sed "s/^/persistent /"
  HS_GENERAL=1 python /tmp/hs_bench.py | sed "s/^/general /"
done
