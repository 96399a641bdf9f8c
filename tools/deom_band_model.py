"""Per-band 8-GPU model (bench.deom_band_model) for compute-heavy hierarchies given on the command line as ns:L pairs,
e.g.  python tools/deom_band_model.py 96:8 128:8 160:8.  One JSON line per hierarchy (world 1; loopback run + model)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
steps = int(os.environ.get("BAND_STEPS", "10"))
for arg in sys.argv[1:]:
    ns, L = (int(x) for x in arg.split(":"))
    out = bench.bench_deom_banded(dev, 1, 0, steps=steps, cases=[bench._band_case(ns, L)])
    for name, ent in out.items():
        m = ent["model_8gpu"]
        print(json.dumps({"case": name, "nmax": ent["nmax"], "state_MB": round(ent["state_bytes"] / 2 ** 20, 1),
                          "one_gpu_ms_per_step": m["one_gpu_unbanded_ms_per_step"],
                          "max_band_stage_us": m["max_band_stage_us"],
                          "largest_peer_transfer_MB": round(m["largest_peer_transfer_bytes"] / 2 ** 20, 2),
                          "speedup_p2p_nolat": m["p2p_nolat"]["speedup"], "speedup_p2p_lat": m["p2p_lat"]["speedup"],
                          "speedup_allgather_lat": m["allgather_lat"]["speedup"]}), flush=True)
