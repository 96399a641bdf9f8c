"""bench.bench_2des called standalone twice (per-grid event times of its timed region), to separate the leg's own
behaviour from what the bench runs before it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for rep in range(2):
    r, _, _ = bench.bench_2des(dev, 1, 0, 65536, 20)
    print(json.dumps({"rep": rep, "ms_per_grid": r["ms_per_grid"], "grid_event_ms": r["grid_event_ms"],
                      "host_issue_ms": r["host_issue_ms"]}), flush=True)
