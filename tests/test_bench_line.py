"""bench.py's stdout contract, on CPU: the compact JSON line built from a recorded full-bench detail file
(profiles/r04/bench_r04f_detail.json, the driver's own command on one MI355X) carries every key the driver parses,
the headline's roofline and cpu_baseline, the 2DES half of BASELINE's metric, and stays short enough for the
driver's stdout tail."""
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_compact_line_keys_and_length():
    import bench
    out = json.load(open(os.path.join(ROOT, "profiles", "r04", "bench_r04f_detail.json")))
    line = bench.compact_line(out, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "twodes"):
        assert k in line, k
    assert line["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    tw = line["twodes"]
    assert tw["value"] > 0 and "roofline" in tw and "shard_1of8" in tw and "cpu_baseline" in tw
    assert line["higher_is_better"] is True and line["scaling"] == "weak"
    assert len(s) < 3500, len(s)
