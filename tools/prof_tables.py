"""Per-kernel tables of a profiling round (tools/profile_r02b.sh output):
    python tools/prof_tables.py <round dir> <out dir>
writes <out>/kernel_durations_by_grid.csv (dispatch durations from the kernel trace, grouped by kernel and grid)
and <out>/pmc_bytes_by_kernel.json (FETCH_SIZE / WRITE_SIZE passes scaled by the calibration kernels' bytes per
unit: mean calibrated HBM bytes per dispatch, grouped the same way)."""
import csv
import json
import os
import re
import statistics
import sys
from collections import defaultdict

d, out = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)


def rows(path):
    return list(csv.DictReader(open(path)))


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):       # drop the argument list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return re.sub(r"\s+", " ", name[:cut]).strip()


def grid(r):
    g = [r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")]
    g = [x for x in g if x not in (None, "", "1")] or ["1"]
    return "x".join(g)


dur = defaultdict(list)
for r in rows(f"{d}/stats/run_kernel_trace.csv"):
    dur[(short(r["Kernel_Name"]), grid(r))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
with open(f"{out}/kernel_durations_by_grid.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "grid", "dispatches", "mean_us", "min_us", "max_us", "total_ms"])
    for (k, g), v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([k, g, len(v), round(statistics.mean(v), 2), round(min(v), 2), round(max(v), 2),
                    round(sum(v) / 1e3, 3)])


def scale(kind, prefix):
    vals = [float(r["Counter_Value"]) for r in rows(f"{d}/calib_{kind}/run_counter_collection.csv")
            if r["Kernel_Name"].startswith(prefix)]
    return (256 << 20) / statistics.mean(vals)


fs, ws = scale("fetch", "read_only"), scale("write", "write_only")
res = {}
for kind, sc in (("fetch", fs), ("write", ws)):
    per = defaultdict(list)
    for r in rows(f"{d}/{kind}/run_counter_collection.csv"):
        per[(short(r["Kernel_Name"]), grid(r))].append(float(r["Counter_Value"]) * sc)
    for (k, g), v in per.items():
        e = res.setdefault(f"{k} grid={g}", {"dispatches": len(v)})
        e[f"{'read' if kind == 'fetch' else 'write'}_bytes_mean"] = round(statistics.mean(v), 1)
        e[f"{'read' if kind == 'fetch' else 'write'}_bytes_max"] = round(max(v), 1)
json.dump({"bytes_per_fetch_unit": fs, "bytes_per_write_unit": ws,
           "kernels": dict(sorted(res.items(), key=lambda kv: -kv[1].get("read_bytes_mean", 0)))},
          open(f"{out}/pmc_bytes_by_kernel.json", "w"), indent=1)
print(f"{len(dur)} kernel/grid groups, {len(res)} PMC groups; bytes per unit fetch {fs:.0f} write {ws:.0f}")
