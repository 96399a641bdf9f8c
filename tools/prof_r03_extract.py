"""Extract the round-3 profile figures from a tools/profile_round.sh output directory (stats + pmc passes):
the persistent Lindblad dispatches (kernel trace), per-launch PMC bytes of the Hermitian Lindblad kernel and of the
batched DEOM stage kernels, and the top dispatches by bytes.  usage: python tools/prof_r03_extract.py gpurun_out/TAG OUTDIR"""
import csv
import json
import os
import statistics
import sys

src, out = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)
rows = list(csv.DictReader(open(f"{src}/stats/run_kernel_trace.csv")))
with open(f"{out}/lindblad_dispatches.txt", "w") as f:
    f.write(f"rocprofv3 --kernel-trace of bench.py --steps 50 --warmup 5 --no-cpu ({src}): persistent GLF dispatches\n")
    for r in rows:
        if "lindblad_rk4_kernel<128" in r["Kernel_Name"]:
            f.write(f"{r['Kernel_Name'][:80]}  grid {r['Grid_Size_X']}  LDS {r['LDS_Block_Size']}  "
                    f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:.3f} ms\n")
res = {}
for kind, unit in (("fetch", 2048), ("write", 1024)):
    agg, grid = {}, {}
    for r in csv.DictReader(open(f"{src}/{kind}/run_counter_collection.csv")):
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"][:110])
        agg[key] = agg.get(key, 0) + float(r["Counter_Value"]) * unit
        grid[key] = int(r["Grid_Size"])
    by = {}
    for (d, k), v in agg.items():
        by.setdefault(f"{k} grid {grid[(d, k)]}", []).append(v)
    res[kind] = {k: {"dispatches": len(v), "median_bytes": statistics.median(v), "max_bytes": max(v)}
                 for k, v in sorted(by.items(), key=lambda x: -max(x[1]))[:40]}
json.dump(res, open(f"{out}/pmc_bytes_by_kernel_grid.json", "w"), indent=1)
print(open(f"{out}/lindblad_dispatches.txt").read())
for kind in res:
    for k, v in list(res[kind].items())[:12]:
        print(kind, f"{v['median_bytes'] / 1e6:10.2f} MB median  {v['dispatches']:5d}  {k[:120]}")
