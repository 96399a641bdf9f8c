"""Summarise a profiling round (tools/profile_round.sh output): kernel stats and PMC bytes."""
import csv
import sys
from collections import defaultdict

d = sys.argv[1]


def rows(path):
    try:
        return list(csv.DictReader(open(path)))
    except FileNotFoundError:
        return []


print("== kernel stats (avg us, calls, %)")
for r in rows(f"{d}/stats/run_kernel_stats.csv")[:14]:
    print(f"  {r['Name'][:70]:70s} {float(r['AverageNs'])/1e3:10.1f} {r['Calls']:>5} {float(r['Percentage']):6.2f}")
cal = {}
for kind in ("fetch", "write"):
    for r in rows(f"{d}/calib_{kind}/run_counter_collection.csv"):
        cal.setdefault(kind, defaultdict(list))[r["Kernel_Name"]].append(float(r["Counter_Value"]))
if cal:
    wr = cal["write"]["write_only(double __vector(2)*, unsigned long)"]
    rd = cal["fetch"]["read_only(double __vector(2) const*, unsigned long, double*)"]
    print(f"== calibration: 256 MiB written -> WRITE_SIZE {wr} ; 256 MiB read -> FETCH_SIZE {rd}")
    wscale = (256 << 20) / (sum(wr) / len(wr))
    fscale = (256 << 20) / (sum(rd) / len(rd))
    print(f"   bytes per WRITE_SIZE unit = {wscale:.1f}, bytes per FETCH_SIZE unit = {fscale:.1f}")
else:
    wscale = fscale = 1024.0
per = defaultdict(dict)
for kind, scale in (("fetch", fscale), ("write", wscale)):
    for r in rows(f"{d}/{kind}/run_counter_collection.csv"):
        key = (r["Kernel_Name"][:60], r["Dispatch_Id"])
        per[key][kind] = float(r["Counter_Value"]) * scale
print("== per-dispatch HBM bytes (calibrated), largest")
items = sorted(per.items(), key=lambda kv: -(kv[1].get("fetch", 0) + kv[1].get("write", 0)))
for (name, did), v in items[:12]:
    print(f"  {name:60s} #{did:>4} read {v.get('fetch', 0)/1e9:9.4f} GB  write {v.get('write', 0)/1e9:9.4f} GB")
