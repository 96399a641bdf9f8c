"""Turn a profiling round's PMC passes (tools/profile_round.sh output) into profiles/pmc_traffic.json
entries: calibrated HBM bytes per unit for one kernel.

    python tools/pmc_to_traffic.py <round dir> <kernel substring> <json key> <units> <unit text> [prefix]

The dispatch used is the one with the largest FETCH_SIZE among those whose name matches (the timed
launch of bench.py); <units> is what that launch processed (e.g. batch x steps density-matrix steps).
FETCH_SIZE / WRITE_SIZE are scaled by the bytes-per-unit the calibration kernels measured
(tools/pmc_calib: 256 MiB read / written)."""
import csv
import json
import os
import sys

d, sub, key, units, unit_text = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4]), sys.argv[5]
pre = sys.argv[6] if len(sys.argv) > 6 else ""  # "g" for the --general passes (gfetch / gwrite)


def rows(path):
    return list(csv.DictReader(open(path)))


def scale(kind, kname):
    vals = [float(r["Counter_Value"]) for r in rows(f"{d}/calib_{kind}/run_counter_collection.csv")
            if r["Kernel_Name"].startswith(kname)]
    return (256 << 20) / (sum(vals) / len(vals))


fscale = scale("fetch", "read_only")
wscale = scale("write", "write_only")
fetch = {r["Dispatch_Id"]: float(r["Counter_Value"]) for r in rows(f"{d}/{pre}fetch/run_counter_collection.csv")
         if sub in r["Kernel_Name"]}
write = {r["Dispatch_Id"]: float(r["Counter_Value"]) for r in rows(f"{d}/{pre}write/run_counter_collection.csv")
         if sub in r["Kernel_Name"]}
fid = max(fetch, key=fetch.get)
wid = max(write, key=write.get)
out = {
    "read_bytes_per_unit": round(fetch[fid] * fscale / units, 2),
    "write_bytes_per_unit": round(write[wid] * wscale / units, 2),
    "unit": unit_text,
    "source": f"{d}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, dispatch {fid}/{wid}; "
              f"{fscale:.0f} B per FETCH_SIZE unit, {wscale:.0f} B per WRITE_SIZE unit (tools/pmc_calib)",
}
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
table = json.load(open(path)) if os.path.exists(path) else {}
table[key] = out
json.dump(table, open(path, "w"), indent=1)
print(key, out)
