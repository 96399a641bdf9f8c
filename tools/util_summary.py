"""Per-kernel utilisation from a rocprofv3 --pmc pass (tools/util_pmc.sh): MFMA busy cycles over 4 x CU-busy cycles
(how fed the matrix pipe is while a CU works), CU-busy cycles per CU and dispatch (compare with the kernel's duration
x clock from a --kernel-trace run: the ratio is the fraction of its wall time the chip is busy), and the SQ wave-cycle
split (parked at s_waitcnt / barriers, issue-stalled, issuing)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)", "anon"))[-72:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CU_CYCLES", 0)):
    n = max(cnt[(k, c)] for c in v)
    if v.get("SQ_BUSY_CU_CYCLES", 0) / n < 1e5:
        continue
    wc = max(1.0, v.get("SQ_WAVE_CYCLES", 0))
    print("%-72s n=%5d mfma/cu4=%.3f cu_busy_per_cu=%8.0f wait_any=%.2f wait_inst=%.2f active=%.2f"
          % (k, n, v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, 4 * v["SQ_BUSY_CU_CYCLES"]),
             v["SQ_BUSY_CU_CYCLES"] / n / 256, v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc,
             v.get("SQ_ACTIVE_INST_ANY", 0) / wc))
