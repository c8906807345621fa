"""Summarise rocprofv3 --pmc CSVs of the persistent kernels: per-dispatch SQ counters of the largest
dispatches (the K-integral launches), normalised per wave-round. Diagnostic tool."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
out = {}
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    eng = os.path.basename(os.path.dirname(f))
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        if "k_stream" not in r["Kernel_Name"] and "k_dfs" not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    if not per:
        continue
    big = sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:2]
    avg = {k: sum(d[1].get(k, 0) for d in big) / len(big) for k in big[0][1]}
    avg["valu_busy_frac_per_simd_est"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
    out[eng] = {"kernel": names[big[0][0]][:60], "dispatches": [d[0] for d in big], "avg": avg}
print(json.dumps(out, indent=1))
