"""Per-shape means of the counters tools/pmc_icache.sh collected: the k_stream dispatches of
tools/try_single.py in order (6 shapes x (1 + reps) launches). Diagnostic tool."""
import collections
import csv
import glob
import json
import os
import sys

root, reps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5
shapes = ["one_task", "eps1e-3", "eps1e-6", "eps1e-8", "eps1e-10", "eps1e-12"]
out = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "k_stream" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    for s, name in enumerate(shapes):
        block = ids[s * (reps + 1) + 1:(s + 1) * (reps + 1)]   # skip each shape's warm-up launch
        for c in per[ids[0]] if ids else []:
            vals = [per[i][c] for i in block if c in per[i]]
            if vals:
                out[name][c] = sum(vals) / len(vals)
print(json.dumps(out, indent=1))
