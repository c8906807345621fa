"""Summarise rocprofv3 --pmc CSVs of the persistent kernels: per-dispatch SQ counters of the largest
dispatches (the K-integral launches), normalised per wave-round. Diagnostic tool."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
WAVES_PER_SIMD = 3   # k_stream: 12 waves per workgroup, one workgroup per CU, 4 SIMDs
TASKS = float(os.environ.get("PMC_TASKS", 8192 * 1464273))   # tasks per dispatch (tools/pmc_profile.sh's launch)
out = {}
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    eng = os.path.basename(os.path.dirname(f))
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        if "k_stream" not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    if not per:
        continue
    big = sorted(per.items(), key=lambda kv: -max(kv[1].values()))[:2]
    avg = {k: sum(d[1].get(k, 0) for d in big) / len(big) for k in big[0][1]}
    if "SQ_ACTIVE_INST_VALU" in avg and avg.get("SQ_WAVE_CYCLES"):
        # SQ_WAVE_CYCLES and SQ_ACTIVE_INST_VALU are both summed over every wave (quad-cycles): their
        # ratio is the share of a WAVE's time in which it issues VALU. The persistent kernel keeps
        # WAVES_PER_SIMD (3) waves resident on every SIMD for the whole dispatch, so the SIMD's VALU
        # busy share is that ratio times 3 (the r02 tool reported the per-wave ratio as per-SIMD).
        avg["valu_issue_frac_per_wave"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
        avg["valu_busy_frac_per_simd_est"] = WAVES_PER_SIMD * avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
    if avg.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                avg[k.lower() + "_share_of_wave_cycles"] = avg[k] / avg["SQ_WAVE_CYCLES"]
    if TASKS:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_INT32"):
            if k in avg:
                avg[k.lower() + "_per_task"] = avg[k] / TASKS
        f64 = sum(avg.get(k, 0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        if f64:
            avg["fp64_insts_per_task"] = f64 / TASKS
    out[eng] = {"kernel": names[big[0][0]][:60], "dispatches": [d[0] for d in big], "avg": avg}
print(json.dumps(out, indent=1))

# hardware-executed FP64 FLOP of the stream kernel's dispatches (whole-device totals of wave-level
# instruction counts x 64 lanes; FMA = 2 FLOP, inactive lanes included) -- the PMC cross-check of
# the algorithmic 38 FLOP per task that bench.py's roofline uses. Pass the kernel's average
# duration (us, from the kernel-trace run) as argv[2] to get the rate.
f64 = {}
for eng, d in out.items():
    a = d["avg"]
    if "SQ_INSTS_VALU_FMA_F64" in a:
        flop = 64.0 * (a.get("SQ_INSTS_VALU_ADD_F64", 0) + a.get("SQ_INSTS_VALU_MUL_F64", 0) +
                       a.get("SQ_INSTS_VALU_TRANS_F64", 0) + 2.0 * a["SQ_INSTS_VALU_FMA_F64"])
        f64[eng] = {"fp64_flop_per_dispatch": flop}
        if len(sys.argv) > 2:
            t = float(sys.argv[2]) * 1e-6
            f64[eng]["fp64_tflops_hw"] = flop / t / 1e12
            f64[eng]["frac_of_78.6"] = flop / t / 78.6e12
if f64:
    print(json.dumps({"fp64_hw": f64}, indent=1))
