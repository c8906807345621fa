"""Fold rocprofv3 --pmc passes of the bench launch (tools/pmc_bench_launch.py under tools/r05_pmc_valu.sh)
into the FP64 / VALU figures the roofline line carries (profiles/<tag>/pmc_valu.json). Diagnostic tool.

  python tools/pmc_valu.py <dir> [--tasks T] [--round-valu 96] [--tasks-per-round 127.17] > pmc_valu.json

<dir> holds p*/run_counter_collection.csv (one rocprofv3 --pmc pass each) and kt/run_kernel_trace.csv
(the kernel-trace pass of the same command). Only the k_stream dispatches of the bench shape count (the
timed launches: every k_stream dispatch but the first, which is the untimed launch that sizes the jobs).

Derived (units: counts are whole-device wave-instruction totals per dispatch; SQ_*_CYCLES and
SQ_ACTIVE_INST_* are quad-cycles summed over waves, MI355X_MICROARCH.md):
  fp64_flop_hw      64 lanes x (ADD + MUL + TRANS + 2 FMA) F64 wave-instructions: what the VALU executed,
                    idle lanes included (the compares are not in these classes)
  valu_busy         SIMD VALU-issue share: ACTIVE_INST_VALU / (WAVE_CYCLES / waves per SIMD) -- the
                    persistent grid keeps 3 waves on every SIMD for the whole dispatch
  issue_bound_frac  the algorithmic frac this instruction stream would reach with the VALU issuing every
                    cycle: frac / valu_busy
  valu_in_round     round_valu (the round's static VALU count, tools/isa_stats.py) x wave-rounds, wave-rounds
                    = tasks / tasks_per_round (the DIAG instance's measured 2 x active lanes per round)
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

FP64_PEAK = 78.6e12
FLOP_PER_TASK = 38
WAVES_PER_SIMD = 3
N_SIMD = 1024
KERNEL = "k_stream<0, false, false, false"   # (r05: a fifth template argument, the waves per workgroup)


def counters(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def durations(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL in r["Kernel_Name"]:
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return [d for _, d in sorted(out)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tasks", type=float, default=32768 * 1464273.0, help="tasks per dispatch")
    ap.add_argument("--round-valu", type=float, default=96.0)
    ap.add_argument("--tasks-per-round", type=float, default=None)
    ap.add_argument("--tag", default=None, help="profiles/<tag> the summary is committed under")
    a = ap.parse_args()
    avg = {}
    npass = {}
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "run_counter_collection.csv"))):
        per = counters(f)
        if not per:
            continue
        # the timed launches: every dispatch after the first (the untimed job-sizing launch)
        ds = sorted(per)[1:] or sorted(per)
        for c in per[ds[0]]:
            avg[c] = sum(per[d][c] for d in ds) / len(ds)
        npass[os.path.basename(os.path.dirname(f))] = len(ds)
    dur = durations(os.path.join(a.dir, "kt", "run_kernel_trace.csv"))
    dur = dur[1:] or dur
    t = sum(dur) / len(dur) * 1e-9
    out = {"tag": a.tag or os.path.basename(os.path.normpath(a.dir)), "kernel": KERNEL, "dispatches_per_pass": npass, "kernel_avg_us": t * 1e6, "kernel_dispatches": len(dur),
           "tasks_per_dispatch": a.tasks, "counters": avg}
    d = {}
    frac = FLOP_PER_TASK * a.tasks / t / FP64_PEAK
    d["frac_algorithmic"] = frac
    d["tflops_algorithmic"] = FLOP_PER_TASK * a.tasks / t / 1e12
    if "SQ_INSTS_VALU_FMA_F64" in avg:
        f64 = {k: avg.get("SQ_INSTS_VALU_" + k + "_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS")}
        flop = 64.0 * (f64["ADD"] + f64["MUL"] + f64["TRANS"] + 2.0 * f64["FMA"])
        d["fp64_wave_insts"] = sum(f64.values())
        d["fp64_wave_insts_per_task"] = sum(f64.values()) / a.tasks
        d["fp64_flop_hw"] = flop
        d["fp64_flop_hw_per_task"] = flop / a.tasks
        d["tflops_fp64_hw"] = flop / t / 1e12
        d["frac_fp64_hw"] = flop / t / FP64_PEAK
    if "SQ_WAVE_CYCLES" in avg:
        waves = WAVES_PER_SIMD * N_SIMD
        d["clock_ghz_from_wave_cycles"] = 4.0 * avg["SQ_WAVE_CYCLES"] / waves / t / 1e9
    if "GRBM_GUI_ACTIVE" in avg:
        # summed over the 8 XCDs (each its own GRBM)
        d["clock_ghz_from_grbm_gui_active"] = avg["GRBM_GUI_ACTIVE"] / 8.0 / t / 1e9
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
        busy = WAVES_PER_SIMD * avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
        d["valu_busy"] = busy
        d["issue_bound_frac"] = frac / busy
        if "SQ_INSTS_VALU" in avg:
            d["cycles_per_valu_inst"] = 4.0 * avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_INSTS_VALU"]
    if "SQ_INSTS_VALU" in avg:
        d["valu_wave_insts"] = avg["SQ_INSTS_VALU"]
        d["valu_wave_insts_per_task"] = avg["SQ_INSTS_VALU"] / a.tasks
        if a.tasks_per_round:
            rounds = a.tasks / a.tasks_per_round
            d["wave_rounds"] = rounds
            d["valu_in_round"] = a.round_valu * rounds
            d["valu_outside_round_share"] = 1.0 - a.round_valu * rounds / avg["SQ_INSTS_VALU"]
    for k in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_INT32", "SQ_INSTS_BRANCH"):
        if k in avg:
            d[k.lower() + "_per_task"] = avg[k] / a.tasks
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_SCA"):
        if k in avg and "SQ_WAVE_CYCLES" in avg:
            d[k.lower() + "_share_of_wave_cycles"] = avg[k] / avg["SQ_WAVE_CYCLES"]
    out["derived"] = d
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
