"""Roofline of the level-synchronous frontier engine's compaction pass (k_level_step), per level.

Reads the rocprofv3 kernel trace (and, if present, the FETCH_SIZE / WRITE_SIZE passes) of
`tools/bench_frontier.py --workload cosh12` (tools/profile_frontier.sh) and the golden per-level
histograms (tests/golden/trees.json): level d reads tasks_per_level[d] records of 32 B {l, r, F(l),
F(r)} and writes 2 x (tasks - leaves)[d] child records of 32 B, and evaluates one F per record (38
FP64 FLOP per task, as k_stream). Prints one JSON object: per level n_in, duration, algorithmic
GB/s, measured HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md) and the FP64 fraction.

  python tools/profile_frontier.py <rocprof dir> [workload key, default cosh4_eps1e-12]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_level_step"
NARROW = 13   # ppls_amd/frontier.py NARROW_LEVELS
REC = 32
FLOP = 38
FP64_PEAK = 78.6e12
HBM_PEAK = 8.0e12


def rows(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        return []
    with open(hits[0], newline="") as f:
        return list(csv.DictReader(f))


def split_runs(disp, grid_key):
    """Dispatches of k_level_step in time order -> integrate() calls: a call starts at its root level
    (one 256-thread block) right after a wider launch. Chained calls may end with a few empty levels."""
    runs, cur, prev = [], [], None
    for r in disp:
        g = int(r[grid_key])
        if cur and g == 256 and prev is not None and prev > 256:
            runs.append(cur)
            cur = []
        cur.append(r)
        prev = g
    if cur:
        runs.append(cur)
    return runs


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "cosh4_eps1e-12"
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))[key]
    tpl, lpl = g["tasks_per_level"], g["leaves_per_level"]
    nlev = len(tpl)
    tr = [r for r in rows(os.path.join(d, "kt", "**", "*kernel_trace.csv"))]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    # r03: one GPU runs the first NARROW levels in one k_level_narrow dispatch; the k_level_step
    # dispatches of a call then start at level NARROW (a call = the dispatches after a narrow one)
    narrows = [r for r in tr if "k_level_narrow" in r["Kernel_Name"]]
    first = 0
    if narrows:
        first = NARROW
        starts = [int(r["Start_Timestamp"]) for r in narrows] + [1 << 62]
        steps = [r for r in tr if KERNEL in r["Kernel_Name"]]
        runs = [[r for r in steps if starts[i] < int(r["Start_Timestamp"]) < starts[i + 1]] for i in range(len(narrows))]
        runs = [r for r in runs if len(r) >= nlev - first]
        narrow_us = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in narrows)
    else:
        runs = [r for r in split_runs([r for r in tr if KERNEL in r["Kernel_Name"]], "Grid_Size_X") if len(r) >= nlev]
        narrow_us = []
    if not runs:
        sys.exit("no complete run of %d level dispatches" % nlev)
    timed = runs[1:] or runs   # the first call is the warmup
    folds = [r for r in tr if "k_level_fold" in r["Kernel_Name"]]
    fold_us = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in folds)

    def pmc(name):
        allr = [r for r in rows(os.path.join(d, name.lower(), "**", "*counter_collection.csv")) if r["Counter_Name"] == name]
        allr.sort(key=lambda r: int(r["Dispatch_Id"]))
        if narrows:
            rr, cur = [], None
            for r in allr:
                if "k_level_narrow" in r["Kernel_Name"]:
                    cur = []
                    rr.append(cur)
                elif KERNEL in r["Kernel_Name"] and cur is not None:
                    cur.append(r)
            rr = [x for x in rr if len(x) >= nlev - first]
            return [[float(x["Counter_Value"]) for x in run[:nlev - first]] for run in rr] or None
        rs = [r for r in allr if KERNEL in r["Kernel_Name"]]
        rr = [x for x in split_runs(rs, "Grid_Size") if len(x) >= nlev]
        return [[float(x["Counter_Value"]) for x in run[:nlev]] for run in rr] or None

    fetch, write = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
    levels = []
    for lev in range(first, nlev):
        i = lev - first
        durs = sorted((int(run[i]["End_Timestamp"]) - int(run[i]["Start_Timestamp"])) * 1e-9 for run in timed)
        t = durs[len(durs) // 2]
        n_in, n_out = tpl[lev], 2 * (tpl[lev] - lpl[lev])
        alg = REC * (n_in + n_out)
        e = {"level": lev, "records_in": n_in, "records_out": n_out, "us": round(t * 1e6, 2),
             "alg_bytes": alg, "alg_GBps": round(alg / t / 1e9, 1), "hbm_frac_alg": round(alg / t / HBM_PEAK, 4),
             "fp64_frac": round(FLOP * n_in / t / FP64_PEAK, 4)}
        if fetch and write:
            hb = sorted((2 * f[i] + w[i]) * 1024 for f, w in zip(fetch, write))
            e["hbm_bytes_measured"] = hb[len(hb) // 2]
        levels.append(e)
    tot_t = sum(e["us"] for e in levels) * 1e-6
    tot_b = sum(e["alg_bytes"] for e in levels)
    widest = max(levels, key=lambda e: e["records_in"])
    print(json.dumps({"kernel": KERNEL, "workload": key, "levels": nlev, "runs_timed": len(timed),
                      "dispatches_per_run": [len(r) for r in runs],
                      "narrow_levels": first, "narrow_us_median": narrow_us[len(narrow_us) // 2] if narrow_us else None,
                      "sum_level_us": round(tot_t * 1e6, 1), "alg_bytes_total": tot_b,
                      "alg_GBps_overall": round(tot_b / tot_t / 1e9, 1),
                      "fp64_frac_overall": round(FLOP * sum(tpl) / tot_t / FP64_PEAK, 4),
                      "fold_us_median": fold_us[len(fold_us) // 2] if fold_us else None,
                      "fold_us_max": fold_us[-1] if fold_us else None,
                      "widest_level": widest, "per_level": levels}, indent=1))


if __name__ == "__main__":
    main()
