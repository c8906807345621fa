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


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "cosh4_eps1e-12"
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))[key]
    tpl, lpl = g["tasks_per_level"], g["leaves_per_level"]
    nlev = len(tpl)
    tr = [r for r in rows(os.path.join(d, "kt", "**", "*kernel_trace.csv")) if KERNEL in r["Kernel_Name"]]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs = len(tr) // nlev
    if runs == 0:
        sys.exit("no complete run of %d level dispatches (%d found)" % (nlev, len(tr)))
    tr = tr[len(tr) - runs * nlev:]   # whole integrate() calls; the first is the warmup

    def pmc(name):
        out = [float(r["Counter_Value"]) for r in rows(os.path.join(d, name.lower(), "**", "*counter_collection.csv"))
               if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
        return out[len(out) - runs * nlev:] if len(out) >= runs * nlev else None

    fetch, write = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
    levels = []
    for lev in range(nlev):
        durs = [(int(tr[k * nlev + lev]["End_Timestamp"]) - int(tr[k * nlev + lev]["Start_Timestamp"])) * 1e-9
                for k in range(1, runs)] or [(int(tr[lev]["End_Timestamp"]) - int(tr[lev]["Start_Timestamp"])) * 1e-9]
        t = sorted(durs)[len(durs) // 2]
        n_in, n_out = tpl[lev], 2 * (tpl[lev] - lpl[lev])
        alg = REC * (n_in + n_out)
        e = {"level": lev, "records_in": n_in, "records_out": n_out, "us": round(t * 1e6, 2),
             "alg_bytes": alg, "alg_GBps": round(alg / t / 1e9, 1), "hbm_frac_alg": round(alg / t / HBM_PEAK, 4),
             "fp64_frac": round(FLOP * n_in / t / FP64_PEAK, 4)}
        if fetch and write:
            hb = [(2 * fetch[k * nlev + lev] + write[k * nlev + lev]) * 1024 for k in range(runs)]
            e["hbm_bytes_measured"] = sorted(hb)[len(hb) // 2]
        levels.append(e)
    tot_t = sum(e["us"] for e in levels) * 1e-6
    tot_b = sum(e["alg_bytes"] for e in levels)
    widest = max(levels, key=lambda e: e["records_in"])
    print(json.dumps({"kernel": KERNEL, "workload": key, "levels": nlev, "runs_timed": max(runs - 1, 1),
                      "sum_level_us": round(tot_t * 1e6, 1), "alg_bytes_total": tot_b,
                      "alg_GBps_overall": round(tot_b / tot_t / 1e9, 1),
                      "fp64_frac_overall": round(FLOP * sum(tpl) / tot_t / FP64_PEAK, 4),
                      "widest_level": widest, "per_level": levels}, indent=1))


if __name__ == "__main__":
    main()
