"""Per-workgroup timeline of the persistent kernel (diagnostics build path, not timed).

  python tools/diag_persist.py [--eps 1e-10] [--reps 5] [--out gpurun_out/diag.json]
Prints, for the last of `reps` integrals: phase times (us, relative to the earliest workgroup
entry), rounds, lane occupancy, queue traffic and the per-workgroup task spread.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ppls_amd import Context, Problem  # noqa: E402


def summarize(d, f):
    col = {k: d[:, i].astype(np.float64) for i, k in enumerate(f)}
    t0 = col["t_start"].min()
    us = lambda v: (v - t0) / 100.0  # 100 MHz ticks -> us
    s = {}
    for k in ("t_start", "t_seeded", "t_first_lead", "t_last_round", "t_exit"):
        v = us(col[k])
        s[k] = {"min": round(v.min(), 2), "p50": round(float(np.median(v)), 2), "max": round(v.max(), 2)}
    r = np.maximum(col["rounds"], 1)
    s["rounds_per_wg"] = {"min": col["rounds"].min(), "p50": float(np.median(col["rounds"])), "max": col["rounds"].max()}
    s["lanes_per_round"] = float(col["active_lanes"].sum() / max(col["rounds"].sum(), 1))
    s["cyc_per_round"] = float(np.median(col["c_round"] / r))
    s["cyc_eval_per_round"] = float(np.median(col["c_eval"] / r))
    s["cyc_seed_per_call"] = float(col["c_seed"].sum() / max(col["seed_calls"].sum(), 1))
    for k in ("c_seed_pass1", "c_seed_pass2", "c_seed_resolve", "c_p1_class", "c_p1_walk", "c_p1_f"):
        s["cyc_" + k[2:] + "_per_call"] = float(col[k].sum() / max(col["seed_calls"].sum(), 1))
    s["cyc_idle_per_wg_p50"] = float(np.median(col["c_idle"]))
    s["cyc_round_per_wg_p50"] = float(np.median(col["c_round"]))
    s["cyc_seed_per_wg_p50"] = float(np.median(col["c_seed"]))
    s["cyc_refill_per_wg_p50"] = float(np.median(col["c_refill"]))
    s["cyc_loop_per_wg_p50"] = float(np.median(col["c_loop"]))   # sum over the workgroup's waves
    s["tasks_per_round"] = float(col["active_tasks"].sum() / max(col["rounds"].sum(), 1))
    # shares of the waves' loop time
    loop = max(float(np.median(col["c_loop"])), 1.0)
    s["share_of_loop"] = {k: round(float(np.median(col[c])) / loop, 3)
                          for k, c in (("round", "c_round"), ("seed", "c_seed"), ("idle_pool", "c_idle"),
                                       ("refill", "c_refill"))}
    s["tasks"] = {"min": col["tasks"].min(), "p50": float(np.median(col["tasks"])), "max": col["tasks"].max(),
                  "sum": col["tasks"].sum()}
    for k in ("leads", "pool_push", "pool_take", "give", "cellar_in", "cellar_out", "prefetch", "lock_spins", "spill_records", "chunks_out", "chunks_in",
              "records_out", "records_in", "seed_calls", "max_cellar"):
        s[k] = {"sum": col[k].sum(), "max": col[k].max()}
    polls = d[:, f.index("polls")].astype(np.uint64)
    s["polls"] = {"sum": float((polls & np.uint64(0xffffffff)).sum()), "saw_ticket": float((polls >> np.uint64(32)).sum())}
    s["t_wait_us_p50"] = float(np.median(col["t_wait"])) / 100.0
    s["max_ring"] = col["max_ring"].max()
    s["seeds"] = {"min": col["seeds"].min(), "max": col["seeds"].max()}
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--k", type=int, default=1, help="integrals per launch")
    ap.add_argument("--c3", action="store_true", help="splitmix64 bounds (SURVEY C3) instead of [0, 5]")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    if args.c3:
        from tools.bench_batch import splitmix64_bounds
        a, b = splitmix64_bounds(args.k)
    else:
        a, b = np.zeros(args.k), np.full(args.k, 5.0)
    if args.k > 1:
        # one plain launch of the same workload first: its tasks size the DIAG launch's jobs, as in the
        # bench (a fresh context's first launch runs the default job split)
        ctx.integrate_many_async(a, b, args.eps)
        ctx.fetch(args.k - 1)
    ctx.set_diagnostics(True)
    res = []
    for _ in range(args.reps):
        if args.k == 1:
            r = ctx.integrate(Problem(eps=args.eps))
        else:
            ctx.integrate_many_async(a, b, args.eps)
            r = ctx.fetch(args.k - 1)
        d, f = ctx.diagnostics()
        res.append(summarize(d, f))
    print(json.dumps({"eps": args.eps, "k": args.k, "tasks": r.tasks, "accepted": r.accepted, "summary": res[-1]}, indent=1,
                     default=float))
    if args.out:
        np.save(args.out.replace(".json", ".npy"), d)
        with open(args.out, "w") as fh:
            json.dump({"eps": args.eps, "fields": f, "summaries": res}, fh, default=float, indent=1)


if __name__ == "__main__":
    main()
