"""Quick engine check on the GPU (diagnostic tool): parity of one engine against the golden trees and
a timing of K-integral launches.  python tools/try_engine.py [--engine dfs] [--k 256] [--reps 4]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context, Problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", default="dfs")
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--diag", action="store_true")
    args = ap.parse_args()
    trees = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))
    batch = json.load(open(os.path.join(ROOT, "tests", "golden", "batch.json")))
    ctx = Context(0)
    ctx.set_engine(args.engine)
    ctx.set_level_histograms(False)
    out = {"engine": args.engine, "workers": ctx.num_workers}
    # small parity first
    g = trees["cosh4_eps1e-3"]
    ctx.integrate_many_async(np.zeros(32), np.full(32, 5.0), 1e-3)
    rs = [ctx.fetch(i) for i in range(32)]
    out["eps1e-3_x32_ok"] = all((r.tasks, r.accepted) == (g["tasks"], g["leaves"]) for r in rs)
    out["eps1e-3_area"] = "%f" % rs[0].area
    from oracle import pyoracle as O
    a, b = O.batch_bounds(256)
    ctx.integrate_many_async(a, b, 1e-3)
    got = [ctx.fetch(i).accepted for i in range(256)]
    out["batch256_ok"] = got == batch["leaves_eps1e-3_first256"][:256]
    # the bench workload
    tag = {1e-10: "cosh4_eps1e-10", 1e-12: "cosh4_eps1e-12", 1e-8: "cosh4_eps1e-8"}[args.eps]
    g = trees[tag]
    k = args.k
    ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), args.eps)
    ctx.synchronize()
    ctx.kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), args.eps)
    ctx.synchronize()
    t1 = time.perf_counter()
    ms, n = ctx.kernel_time()
    rs = [ctx.fetch(i) for i in range(k)]
    bad = [(i, r.tasks, r.accepted) for i, r in enumerate(rs) if (r.tasks, r.accepted) != (g["tasks"], g["leaves"])]
    out["bench_ok"] = not bad
    out["bad"] = bad[:5]
    out["area0"] = rs[0].area
    out["area_rel_err"] = abs(rs[0].area - float(g["area_quad"])) / float(g["area_quad"])
    out["kernel_us"] = ms * 1e3 / max(n, 1)
    out["accepted_per_s_kernel"] = g["leaves"] * k / (ms * 1e-3 / max(n, 1))
    out["tasks_per_s_kernel"] = g["tasks"] * k / (ms * 1e-3 / max(n, 1))
    out["wall_accepted_per_s"] = g["leaves"] * k * args.reps / (t1 - t0)
    if args.diag:
        ctx.set_diagnostics(True)
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), args.eps)
        d, f = ctx.diagnostics()
        col = dict(zip(f, d.T.astype(np.float64)))
        out["diag"] = {key: float(col[key].sum()) for key in ("rounds", "active_lanes", "give", "pool_take",
                                                             "seed_calls", "seeds", "mixed_rounds", "c_seed", "c_loop")}
        out["diag"]["lanes_per_iter"] = out["diag"]["active_lanes"] / max(out["diag"]["rounds"], 1)
        out["diag"]["iters_per_wg_max"] = float(col["rounds"].max())
        out["diag"]["iters_per_wg_min"] = float(col["rounds"].min())
        t = (col["t_exit"] - col["t_start"].min()) / 100.0
        out["diag"]["t_exit_us"] = [float(t.min()), float(np.median(t)), float(t.max())]
        tl = (col["t_last_round"] - col["t_start"].min()) / 100.0
        out["diag"]["t_last_us"] = [float(tl.min()), float(np.median(tl)), float(tl.max())]
        for key in ("t_seeded", "t_first_lead"):
            if key in col:
                v = col[key][(col[key] > 0) & (col[key] < 2 ** 62)]
                if v.size:
                    tv = (v - col["t_start"].min()) / 100.0
                    out["diag"][key + "_us"] = [float(tv.min()), float(np.median(tv)), float(tv.max())]
        ts = (col["t_start"] - col["t_start"].min()) / 100.0
        out["diag"]["t_start_us"] = [float(ts.min()), float(np.median(ts)), float(ts.max())]
        for key in ("leads", "chunks_out", "chunks_in", "records_out", "pool_push", "cellar_out", "tasks"):
            if key in col:
                out["diag"][key] = float(col[key].sum())
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
