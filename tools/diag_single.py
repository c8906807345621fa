"""Timeline of ONE integral in one persistent launch (diagnostic tool): where the lone-integral
latency goes. Runs K=1 launches with the DIAG kernel instance and prints, over the 256 workgroups,
quantiles (us after the first workgroup started) of: start, seeded, last round, first lead
(workgroup went idle), exit; plus rounds and seeds per workgroup and the kernel time of plain
(non-DIAG) launches for comparison.   python tools/diag_single.py [--eps 1e-10] [--reps 5]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402


def q(v):
    return [round(float(x), 2) for x in np.quantile(v, [0.0, 0.5, 0.9, 1.0])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--k", type=int, default=1, help="integrals per launch (k < 16: the per-CU instance)")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    one = (np.zeros(args.k), np.full(args.k, 5.0))
    for _ in range(2):
        ctx.integrate_many_async(*one, args.eps)
    ctx.synchronize()
    ctx.kernel_timing(True)
    for _ in range(args.reps):
        ctx.integrate_many_async(*one, args.eps)
    ctx.synchronize()
    ms, n = ctx.kernel_time()
    ctx.kernel_timing(False)
    out = {"eps": args.eps, "k": args.k, "kernel_us_plain": ms * 1e3 / max(n, 1)}
    ctx.set_diagnostics(True)
    ctx.kernel_timing(True)
    ctx.integrate_many_async(*one, args.eps)
    ctx.synchronize()
    ms, n = ctx.kernel_time()
    ctx.kernel_timing(False)
    out["kernel_us_diag"] = ms * 1e3 / max(n, 1)
    d, f = ctx.diagnostics()
    col = dict(zip(f, d.T.astype(np.float64)))
    t0 = col["t_start"].min()
    us = lambda k: (col[k] - t0) / 100.0   # s_memrealtime: 100 MHz
    for k in ("t_start", "t_init", "t_seed_in", "t_class", "t_seeded", "t_last_round", "t_done", "t_broke", "t_flushed", "t_fold", "t_exit"):
        out[k + "_us_q0_50_90_100"] = q(us(k))
    lead = col["t_first_lead"]
    ok = lead < 2 ** 63
    if ok.any():
        out["t_first_lead_us_q0_50_90_100"] = q((lead[ok] - t0) / 100.0)
    out["t_wait_us_per_wg_q"] = q(col["t_wait"] / 100.0)
    if "cu" in col:   # start and exit by XCD (the CU slot's bits 8-10)
        xcc = col["cu"].astype(np.int64) >> 8
        out["t_start_us_by_xcd_min_max"] = {int(x): [round(float(us("t_start")[xcc == x].min()), 2),
                                                     round(float(us("t_start")[xcc == x].max()), 2)] for x in np.unique(xcc)}
        out["t_seeded_us_by_xcd_max"] = {int(x): round(float(us("t_seeded")[xcc == x].max()), 2) for x in np.unique(xcc)}
    for k in ("rounds", "seeds", "seed_calls", "active_lanes", "c_seed", "c_seed_pass1", "c_seed_pass2", "c_seed_resolve", "c_p1_class", "c_p1_walk", "c_p1_f", "c_loop", "c_round", "leads"):
        if k in col:
            out[k + "_q0_50_90_100"] = q(col[k])
    out["tasks"] = float(col["tasks"].sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
