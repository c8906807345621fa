"""Where a lone launch's workgroups start, per XCD (diagnostic tool): the DIAG kernel instance of a
K=1 launch records each workgroup's start (s_memrealtime) and hardware CU slot. Three set-ups:
  reused  -- the launch reuses slot 0 (a k_reset and a memset of its per-CU words precede it),
  fresh   -- every launch takes a slot never used before (nothing precedes it on the stream),
  settled -- slot 0, but the stream is drained and the host sleeps 1 ms before the launch.
Also the plain (non-DIAG) kernel time of the same three.   python tools/xcd_start.py [--eps 1e-10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402


def starts(ctx):
    d, f = ctx.diagnostics()
    col = dict(zip(f, d.T.astype(np.float64)))
    t0 = col["t_start"].min()
    us = (col["t_start"] - t0) / 100.0
    xcc = col["cu"].astype(np.int64) >> 8
    return {int(x): round(float(us[xcc == x].max()), 2) for x in np.unique(xcc)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    one = (np.zeros(1), np.full(1, 5.0))
    out = {"eps": a.eps}
    for _ in range(3):
        ctx.integrate_many_async(*one, a.eps)
    ctx.synchronize()
    # plain kernel times
    for mode in ("reused", "fresh", "settled"):
        ctx.kernel_timing(True)
        for r in range(a.reps):
            if mode == "settled":
                ctx.synchronize()
                time.sleep(1e-3)
            ctx.integrate_many_async(*one, a.eps, first_slot=(100 + r) if mode == "fresh" else 0)
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        ctx.synchronize()
        out[mode + "_kernel_us"] = round(ms * 1e3 / max(n, 1), 2)
    # DIAG launches: the latest start per XCD (us after the first workgroup started)
    ctx.set_diagnostics(True)
    for mode in ("reused", "fresh", "settled"):
        if mode == "settled":
            ctx.synchronize()
            time.sleep(1e-3)
        ctx.integrate_many_async(*one, a.eps, first_slot=200 if mode == "fresh" else 0)
        ctx.synchronize()
        out[mode + "_start_us_by_xcd"] = starts(ctx)
    ctx.set_diagnostics(False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
