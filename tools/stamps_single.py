"""Plain-instance timeline of lone-integral launches (diagnostic; needs a library built with
-DAQ_STAMPS=1: python ppls_amd/build.py --variant stamps -DAQ_STAMPS=1, then
AQ_LIB=$PWD/ppls_amd/_build/libaquad_stamps.so python tools/stamps_single.py).

Every wave keeps the 100 MHz realtime clock at entry, after its ring set-up, after the workgroup
barrier, at its first seeding's start, bounds, F evaluation and end, when it first counts itself
idle, when it first leads and sees the end, when it leaves the loop, after its flush and at its
exit (aq_stream.h ST_*). Printed: the quantiles over waves of each
point relative to the earliest entry, per tree size, with the kernel's own HIP-event time.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context, Problem  # noqa: E402

# aq_stream.h ST_* order (ST_XCC = 9 holds the XCD id, not a time)
NAMES = ["entry", "init", "seed_in", "seeded", "idle", "lead", "broke", "flushed", "exit", None,
         "pre", "class", "feval", "done", "karg"] + [None] * 8
ORDER = ["entry", "karg", "pre", "init", "seed_in", "class", "feval", "seeded", "idle", "lead", "done", "broke",
         "flushed", "exit"]
ST_XCC, ST_STRIDE = 9, 24
NW = int(os.environ.get("AQ_STAMPS_NW", "8"))   # waves per workgroup of the lone instance (aq_abi.inc AQ_LONE_NW)


def timeline(ctx, grid):
    n = grid * NW * ST_STRIDE
    buf = (ctypes.c_uint64 * n)()
    rc = ctx.L.aq_debug_stamps(buf, ctypes.c_size_t(n))
    if rc:
        raise RuntimeError("aq_debug_stamps rc=%d" % rc)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(grid * NW, ST_STRIDE).astype(np.int64)
    t0 = a[:, 0].min()
    out = {}
    for nm in ORDER:
        i = NAMES.index(nm)
        v = a[:, i]
        v = v[v > 0]
        if len(v) == 0:
            continue
        us = (v - t0) / 100.0   # 100 MHz
        out[nm] = [round(float(np.quantile(us, q)), 2) for q in (0, 0.5, 0.9, 1.0)] + [int(len(v))]
    xcc = a[:, ST_XCC]
    out["entry_by_xcc_max"] = {int(x): round(float((a[xcc == x, 0].max() - t0) / 100.0), 2) for x in np.unique(xcc)}
    out["exit_by_xcc_max"] = {int(x): round(float((a[xcc == x, 8].max() - t0) / 100.0), 2) for x in np.unique(xcc)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    ctx.L.aq_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    grid = ctx.num_cus
    res = {"lib": os.environ.get("AQ_LIB", "default"), "grid": grid,
           "points": ORDER, "format": "us after the earliest wave entry: q0, q50, q90, q100, waves"}
    for name, p in [("one_task", Problem(eps=1e9)), ("eps1e-6", Problem(eps=1e-6)),
                    ("eps1e-10", Problem(eps=1e-10))]:
        ctx.integrate_async(p, 0)
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(args.reps):
            ctx.integrate_async(p, 0)
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        ctx.synchronize()
        r = ctx.fetch(0)
        d = {"kernel_us": round(ms * 1e3 / n, 2), "tasks": r.tasks}
        d.update(timeline(ctx, grid))
        res[name] = d
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
