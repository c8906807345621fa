"""Where a long launch's wave time goes (diagnostic; needs a library built with -DAQ_STAMPS=1, e.g.
python -c "from ppls_amd import build as b; b.build_variant('stamps', ['-DAQ_STAMPS=1'])", then
AQ_LIB=$PWD/ppls_amd/_build/libaquad_stamps.so python tools/stamps_burst.py).

Every wave of the plain instance sums the shader cycles it spends inside bursts of rounds (from the
burst's set-up to its push-back, cellar moves within it included) and in its whole loop, and counts
its bursts and rounds (aq_stream.h ST_CB .. ST_NR; two s_memtime per burst, no LDS atomics). One
untimed launch sizes the jobs, then one launch of --k copies of cosh4 on [0, 5] at --eps is read.
Prints one JSON line: the share of loop cycles outside bursts, cycles per round inside bursts, rounds
per burst, and their spread over waves.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402

ST_CB, ST_CL, ST_NB, ST_NR, ST_CS, ST_CF, ST_CBD, ST_NS, ST_STRIDE = 15, 16, 17, 18, 19, 20, 21, 22, 24
NW = 12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=32768)
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--c3", action="store_true", help="splitmix64 bounds (SURVEY C3) instead of [0, 5]")
    ap.add_argument("--batch", action="store_true",
                    help="through aq_integrate_batch (size-ordered chunks; the stamps are its last launch's)")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    if args.c3:
        from tools.bench_batch import splitmix64_bounds
        a, b = splitmix64_bounds(args.k)
    else:
        a, b = np.zeros(args.k), np.full(args.k, 5.0)
    if args.batch:
        ctx.integrate_batch(a, b, args.eps)
        ctx.kernel_timing(True)
        _, tasks, _ = ctx.integrate_batch(a, b, args.eps)
        r = type("R", (), {"tasks": int(tasks[-1])})
    else:
        ctx.integrate_many_async(a, b, args.eps)
        ctx.fetch(args.k - 1)
        ctx.kernel_timing(True)
        ctx.integrate_many_async(a, b, args.eps)
        r = ctx.fetch(args.k - 1)
    ms, _ = ctx.kernel_time()
    grid = ctx.num_workers // NW
    n = grid * NW * ST_STRIDE
    buf = (ctypes.c_uint64 * n)()
    rc = ctx.L.aq_debug_stamps(buf, ctypes.c_size_t(n))
    if rc:
        raise RuntimeError("aq_debug_stamps rc=%d" % rc)
    s = np.frombuffer(buf, dtype=np.uint64).reshape(grid * NW, ST_STRIDE).astype(np.float64)
    cb, cl, nb, nr = s[:, ST_CB], s[:, ST_CL], s[:, ST_NB], s[:, ST_NR]
    q = lambda v: [round(float(np.quantile(v, x)), 4) for x in (0.0, 0.5, 1.0)]
    out = {"k": args.k, "eps": args.eps, "c3": args.c3, "kernel_ms": ms, "tasks_last": r.tasks,
           "outside_bursts_share": float(1.0 - cb.sum() / cl.sum()),
           "outside_bursts_share_q": q(1.0 - cb / np.maximum(cl, 1.0)),
           "cycles_per_round_in_bursts": float(cb.sum() / max(nr.sum(), 1.0)),
           "rounds_per_burst": float(nr.sum() / max(nb.sum(), 1.0)),
           "bursts": float(nb.sum()), "rounds": float(nr.sum()),
           "loop_cycles_per_wave_q": q(cl)}
    ns = max(s[:, ST_NS].sum(), 1.0)
    out["seeding"] = {"passes": float(ns), "share_of_loop": float(s[:, ST_CS].sum() / cl.sum()),
                      "cycles_per_pass": float(s[:, ST_CS].sum() / ns),
                      "flush_cycles_per_pass": float(s[:, ST_CF].sum() / ns),
                      "bounds_cycles_per_pass": float(s[:, ST_CBD].sum() / ns)}
    # the launch's timeline: quantiles over waves of the realtime stamps (us after the first entry) --
    # first seeding, first idle (out of jobs), first lead, end seen, exit
    t = s.astype(np.int64)
    t0 = t[:, 0][t[:, 0] > 0].min()
    for name, col in (("seed_in", 2), ("idle", 4), ("lead", 5), ("done", 13), ("exit", 8)):
        v = t[:, col]
        v = v[v > 0]
        if len(v):
            out["t_" + name + "_us"] = [round(float(np.quantile((v - t0) / 100.0, x)), 1) for x in (0.0, 0.1, 0.5, 0.9, 1.0)]
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
