"""Wall-clock latency of one synchronous aq_integrate call (what a drop-in caller sees) against the
kernel time of the same launches (HIP events, in a second pass: `wall_timed_us` is that pass's wall),
averaged over --reps calls after a warm-up, through the CLI-style C path (ctypes call of aq_integrate,
no Python work between calls).
    python tools/try_wall.py [--reps 50]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context, Problem, SIN_RECIP  # noqa: E402
from ppls_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    out = {}
    for name, p in [("one_task", Problem(eps=1e9)), ("cosh4_eps1e-10", Problem(eps=1e-10)),
                    ("sin_recip_eps1e-9", Problem(integrand=SIN_RECIP, a=1e-4, b=1.0, eps=1e-9))]:
        for _ in range(3):
            ctx.integrate(p)
        cp = _lib.aq_problem(p.integrand, p.max_depth, p.a, p.b, p.eps, 0, 0)
        res = _lib.aq_result()
        # the wall without kernel timing (its events would sit in the measured calls), then the
        # kernel time of the same calls in a second pass
        t0 = time.perf_counter()
        for _ in range(args.reps):
            rc = ctx.L.aq_integrate(ctx._h, ctypes.byref(cp), ctypes.byref(res))
            assert rc == 0, rc
        wall = (time.perf_counter() - t0) / args.reps
        ctx.kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            rc = ctx.L.aq_integrate(ctx._h, ctypes.byref(cp), ctypes.byref(res))
            assert rc == 0, rc
        wall_timed = (time.perf_counter() - t0) / args.reps
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        out[name] = {"wall_us": round(wall * 1e6, 1), "wall_timed_us": round(wall_timed * 1e6, 1),
                     "kernel_us": round(ms * 1e3 / n, 1), "tasks": res.tasks}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
