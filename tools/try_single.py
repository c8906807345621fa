"""Lone-integral kernel time (K=1 launches, HIP events) across tree sizes, from a 1-task tree to
eps=1e-12: separates the fixed cost of a persistent launch (start-up, seeding, termination) from
the per-task cost.  python tools/try_single.py [--reps 30]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context, Problem, SIN_RECIP  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--deep", action="store_true", help="also eps=1e-13 .. 1e-15 (30-150 M-task trees, 3 reps)")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    out = {"lib": os.environ.get("AQ_LIB", "default")}
    for name, p in [("one_task", Problem(eps=1e9)), ("eps1e-3", Problem(eps=1e-3)), ("eps1e-6", Problem(eps=1e-6)),
                    ("eps1e-8", Problem(eps=1e-8)), ("eps1e-10", Problem(eps=1e-10)), ("eps1e-12", Problem(eps=1e-12)),
                    ("sin_recip_eps1e-9", Problem(integrand=SIN_RECIP, a=1e-4, b=1.0, eps=1e-9))] + (
                   [("eps1e-13", Problem(eps=1e-13)), ("eps1e-14", Problem(eps=1e-14)), ("eps1e-15", Problem(eps=1e-15))]
                   if args.deep else []):
        ctx.integrate_async(p, 0)
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(args.reps if not name.startswith("eps1e-1") or name in ("eps1e-10", "eps1e-12") else 3):
            ctx.integrate_async(p, 0)
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        r = ctx.fetch(0)
        out[name] = {"us": round(ms * 1e3 / n, 2), "tasks": r.tasks}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
