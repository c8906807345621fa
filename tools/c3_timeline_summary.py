"""Fold a `rocprofv3 --kernel-trace --memory-copy-trace --output-format csv` run of tools/c3_timeline.py
into the device timeline of its last aq_integrate_batch call (events, per-op totals, and the share of
the call's device span no k_stream covers). Diagnostic tool.

  python tools/c3_timeline_summary.py <rocprof dir> [--gap-us 300] [--what TEXT] > timeline.json

Calls are told apart by idle gaps longer than --gap-us between consecutive device events (the host
synchronises and checks counts between calls).
"""
import argparse
import collections
import csv
import glob
import json
import os


def rows(pattern, name_of):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name_of(r)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap-us", type=float, default=300.0)
    ap.add_argument("--what", default="")
    a = ap.parse_args()
    ev = rows(os.path.join(a.dir, "**", "*kernel_trace.csv"), lambda r: r["Kernel_Name"])
    ev += rows(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), lambda r: r["Direction"])
    ev.sort()
    groups, cur, end = [], [], None
    for s, e, n in ev:
        if cur and s - end > a.gap_us * 1e3:
            groups.append(cur)
            cur = []
        end = e if not cur else max(end, e)
        cur.append((s, e, n))
    if cur:
        groups.append(cur)
    last = groups[-1]
    t0 = last[0][0]
    span = max(e for _, e, _ in last) - t0
    tot = collections.defaultdict(float)
    for s, e, n in last:
        tot[n] += (e - s) / 1e3
    # device time covered by at least one k_stream
    cover, ce = 0.0, None
    for s, e, n in sorted(x for x in last if "k_stream" in x[2]):
        if ce is None or s >= ce:
            cover += e - s
            ce = e
        elif e > ce:
            cover += e - ce
            ce = e
    out = {"what": a.what, "calls_seen": len(groups), "span_us": span / 1e3, "k_stream_cover_us": cover / 1e3,
           "outside_k_stream_us": (span - cover) / 1e3, "totals_us": {k: round(v, 1) for k, v in sorted(tot.items())},
           "events": [{"start_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1), "op": n}
                      for s, e, n in last]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
