"""Fold one round's rocprofv3 output (tools/profile_round.sh) into the committed profiles/ files.

profiles/<tag>_kernel_stats.csv     rocprofv3 --kernel-trace --stats summary, verbatim
profiles/<tag>_summary.json         per-kernel dispatch durations from the trace, the bench line run
                                    under the profiler (its HIP-event kernel average beside rocprof's),
                                    and the PMC traffic per dispatch of the hot kernel
profiles/pmc_traffic.json           {"hbm_bytes_per_launch": ...} read by bench.py's roofline.traffic

HBM bytes follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and WRITE_SIZE
are in KiB, each collected in its own pass; on gfx950 FETCH_SIZE reads half the bytes, so it is
doubled (hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOT = "k_stream"


def find(d, name):
    hits = sorted(glob.glob(os.path.join(d, "**", name), recursive=True))
    return hits[0] if hits else None


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def col(row, *names):
    low = {k.lower(): v for k, v in row.items()}
    for n in names:
        if n.lower() in low:
            return low[n.lower()]
    raise KeyError(names)


def bench_line(path):
    try:
        with open(path) as f:
            for line in f:
                if line.startswith("{"):
                    return json.loads(line)
    except OSError:
        pass
    return None


def counter(d, name):
    p = find(d, "*counter_collection.csv")
    if p is None:
        return None
    vals = []
    for r in rows(p):
        if HOT in col(r, "Kernel_Name") and col(r, "Counter_Name") == name:
            vals.append(float(col(r, "Counter_Value")))
    if not vals:
        return None
    return {"dispatches": len(vals), "avg": sum(vals) / len(vals), "min": min(vals), "max": max(vals)}


def main():
    tag, out = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    summary = {"tag": tag}

    stats = find(os.path.join(out, "kt"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    trace = find(os.path.join(out, "kt"), "*kernel_trace.csv")
    if trace:
        per = {}
        for r in rows(trace):
            name = col(r, "Kernel_Name")
            dur = (int(col(r, "End_Timestamp")) - int(col(r, "Start_Timestamp"))) / 1e3
            per.setdefault(name, []).append(dur)
        summary["kernels"] = {k: {"dispatches": len(v), "avg_us": sum(v) / len(v), "min_us": min(v),
                                  "max_us": max(v)} for k, v in per.items()}
    b = bench_line(os.path.join(out, "bench_kt.json"))
    if b:
        summary["bench_under_rocprof"] = b
        hot = [v for k, v in summary.get("kernels", {}).items() if HOT in k]
        if hot:
            summary["hot_kernel_avg_us"] = {"rocprofv3": hot[0]["avg_us"],
                                            "bench_hip_events": b["roofline"]["kernel_avg_us"]}

    fetch = counter(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = counter(os.path.join(out, "write"), "WRITE_SIZE")
    summary["pmc"] = {"FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write}
    if fetch and write:
        hbm = (2.0 * fetch["avg"] + write["avg"]) * 1024.0
        tasks = b["roofline"]["tasks_per_launch"] if b else None
        summary["hbm_bytes_per_launch"] = hbm
        with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
            json.dump({"tag": tag, "kernel": HOT, "hbm_bytes_per_launch": hbm,
                       "fetch_size_kib_avg": fetch["avg"], "write_size_kib_avg": write["avg"],
                       "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE reads half)",
                       "tasks_per_launch": tasks,
                       "hbm_bytes_per_task": hbm / tasks if tasks else None}, f, indent=1)
            f.write("\n")
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
        f.write("\n")
    print(json.dumps({k: v for k, v in summary.items() if k != "bench_under_rocprof"}, indent=1))


if __name__ == "__main__":
    main()
