"""bench.py's multi-rank line fields under torch.distributed gloo, world_size 2, on CPU.

The driver's N-GPU runs print one line from rank 0; it must show that the collective really spanned
N ranks (ranks_seen: an all-reduce of ones), the backend, and every rank's kernel time and tasks with
their imbalance. The same functions bench.py calls (ranks_seen, rank_stats, bench_line) run here over
gloo with stand-in measurements -- the RCCL path runs them with the GPU's."""
import argparse
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    try:
        import bench
        seen = bench.ranks_seen(dist, "cpu", True)
        # stand-ins: rank r ran 4 launches of (10 + r) ms each and 1000 (r + 1) tasks
        stats = bench.rank_stats(dist, "cpu", True, 40.0 + 4 * rank, 4, 1000.0 * (rank + 1), 0.05 + 0.01 * rank)
        args = argparse.Namespace(warmup=2, eps=1e-10)
        tot = np.array([[0.0, 1464273.0, 732137.0, 0.0]] * 8)
        line = bench.bench_line(args, world, 8, 1, 8, 0.06, 8 * 732137.0, 8 * 1464275.0, tot, 8.0, 256, 0.0, 0,
                                seen == world, dist.get_backend(), seen, stats, 1e12, 10.0, 8 * 1464273.0 / world,
                                None)
        q.put((rank, line))
    finally:
        dist.destroy_process_group()


def test_bench_line_multi_rank_fields():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    lines = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    line = lines[0]
    assert line["ranks_seen"] == 2 and line["n_gpus"] == 2 and line["backend"] == "gloo"
    assert line["verified"] is True
    pr = line["per_rank"]
    assert pr["kernel_ms"] == [40.0, 44.0] and pr["launches"] == [4, 4] and pr["tasks"] == [1000, 2000]
    assert abs(pr["task_imbalance"] - 2000 / 1500) < 1e-12
    assert abs(pr["kernel_imbalance"] - 44 / 42) < 1e-12
    assert lines[1]["per_rank"] == pr   # every rank holds the same gathered view
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line


def test_bench_line_single_process():
    """Without a process group: ranks_seen 1, one per-rank row."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.ranks_seen(dist, "cpu", False) == 1
    st = bench.rank_stats(dist, "cpu", False, 12.5, 2, 100.0, 0.02)
    assert st["kernel_ms"] == [12.5] and st["tasks"] == [100] and st["task_imbalance"] == 1.0
