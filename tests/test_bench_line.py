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
        line = bench.bench_line(args, world, 8, 1, 8, 0.06, 8 * 732137.0, 8 * 1464275.0, tot, 8.0, (256, 3072, 256), 0.0, 0,
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


def test_launcher_spawns_n_ranks_after_the_cpu_baseline():
    """--gpus 2 with no launcher: the CPU baseline is timed first (no GPU call in this process), then
    ONE child torch.distributed.run starts 2 ranks of this same script with the same arguments, the
    baseline travels to rank 0 through the environment, and the children's status is returned."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    calls, order = [], []
    args = bench.parse(["--gpus", "2", "--steps", "3", "--warmup", "1"])

    def baseline(eps):
        order.append("baseline")
        return {"value": 1.0, "kind": "port", "eps": eps}

    def runner(cmd, env):
        order.append("runner")
        calls.append((cmd, env))
        return 7

    rc = bench.spawn_ranks(args, ["--gpus", "2", "--steps", "3", "--warmup", "1"], runner=runner, baseline=baseline)
    assert rc == 7 and order == ["baseline", "runner"] and len(calls) == 1
    cmd, env = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd and "127.0.0.1" in cmd
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"]
    assert json.loads(env[bench.CPU_ENV]) == {"value": 1.0, "kind": "port", "eps": 1e-10}
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"   # the dmabuf IPC mode RCCL needs, set for the ranks
    # --no-cpu-baseline: nothing timed, nothing handed over
    calls.clear()
    order.clear()
    args = bench.parse(["--gpus", "4", "--no-cpu-baseline"])
    env0 = dict(os.environ)
    env0.pop(bench.CPU_ENV, None)
    rc = bench.spawn_ranks(args, ["--gpus", "4", "--no-cpu-baseline"], runner=runner, baseline=baseline)
    assert rc == 7 and order == ["runner"] and bench.CPU_ENV not in calls[0][1]


def test_launcher_world_size_mismatch_fails():
    """Under a launcher, WORLD_SIZE != --gpus is an error exit (before any GPU call), not a fallback."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_c3_bounds_and_kat_fixture():
    """The bench's C3 generator reproduces the committed splitmix64 bounds, and the exact KAT of the
    first 10 000 draws at eps=1e-10 is consistent (T = 2L - 1 summed, mean leaves 153 330.8)."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "tests", "golden", "batch.json")) as f:
        g = json.load(f)
    a, b = bench.splitmix64_bounds(16)
    assert [[float(x).hex(), float(y).hex()] for x, y in zip(a, b)] == g["first_bounds_hex"]
    n = g["kat_n_eps1e-10"]
    assert n == 10000 and g["kat_sum_tasks_eps1e-10"] == 2 * g["kat_sum_leaves_eps1e-10"] - n
    assert round(g["kat_sum_leaves_eps1e-10"] / n, 1) == 153330.8
    # every key the bench's C3 passes read exists, for both tolerances; the eps=1e-3 KAT is SURVEY's 711.5
    for keys in bench.C3_GOLDEN.values():
        assert all(k in g for k in keys.values())
    k3 = bench.C3_GOLDEN[1e-3]
    assert g[k3["kat_tasks"]] == 2 * g[k3["kat_leaves"]] - g[k3["kat_n"]]
    assert round(g[k3["kat_leaves"]] / g[k3["kat_n"]], 1) == 711.5
    assert len(g[k3["leaves"]]) == len(g[k3["area_hex"]]) == 256


def test_area_check():
    sys.path.insert(0, ROOT)
    import bench
    want = bench.GOLDEN[1e-10][2]
    assert bench.areas_ok([want, want * (1 + 5e-13)], want)
    assert not bench.areas_ok([want, want * (1 + 2e-12)], want)


def _rotation_worker(rank, world, port, shard_tasks, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    try:
        import bench
        seen = bench.ranks_seen(dist, "cpu", True)
        workers = bench.agree_on_workers(dist, "cpu", True, 3072)
        K, B = 20, 32768
        lb = max(1, min(world, (1 << 18) // B))          # bench.py: N batches per launch within 262144 slots
        plan = bench.launch_plan(K, lb)
        tasks = 0
        for m in plan:
            sh = bench.shard_rotation(rank, world, m * B)
            tasks += int((np.bincount(sh, minlength=world) * np.asarray(shard_tasks, np.int64)).sum())
        stats = bench.rank_stats(dist, "cpu", True, 1.0, len(plan), float(tasks), 0.1)
        q.put((rank, seen, workers, plan, stats))
    finally:
        dist.destroy_process_group()


def test_shard_rotation_balances_eight_ranks(oracle):
    """VERDICT r4 #5c: the N = 8 launch pattern bench.py's driver run will use -- 20 timed steps of
    32768 integrals as launches of 8 + 8 + 4 steps, each rank holding shard (rank + i) mod 8 of the
    launch's i-th integral -- over a gloo group of 8 ranks on CPU, with every shard's task count from
    the oracle's restatement of the device partition (16 virtual workers: 2 shares x 8 shards,
    tests/conftest.py device_seed_S). The ranks' tasks must be equal (imbalance <= 1.01) and sum to
    the 20 x 32768 whole trees; the snake partition's raw per-shard skew is kept in the assertion."""
    from conftest import device_seed_S
    world = 8
    G = 3072 // (192 * world)          # aq_stream.h AQ_GSPLIT_DEFAULT waves per share and shard
    shard_tasks = [oracle.integrate_shard(s, world, G=G, S=device_seed_S(G, world), eps=1e-10).tasks
                   for s in range(world)]
    total = 1464273
    assert sum(shard_tasks) == total
    assert max(shard_tasks) / (total / world) > 1.005   # the skew the rotation has to cancel
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rotation_worker, args=(r, world, port, shard_tasks, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen, workers, plan, stats = got[0]
    assert seen == world and workers == [3072] * world
    assert plan == [8, 8, 4]
    assert stats["task_imbalance"] <= 1.01
    assert sum(stats["tasks"]) == 20 * 32768 * total
    assert all(got[r][3] == stats for r in range(world))   # every rank holds the same gathered view


def _workers_mismatch(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    try:
        import bench
        try:
            bench.agree_on_workers(dist, "cpu", True, 3072 if rank == 0 else 2048)
            q.put((rank, "agreed"))
        except SystemExit as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_ranks_with_different_partitions_fail():
    """ranks whose persistent worker counts differ (AQ_GRID, CU count) would combine shards
    of different partitions; bench.py's check fails on every rank instead."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_workers_mismatch, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all("disagree" in got[r] for r in range(world))
