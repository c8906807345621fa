"""Multi-GPU combine logic (ppls_amd/dist.py) under torch.distributed gloo, world_size 2, on CPU.

The shard backend is the CPU oracle's restatement of the device partition (oracle/aq_oracle.c
aqo_integrate_shard), so the collective path is exercised exactly as it runs over RCCL, and the
combined result must equal the single-process tree bit for bit in counts."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


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
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        from oracle import pyoracle as O
        from ppls_amd.aquad import Problem, Result
        from ppls_amd.dist import integrate_distributed, tasks_per_process

        def shard_fn(p, r, w):
            o = O.integrate_shard(r, w, G=256, integrand=p.integrand, a=p.a, b=p.b, eps=p.eps)
            return Result(o.area, o.tasks, o.leaves, o.levels, 256)

        out = []
        for prob in (Problem(eps=1e-8), Problem(integrand=1, a=1e-4, b=1.0, eps=1e-7)):
            res = integrate_distributed(prob, shard_fn=shard_fn)
            out.append((res.area, res.tasks, res.accepted, res.levels, tasks_per_process(res)))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_combine_equals_single(world, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = [oracle.integrate(eps=1e-8), oracle.integrate(oracle.SIN_RECIP, 1e-4, 1.0, 1e-7)]
    for rank in range(world):
        for got, want in zip(results[rank], ref):
            area, tasks, acc, levels, tpp = got
            assert tasks == want.tasks and acc == want.leaves and levels == want.levels
            assert abs(area - want.area) <= 1e-12 * abs(want.area)
            assert tpp[0] == 0 and sum(tpp) == want.tasks and len(tpp) == world + 1
    assert results[0] == results[1]
