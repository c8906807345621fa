"""Multi-GPU combine logic (ppls_amd/dist.py) under torch.distributed gloo, world_size 2, on CPU.

The shard backend is the CPU oracle's restatement of the device partition (oracle/aq_oracle.c
aqo_integrate_shard), so the collective path is exercised exactly as it runs over RCCL, and the
combined result must equal the single-process tree bit for bit in counts. Also: a failing rank makes
every rank raise (no hang), and the rebalanced batch keeps exact counts and balances the load."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _shard_row(p, r, w):
    from conftest import exact_row
    from oracle import pyoracle as O
    o = O.integrate_shard(r, w, G=256, integrand=p.integrand, a=p.a, b=p.b, eps=p.eps)
    return exact_row([o.area_quad_hi, o.area_quad_lo], o.tasks, o.leaves, 0, o.levels)


def _worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from ppls_amd.aquad import Problem
        from ppls_amd.dist import integrate_distributed, tasks_per_process
        out = []
        for prob in (Problem(eps=1e-8), Problem(integrand=1, a=1e-4, b=1.0, eps=1e-7), Problem(integrand=2, eps=1e-11)):
            res = integrate_distributed(prob, shard_fn=_shard_row)
            out.append((res.area, res.tasks, res.accepted, res.levels, tasks_per_process(res)))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(target, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=timeout) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_combine_equals_single(world, oracle):
    results = _run(_worker, world)
    ref = [oracle.integrate(eps=1e-8), oracle.integrate(oracle.SIN_RECIP, 1e-4, 1.0, 1e-7),
           oracle.integrate(oracle.USER, 0.0, 5.0, 1e-11)]
    for rank in range(world):
        for got, want in zip(results[rank], ref):
            area, tasks, acc, levels, tpp = got
            assert tasks == want.tasks and acc == want.leaves and levels == want.levels
            assert abs(area - want.area) <= 1e-12 * abs(want.area)
            assert tpp[0] == 0 and sum(tpp) == want.tasks and len(tpp) == world + 1
    assert all(results[r] == results[0] for r in range(world))   # identical on every rank


def _fail_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from ppls_amd.aquad import AquadError, Problem
        from ppls_amd.dist import integrate_distributed

        def shard_fn(p, r, w):
            if r == 1:
                raise AquadError("injected: maximum refinement depth reached", -5)
            return _shard_row(p, r, w)
        try:
            integrate_distributed(Problem(eps=1e-6), shard_fn=shard_fn)
            q.put((rank, "no error"))
        except AquadError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_failing_rank_raises_everywhere():
    """a rank that fails before the collective must not leave the others hanging."""
    results = _run(_fail_worker, 2, timeout=120)
    assert all("rank 1 failed" in results[r] and "depth" in results[r] for r in range(2)), results


class _OracleBatchRunner:
    """CPU stand-in for HipBatchRunner: each unit (integral, shard s of S) through the oracle's shard
    restatement (any partition shared by all ranks sums to the whole tree)."""

    def run(self, a, b, shards, nshards, eps, integrand):
        from conftest import exact_row
        from oracle import pyoracle as O
        rows = []
        for x, y, s in zip(a, b, shards):
            o = O.integrate_shard(int(s), int(nshards), G=2, integrand=integrand, a=float(x), b=float(y), eps=eps)
            rows.append(exact_row([o.area_quad_hi, o.area_quad_lo], o.tasks, o.leaves, 0, o.levels))
        self.ms = 0.0
        return np.array(rows, np.int64).reshape(-1, 72)


def _batch_worker(rank, world, port, rebalance, *rest):
    shards, q = (rest[0], rest[1]) if len(rest) == 2 else (None, rest[0])   # (_run appends the queue)
    _init(rank, world, port)
    try:
        from ppls_amd.dist import integrate_batch_distributed
        n = 12
        a = np.full(n, 1e-4)
        b = np.ones(n)
        r = integrate_batch_distributed(a, b, 1e-7, integrand=1, runner=_OracleBatchRunner(),
                                        shards_per_integral=shards or 4 * world, window=3, rebalance=rebalance)
        q.put((rank, (r.area.tolist(), r.tasks.tolist(), r.accepted.tolist(), r.tasks_per_rank, r.rounds)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("rebalance", [False, True])
def test_gloo_rebalanced_batch(oracle, rebalance):
    """sin(1/x) batch over 2 ranks: exact per-integral counts either way; with rebalancing the ranks'
    task counts end within 15 % of each other, where the static shard split leaves them ~1.5x apart."""
    world = 2
    results = _run(_batch_worker, world, rebalance, timeout=300)
    want = oracle.integrate(oracle.SIN_RECIP, 1e-4, 1.0, 1e-7)
    area, tasks, acc, per_rank, rounds = results[0]
    assert all(t == want.tasks for t in tasks) and all(x == want.leaves for x in acc)
    assert all(abs(v - want.area) <= 1e-12 * abs(want.area) for v in area)
    assert sum(per_rank) == 12 * want.tasks and rounds == (5 if rebalance else 4)   # a short first round
    ratio = max(per_rank) / min(per_rank)
    if rebalance:
        assert ratio < 1.15, per_rank
    else:
        assert ratio > 1.3, per_rank
    assert results[1] == results[0]


@pytest.mark.parametrize("rebalance", [False, True])
def test_gloo_batch_whole_integral_units(oracle, rebalance):
    """Whole integrals as the units (shards_per_integral=1, the default for batches of >= 4 integrals
    per rank): exact counts, and 12 equal integrals split 6 / 6 over 2 ranks either way."""
    world = 2
    results = _run(_batch_worker, world, rebalance, 1, timeout=300)
    want = oracle.integrate(oracle.SIN_RECIP, 1e-4, 1.0, 1e-7)
    area, tasks, acc, per_rank, rounds = results[0]
    assert all(t == want.tasks for t in tasks) and all(x == want.leaves for x in acc)
    assert all(abs(v - want.area) <= 1e-12 * abs(want.area) for v in area)
    assert per_rank == [6 * want.tasks, 6 * want.tasks]
    assert results[1] == results[0]


class _BitsRunner(_OracleBatchRunner):
    """A runner that returns device error bits in its rows instead of raising (rank 1 only)."""

    def __init__(self, rank):
        self.rank = rank

    def run(self, a, b, shards, nshards, eps, integrand):
        rows = super().run(a, b, shards, nshards, eps, integrand)
        if self.rank == 1 and rows.size:
            rows[0, 71] |= 4 << 32   # ERRB_DEPTH in the levels | error << 32 word
        return rows


def _bits_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from ppls_amd.aquad import AquadError
        from ppls_amd.dist import integrate_batch_distributed
        try:
            integrate_batch_distributed(np.full(4, 1e-4), np.ones(4), 1e-5, integrand=1, runner=_BitsRunner(rank),
                                        shards_per_integral=2, window=4, rebalance=False)
            q.put((rank, "no error"))
        except AquadError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_batch_error_bits_raise_everywhere():
    """error bits a runner RETURNS (not raises) on one rank make every rank raise -- the
    healthy ranks must not be left in the all-reduce."""
    results = _run(_bits_worker, 2, timeout=120)
    assert all("rank 1 failed" in results[r] and "depth" in results[r] for r in range(2)), results


def _workers_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        import types
        from ppls_amd.aquad import AquadError
        from ppls_amd.dist import integrate_batch_distributed
        runner = _OracleBatchRunner()
        runner.ctx = types.SimpleNamespace(num_workers=3072 if rank == 0 else 2048)   # e.g. AQ_GRID on rank 1
        try:
            integrate_batch_distributed(np.full(4, 1e-4), np.ones(4), 1e-5, integrand=1, runner=runner,
                                        shards_per_integral=2, window=4, rebalance=False)
            q.put((rank, "no error"))
        except AquadError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_batch_ranks_on_different_partitions_raise():
    """the shard partition follows the persistent worker count; ranks that disagree on it
    (AQ_GRID, CU counts) raise together before any shard runs, instead of combining shards of
    different partitions into wrong counts."""
    results = _run(_workers_worker, 2, timeout=120)
    assert all("disagree" in results[r] for r in range(2)), results


def _own_ctx_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        import ppls_amd.dist as D
        from ppls_amd.aquad import AquadError, Problem
        closed = []

        class _FakeContext:
            """Stands in for the Context integrate_distributed creates itself (own=True): it disagrees
            on the worker count across the ranks and records its close()."""
            def __init__(self, device):
                self.device = device
                self.num_workers = 3072 if rank == 0 else 2048

            def close(self):
                closed.append(True)

        D.Context = _FakeContext
        try:
            D.integrate_distributed(Problem(eps=1e-6))
            q.put((rank, ("no error", closed)))
        except AquadError as e:
            q.put((rank, (str(e), closed)))
    finally:
        dist.destroy_process_group()


def test_gloo_own_context_closed_when_partitions_disagree():
    """a Context integrate_distributed created itself is closed when the partition check
    raises (it used to leak ~1.2 GiB of device memory per rank on that path)."""
    results = _run(_own_ctx_worker, 2, timeout=120)
    for r in range(2):
        msg, closed = results[r]
        assert "disagree" in msg and closed == [True], results
