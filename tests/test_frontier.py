"""Frontier engine with live rebalancing: the transfer plan, the multi-rank protocol
on CPU (gloo, world_size 2 and 3, oracle stepper) and, on the GPU, the HIP level step against the
golden trees. Bar: task / accepted counts bit-exact, area within 1e-12 of the quad-precision sum."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

AREA_RTOL = 1e-12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_plan_moves_balances():
    from ppls_amd.frontier import plan_moves
    rng = np.random.default_rng(3)
    for n in (2, 3, 5, 8):
        for _ in range(200):
            counts = [int(v) for v in rng.integers(0, 1000, n)]
            if rng.random() < 0.3:
                counts = [0] * n
                counts[int(rng.integers(0, n))] = int(rng.integers(0, 5000))
            moves = plan_moves(counts)
            after = list(counts)
            for s, d, k in moves:
                assert k > 0 and s != d
                after[s] -= k
                after[d] += k
            assert sum(after) == sum(counts)
            assert max(after) - min(after) <= 1
            senders = {s for s, _, _ in moves}
            receivers = {d for _, d, _ in moves}
            assert not senders & receivers          # a rank only sends or only receives
            assert plan_moves(counts) == moves      # deterministic (every rank computes the same)


def test_level_step_restatement_matches_oracle_tree(trees):
    """The CPU level step, iterated from the root, regenerates the golden per-level histogram."""
    from oracle import pyoracle as O
    g = trees["cosh4_eps1e-8"]
    fr = np.array([[0.0, 5.0, O.F(0.0), O.F(5.0)]])
    per_level, leaves = [], 0
    depth = 0
    while fr.shape[0]:
        kids, la, tasks, err = O.level_step(fr, 1e-8, depth, 96)
        assert err == 0
        per_level.append(tasks)
        leaves += la.size
        fr = kids
        depth += 1
    assert per_level == g["tasks_per_level"]
    assert sum(per_level) == g["tasks"] and leaves == g["leaves"]


def _worker(rank, world, port, name, every, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import json
        from oracle import pyoracle as O
        from ppls_amd import Problem, frontier
        g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "trees.json")))[name]
        p = Problem(0 if g["integrand"] == "cosh4" else 1, g["a"], g["b"], g["eps"])
        r = frontier.integrate(p, stepper=O.FrontierStepper(), rebalance_every=every, capacity=1 << 20)
        q.put((rank, r.tasks, r.accepted, r.area, r.tasks_per_rank, r.tasks_per_level, r.rebalances,
               r.moved_records))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,every", [(2, "cosh4_eps1e-8", 1), (3, "sin_recip_eps1e-9", 2),
                                              (2, "sin_recip_eps1e-9", 1)])
def test_rebalanced_frontier_gloo(trees, world, name, every):
    g = trees[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, every, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, tasks, acc, area, per_rank, per_level, nreb, moved in out:
        assert (tasks, acc) == (g["tasks"], g["leaves"])
        assert per_level == g["tasks_per_level"]
        assert abs(area - float(g["area_quad"])) <= AREA_RTOL * abs(float(g["area_quad"]))
        assert sum(per_rank) == g["tasks"]
        assert nreb > 0 and moved > 0
        # rebalanced every level: each level's frontier is split to within one record, so a rank
        # carries at most its share plus one task per level; every 2 levels: within 1.5x
        if every == 1:
            assert max(per_rank) <= g["tasks"] / world + len(per_level) + 1
        else:
            assert max(per_rank) <= 1.5 * g["tasks"] / world


@pytest.mark.gpu
def test_frontier_hip_single_rank(trees):
    from ppls_amd import Context, Problem, frontier
    with Context(0) as ctx:
        st = frontier.HipStepper(ctx)
        for name in ("cosh4_eps1e-3", "cosh4_eps1e-10", "sin_recip_eps1e-9", "cosh4_eps1e-12"):
            g = trees[name]
            p = Problem(0 if g["integrand"] == "cosh4" else 1, g["a"], g["b"], g["eps"])
            r = frontier.integrate(p, stepper=st)
            assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"]), name
            assert r.tasks_per_level == g["tasks_per_level"]
            assert abs(r.area - float(g["area_quad"])) <= AREA_RTOL * abs(float(g["area_quad"]))


@pytest.mark.gpu
def test_frontier_c_loop_equals_python_loop(trees):
    """One GPU: the C host loop (aq_frontier_integrate) and the Python chained loop run the same levels:
    identical counts and per-level histograms, areas within the double-double fold's rounding."""
    from ppls_amd import Context, Problem, frontier
    with Context(0) as ctx:
        st = frontier.HipStepper(ctx)
        for name in ("cosh4_eps1e-10", "sin_recip_eps1e-9"):
            g = trees[name]
            p = Problem(0 if g["integrand"] == "cosh4" else 1, g["a"], g["b"], g["eps"])
            rc = frontier.integrate(p, stepper=st)
            rp = frontier.integrate(p, stepper=st, c_loop=False)
            assert (rc.tasks, rc.accepted, rc.levels) == (rp.tasks, rp.accepted, rp.levels) == (g["tasks"], g["leaves"],
                                                                                                  g["levels"]), name
            assert rc.tasks_per_level == rp.tasks_per_level == g["tasks_per_level"]
            assert abs(rc.area - rp.area) <= 1e-13 * abs(rp.area)


@pytest.mark.gpu
def test_frontier_hip_capacity_overflow_raises():
    """A frontier wider than the buffers fails loudly on the chained path too (the device count
    passes the capacity between host looks; the kernel flags the dropped children)."""
    from ppls_amd import AquadError, Context, Problem, frontier
    with Context(0) as ctx:
        with pytest.raises(AquadError):
            frontier.integrate(Problem(0, 0.0, 5.0, 1e-12), stepper=frontier.HipStepper(ctx), capacity=1 << 16)
        r = frontier.integrate(Problem(0, 0.0, 5.0, 1e-3), stepper=frontier.HipStepper(ctx), capacity=1 << 16)
        assert (r.tasks, r.accepted) == (6567, 3284)   # the context is usable afterwards


@pytest.mark.gpu
def test_level_step_hip_matches_restatement():
    """One HIP level step on a random frontier against the CPU restatement: same children set,
    same accepted areas (bit-exact per record: the device F is glibc-exact)."""
    from oracle import pyoracle as O
    from ppls_amd import Context
    rng = np.random.default_rng(5)
    l = np.sort(rng.uniform(0.0, 5.0, 20000))
    w = rng.uniform(1e-6, 1e-2, l.size)
    fin = np.stack([l, l + w, O.F(l), O.F(l + w)], axis=1)
    with Context(0) as ctx:
        dev = torch.device("cuda", 0)
        tin = torch.from_numpy(fin).to(dev)
        tout = torch.empty((2 * fin.shape[0], 4), dtype=torch.float64, device=dev)
        nout = torch.zeros(1, dtype=torch.int32, device=dev)
        acc = torch.zeros(8, dtype=torch.float64, device=dev)
        from ppls_amd.frontier import HipStepper
        st = HipStepper(ctx)
        st.step(0, tin, fin.shape[0], tout, tout.shape[0], 1e-10, 10, 96, nout, acc)
        st.sync()
        n = int(nout.item())
        got = tout[:n].cpu().numpy()
        a = acc.cpu().numpy()
    kids, leaves, tasks, err = O.level_step(fin, 1e-10, 10, 96)
    assert err == 0 and n == kids.shape[0] and int(a[2]) == tasks and int(a[3]) == leaves.size
    key = lambda m: m[np.lexsort((m[:, 1], m[:, 0]))]
    assert np.array_equal(key(got), key(kids))
    want = float(np.sum(leaves.astype(np.longdouble)))
    assert abs((a[0] + a[1]) - want) <= 1e-14 * abs(want)


def _gpu_worker(rank, world, port, every, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import json
        from ppls_amd import Context, Problem, frontier
        trees = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "trees.json")))
        res = []
        with Context(0) as ctx:
            for name in ("sin_recip_eps1e-9", "cosh4_eps1e-10"):
                g = trees[name]
                p = Problem(0 if g["integrand"] == "cosh4" else 1, g["a"], g["b"], g["eps"])
                r = frontier.integrate(p, stepper=frontier.HipStepper(ctx), rebalance_every=every)
                res.append((name, r.tasks, r.accepted, r.area, r.tasks_per_rank, r.moved_records))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("every", [1, 3])
def test_rebalanced_frontier_two_ranks_one_gpu(trees, every):
    """The HIP level step under the multi-rank protocol: two processes on one GPU (gloo moves the
    records through host memory; on a multi-GPU node the same code moves them with RCCL). With
    rebalance_every=3 the levels between rebalancing chain on the device (aq_level_step_chained) and
    a move rewrites the device count the next chained step reads."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, every, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=150) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out:
        for name, tasks, acc, area, per_rank, moved in res:
            g = trees[name]
            assert (tasks, acc) == (g["tasks"], g["leaves"]), name
            assert abs(area - float(g["area_quad"])) <= AREA_RTOL * abs(float(g["area_quad"]))
            assert moved > 0
            assert max(per_rank) <= (g["tasks"] / 2 + 64 if every == 1 else 0.75 * g["tasks"])


@pytest.mark.gpu
def test_levels_after_small_frontier_on_one_context(trees):
    """a small-capacity frontier run leaves smaller buffers in the context; the level path
    that follows on the same context grows them to its own minimum instead of overflowing."""
    from ppls_amd import Context, Problem, frontier
    g = trees["cosh4_eps1e-12"]
    with Context(0) as ctx:
        r = frontier.integrate(Problem(0, 0.0, 5.0, 1e-3), stepper=frontier.HipStepper(ctx), capacity=1 << 16)
        assert (r.tasks, r.accepted) == (6567, 3284)
        lv = ctx.integrate_levels(Problem(0, 0.0, 5.0, 1e-12))
        assert (lv.tasks, lv.accepted, lv.levels) == (g["tasks"], g["leaves"], g["levels"])
        assert lv.tasks_per_level == g["tasks_per_level"]
