"""The torch.distributed RCCL paths executed on the GPU (backend "nccl" = RCCL): a world_size-1
process group on the one-GPU box runs the same device-tensor collectives an 8-GPU node runs --
dist.integrate_distributed's exact int64 combine, the frontier engine's per-level size all-gather,
the rebalanced batch's row all-reduce, and bench.py's timed-region all-reduce (under
torch.distributed.run). Counts bit-exact against the golden trees."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def gctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


def test_integrate_distributed_over_rccl(nccl_group, gctx, trees):
    from ppls_amd import Problem
    from ppls_amd.dist import integrate_distributed, tasks_per_process
    for name, f in [("cosh4_eps1e-10", 0), ("sin_recip_eps1e-9", 1), ("gauss_eps1e-13", 2)]:
        g = trees[name]
        r = integrate_distributed(Problem(f, g["a"], g["b"], g["eps"]), ctx=gctx)
        assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"]), name
        assert abs(r.area - float(g["area_quad"])) <= 1e-12 * abs(float(g["area_quad"]))
        assert tasks_per_process(r) == [0, g["tasks"]]


def test_frontier_over_rccl(nccl_group, gctx, trees):
    from ppls_amd import Problem, frontier
    g = trees["sin_recip_eps1e-9"]
    r = frontier.integrate(Problem(1, g["a"], g["b"], g["eps"]), stepper=frontier.HipStepper(gctx))
    assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"])
    assert r.tasks_per_level == g["tasks_per_level"]


def test_rebalanced_batch_over_rccl(nccl_group, gctx, trees):
    from ppls_amd.dist import HipBatchRunner, integrate_batch_distributed
    g = trees["sin_recip_eps1e-9"]
    n = 16
    r = integrate_batch_distributed(np.full(n, 1e-4), np.ones(n), 1e-9, integrand=1, runner=HipBatchRunner(gctx),
                                    shards_per_integral=8, window=8)
    assert (r.tasks == g["tasks"]).all() and (r.accepted == g["leaves"]).all()
    assert np.all(np.abs(r.area - float(g["area_quad"])) <= 1e-12 * float(g["area_quad"]))
    assert r.tasks_per_rank == [n * g["tasks"]]


def test_bench_collective_block_under_torchrun():
    """bench.py launched by torch.distributed.run with one rank: the process group is created and
    the timed region's all-reduce runs over RCCL; the line it prints is verified bit-exact."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--steps", "2", "--warmup", "1", "--batch", "512", "--no-cpu-baseline", "--no-single"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["verified"] is True and res["n_gpus"] == 1 and res["value"] > 0
