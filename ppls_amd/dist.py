"""Multi-GPU quadrature: one process per GPU, torch.distributed (backend "nccl" = RCCL over xGMI).

Replaces the reference's inter-process layer (/root/reference/aquadPartA.c: farmer/worker
MPI_Send/MPI_Recv, :145-170, and the serial `result += buff[0]` combine, :149). The tree is
partitioned with NO data-path communication: every rank runs aq_integrate_shard() on its
cyclic share of the depth-D frontier (include/aquad.h), then ONE all-reduce combines
{area, tasks, accepted} and one all-gather collects the per-rank task counts that become the
"Tasks Per Process" row (process 0 = farmer = 0, process r+1 = GPU r).

`shard_fn(problem, rank, world) -> Result` is injectable so the same combine logic runs under
`gloo` on CPU in tests (with the CPU oracle as the shard backend). The default is the HIP engine.
"""
import os
from typing import Callable, Optional

import torch
import torch.distributed as dist

from .aquad import Context, Problem, Result


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def _device_for(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def combine(part: Result, group=None) -> Result:
    """All-reduce one shard's partial result into the whole-run result (identical on every rank)."""
    dev = _device_for(group)
    world = dist.get_world_size(group)
    f = torch.tensor([part.area], dtype=torch.float64, device=dev)
    c = torch.tensor([part.tasks, part.accepted, part.spilled], dtype=torch.int64, device=dev)
    m = torch.tensor([part.levels], dtype=torch.int64, device=dev)
    per = torch.tensor([part.tasks], dtype=torch.int64, device=dev)
    gathered = [torch.zeros_like(per) for _ in range(world)]
    dist.all_reduce(f, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(c, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    dist.all_gather(gathered, per, group=group)
    out = Result(area=float(f.item()), tasks=int(c[0].item()), accepted=int(c[1].item()), levels=int(m.item()),
                 n_cu=part.n_cu * world, spilled=int(c[2].item()))
    out.tasks_per_cu = {}
    out.tasks_per_rank = [int(g.item()) for g in gathered]
    return out


def integrate_distributed(problem: Problem, group=None, ctx: Optional[Context] = None,
                          shard_fn: Optional[Callable[[Problem, int, int], Result]] = None) -> Result:
    """This rank's shard on its own GPU, then the collective combine."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if shard_fn is None:
        own = ctx is None
        ctx = ctx or Context(local_rank())
        try:
            part = ctx.integrate_shard(problem, rank, world)
        finally:
            if own:
                ctx.close()
    else:
        part = shard_fn(problem, rank, world)
    return combine(part, group)


def tasks_per_process(res: Result):
    """[0 (farmer)] + per-rank task counts: the reference's tasks_per_process[] (aquadPartA.c:72, :162)."""
    return [0] + list(getattr(res, "tasks_per_rank", []))
