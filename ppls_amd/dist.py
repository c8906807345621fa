"""Multi-GPU quadrature: one process per GPU, torch.distributed (backend "nccl" = RCCL over xGMI).

Replaces the reference's inter-process layer (/root/reference/aquadPartA.c: farmer/worker
MPI_Send/MPI_Recv, :145-170, and the serial `result += buff[0]` combine, :149).

integrate_distributed -- one integral. Every rank runs aq_integrate_shard() on its cyclic share of
    the depth-D frontier (include/aquad.h), then ONE int64 all-reduce of the exact rows (area limbs,
    tasks, accepted, spilled: the area is the correctly rounded exact sum, whatever the partition)
    and one all-gather of {tasks, levels, error} per rank, whose task counts become the "Tasks Per
    Process" row (process 0 = farmer = 0, process r+1 = GPU r).

integrate_batch_distributed -- a batch, kept balanced live. Each integral is cut into S shards
    (units); every round the ranks take one window of the batch, split by a deterministic
    longest-processing-time plan over the units' predicted cost, each rank runs its units in ONE
    persistent launch (aq_integrate_mixed_async), and the ranks all-gather the units' measured task
    counts, which become the next round's cost model. No per-level host synchronisation: one launch
    + one all-gather per round. This is the farmer's dynamic dispatch (:144-166: idle workers get the
    next task) at the granularity of shards and launches.

Errors: a rank that fails (AquadError) still joins the collectives with an error code, so every
rank raises the same error instead of the healthy ranks hanging in the collective.

`shard_fn(problem, rank, world) -> exact row` is injectable so the same combine logic runs under
`gloo` on CPU in tests (with the CPU oracle as the shard backend). The default is the HIP engine.
"""
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .aquad import AquadError, Context, Problem, Result, exact_round

ROW = _lib.AQ_EXACT_ROW          # int64 row: limbs[AQ_XS_LIMBS], tasks, accepted, spilled, levels | error << 32
XL = _lib.AQ_XS_LIMBS


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def comm_device(group=None, ctx: Optional[Context] = None) -> torch.device:
    """Where this rank's collective tensors live: the context's GPU under nccl (never just the current
    device: RCCL rejects two ranks on one GPU), the CPU under gloo."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", ctx.device if ctx is not None else local_rank())
    return torch.device("cpu")


def _agree_on_errors(code: int, dev, group) -> None:
    """Every rank learns every rank's error code (one all-gather); any failure raises everywhere."""
    world = dist.get_world_size(group)
    mine = torch.tensor([code], dtype=torch.int64, device=dev)
    codes = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(codes, mine, group=group)
    bad = [(r, int(c.item())) for r, c in enumerate(codes) if int(c.item()) != 0]
    if bad:
        r, c = bad[0]
        raise AquadError(f"rank {r} failed ({_lib.load().aq_strerror(c).decode() if c < 0 else 'error'}, code {c})", c)


def _agree_on_workers(num_workers: int, dev, group) -> None:
    """The shard partition (shares, seed depth) is a function of the persistent worker count, so every
    rank must run the same one: ranks with different AQ_GRID settings or CU counts would combine shards
    of different partitions into wrong counts with no error. One all-gather; a mismatch raises on
    every rank (as aq_group does for the contexts of one process)."""
    world = dist.get_world_size(group)
    mine = torch.tensor([int(num_workers)], dtype=torch.int64, device=dev)
    rows = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(rows, mine, group=group)
    seen = [int(r.item()) for r in rows]
    if len(set(seen)) != 1:
        raise AquadError(f"ranks disagree on the persistent worker count {seen}: their shard partitions differ",
                         -1)   # AQ_EINVAL


def _err_code_from_bits(bits: int) -> int:
    """The C ABI's error code for a row's device error bits (aq_abi.inc err_from_bits)."""
    if bits & 1:
        return -3    # AQ_ETIMEOUT
    if bits & 2:
        return -4    # AQ_EOVERFLOW
    if bits & 4:
        return -5    # AQ_EDEPTH
    return -1


def combine_rows(row: np.ndarray, group=None, dev=None, err: int = 0) -> Result:
    """All-reduce one rank's exact row into the whole-run result (identical on every rank)."""
    dev = dev or torch.device("cpu")
    _agree_on_errors(err, dev, group)
    world = dist.get_world_size(group)
    s = torch.from_numpy(np.array(row[:XL + 3], np.int64)).to(dev)   # a copy: the all-reduce works in place
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    lev_err = int(row[XL + 3])
    info = torch.tensor([int(row[XL]), lev_err & 0xffffffff, lev_err >> 32], dtype=torch.int64, device=dev)
    gathered = [torch.zeros_like(info) for _ in range(world)]
    dist.all_gather(gathered, info, group=group)
    tot = s.cpu().numpy()
    rows = [g.cpu().numpy() for g in gathered]
    levels = max(int(r[1]) for r in rows)
    error = 0
    for r in rows:
        error |= int(r[2])
    if error:
        raise AquadError(f"a shard reported device error bits {error:#x}", error)
    out = Result(area=exact_round(tot[:XL]), tasks=int(tot[XL]), accepted=int(tot[XL + 1]), levels=levels, n_cu=0,
                 spilled=int(tot[XL + 2]))
    out.tasks_per_gpu = [int(r[0]) for r in rows]
    out.tasks_per_rank = out.tasks_per_gpu
    return out


def integrate_distributed(problem: Problem, group=None, ctx: Optional[Context] = None,
                          shard_fn: Optional[Callable[[Problem, int, int], np.ndarray]] = None) -> Result:
    """This rank's shard on its own GPU, then the collective combine (every rank gets the result)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"
    own = False
    if shard_fn is None and ctx is None:
        if nccl:
            torch.cuda.set_device(local_rank())
        ctx = Context(local_rank())
        own = True
    row, err = np.zeros(ROW, np.int64), 0
    # (the partition check can raise: a context this call created is closed on that path too)
    try:
        dev = comm_device(group, ctx if shard_fn is None else None) if (nccl or shard_fn is None) else torch.device("cpu")
        if shard_fn is None:
            _agree_on_workers(ctx.num_workers, dev, group)
        try:
            if shard_fn is None:
                row = ctx.integrate_shard_exact(problem, rank, world)   # internal slot: async slots untouched
            else:
                row = np.asarray(shard_fn(problem, rank, world), np.int64)
        except AquadError as e:
            err = e.code if e.code else -1
    finally:
        if own:
            ctx.close()
    return combine_rows(row, group, dev, err)


def tasks_per_process(res: Result):
    """[0 (farmer)] + per-rank task counts: the reference's tasks_per_process[] (aquadPartA.c:72, :162)."""
    return [0] + list(getattr(res, "tasks_per_rank", []))


# ---- the rebalanced batch ----------------------------------------------------------------------

def lpt_plan(costs: np.ndarray, world: int, start=None) -> List[List[int]]:
    """Longest-processing-time-first assignment of units to ranks (deterministic: ties by index),
    identical on every rank because every rank holds the same cost vector. `start`: the ranks'
    loads so far (the earlier rounds' measured tasks), so a round's odd unit goes where it evens out."""
    order = sorted(range(len(costs)), key=lambda u: (-float(costs[u]), u))
    load = [0.0] * world if start is None else [float(x) for x in start]
    plan: List[List[int]] = [[] for _ in range(world)]
    for u in order:
        r = min(range(world), key=lambda k: (load[k], k))
        plan[r].append(u)
        load[r] += float(costs[u])
    return [sorted(p) for p in plan]


@dataclass
class BatchResult:
    area: np.ndarray                  # per integral
    tasks: np.ndarray
    accepted: np.ndarray
    rounds: int = 0
    tasks_per_rank: List[int] = field(default_factory=list)      # tasks each rank evaluated
    kernel_ms_per_rank: List[float] = field(default_factory=list)
    predicted_imbalance: List[float] = field(default_factory=list)   # per round: max / mean planned cost


class HipBatchRunner:
    """The product path: a rank's units of a round in ONE persistent launch, rows read back exactly."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def run(self, a, b, shards, nshards, eps, integrand) -> np.ndarray:
        if len(a) == 0:
            return np.zeros((0, ROW), np.int64)
        n = len(a)
        dev = torch.device("cuda", self.ctx.device)
        out = torch.empty((n, ROW), dtype=torch.int64, device=dev)
        # the caching allocator orders `out` on torch's current stream, but the gather below writes it
        # on the library's own stream: whatever torch work still uses the block must finish first
        torch.cuda.current_stream(dev).synchronize()
        self.ctx.kernel_timing(True)
        try:
            self.ctx.integrate_mixed_async(a, b, shards, nshards, eps, first_slot=0, integrand=integrand)
            # every unit's row in one device gather, one copy back and one synchronisation
            self.ctx.gather_exact(0, n, out.data_ptr())
            self.ms, _ = self.ctx.kernel_time()   # synchronises the context's stream
        finally:
            self.ctx.kernel_timing(False)
        return out.cpu().numpy()


def integrate_batch_distributed(a, b, eps, integrand=0, group=None, runner=None, shards_per_integral=None,
                                window=None, rebalance=True) -> BatchResult:
    """A batch of integrals over every rank of `group`, rebalanced between launches (module doc).

    rebalance=False is the static partition for comparison: integral i's shard s always runs on rank
    s mod world (the per-GPU subranges of the north star's first sentence).

    shards_per_integral=1 makes whole integrals the units (static: integral i on rank i mod world):
    the choice for batches of small trees, whose shards would be seeding-bound."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    n = a.size
    # default unit: the whole integral when the batch gives every rank several (shards of small trees
    # are seeding-bound: config 4's 4096 sin(1/x) integrals over 8 ranks, makespan 0.75 ms whole vs
    # 4.56 ms rebalanced in 32 shards each); else 4 shards per rank and integral
    S = max(1, int(shards_per_integral or (1 if n >= 4 * world else 4 * world)))
    window = int(window or max(1, min(n, 8192 // S)))
    dev = torch.device("cpu") if dist.get_backend(group) != "nccl" else torch.device("cuda", runner.ctx.device)
    if runner is None:
        raise AquadError("integrate_batch_distributed needs a runner (HipBatchRunner(ctx) on the GPU)")
    if getattr(runner, "ctx", None) is not None:
        _agree_on_workers(runner.ctx.num_workers, dev, group)
    total = np.zeros((n, ROW), np.int64)
    shard_cost = np.ones(S)               # cost model: mean measured tasks of shard index s
    seen = np.zeros(S)
    my_tasks = 0
    my_ms = 0.0
    done = np.zeros(world)                # measured tasks each rank has run (the same on every rank)
    imb = []
    rounds = 0
    # the first round has no measurements (uniform costs): keep it short, so the unplanned part of
    # the batch is small; every later round is planned from the measured shard costs
    starts = [0]
    first = max(1, window // 4) if rebalance else window
    while starts[-1] + (first if len(starts) == 1 else window) < n:
        starts.append(starts[-1] + (first if len(starts) == 1 else window))
    bounds_ = list(zip(starts, starts[1:] + [n]))
    for w0, w1 in bounds_:
        ids = np.arange(w0, w1)
        units = [(int(i), s) for i in ids for s in range(S)]
        if rebalance:
            plan = lpt_plan(np.array([shard_cost[s] for _, s in units]), world, start=done)
        else:
            plan = [[u for u, (i, s) in enumerate(units) if (s if S > 1 else i) % world == r] for r in range(world)]
        loads = [sum(shard_cost[units[u][1]] for u in p) for p in plan]
        imb.append(max(loads) / (sum(loads) / world))
        mine = [units[u] for u in plan[rank]]
        err = 0
        rows = np.zeros((len(mine), ROW), np.int64)
        try:
            rows = runner.run(a[[i for i, _ in mine]], b[[i for i, _ in mine]],
                              np.array([s for _, s in mine], np.int32), S, eps, integrand)
            my_ms += getattr(runner, "ms", 0.0)
        except AquadError as e:
            err = e.code if e.code else -1
        # device error bits in the rows (a runner that returns them instead of raising) join the
        # agreement too: every rank raises together, none is left waiting in the all-reduce below
        bits = int(np.bitwise_or.reduce(rows[:, XL + 3] >> 32)) if rows.size else 0
        if bits and not err:
            err = _err_code_from_bits(bits)
        _agree_on_errors(err, dev, group)
        # every rank learns every unit's row: its share of the exact sums and the measured costs
        full = np.zeros((len(units), ROW), np.int64)
        for j, u in enumerate(plan[rank]):
            full[u] = rows[j]
        t = torch.from_numpy(full).to(dev)   # (`full` is this round's scratch: reduced in place is fine)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        full = t.cpu().numpy()
        for r in range(world):
            done[r] += float(sum(full[u, XL] for u in plan[r]))
        for u, (i, s) in enumerate(units):
            total[i, :XL + 3] += full[u, :XL + 3]
            seen[s] += 1
            shard_cost[s] += (float(full[u, XL]) - shard_cost[s]) / seen[s]
        my_tasks += int(rows[:, XL].sum()) if rows.size else 0
        rounds += 1
    per_rank = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(per_rank, torch.tensor([float(my_tasks), my_ms], dtype=torch.float64, device=dev), group=group)
    return BatchResult(area=np.array([exact_round(r[:XL]) for r in total]), tasks=total[:, XL].copy(),
                       accepted=total[:, XL + 1].copy(), rounds=rounds,
                       tasks_per_rank=[int(p[0].item()) for p in per_rank],
                       kernel_ms_per_rank=[float(p[1].item()) for p in per_rank], predicted_imbalance=imb)
