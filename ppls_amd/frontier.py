"""Rebalanced frontier engine across GPUs (BASELINE.json north star: "frontier sizes
are exchanged and rebalanced periodically over RCCL on xGMI").

Reference: /root/reference/aquadPartA.c. The reference balances load with its farmer's bag of tasks
(:125-173): any idle worker gets the next interval. Across GPUs the same job is done here level by
level: every rank holds a breadth-first frontier of intervals of one tree depth in HBM, applies the
task step (:183-202) to all of it with one HIP launch (aq_level_step, include/aquad.h), and after
every `rebalance_every` levels the ranks

  1. all-gather their frontier sizes (one int64 per rank), and
  2. move records from ranks above the mean to ranks below it with grouped point-to-point
     send / recv of contiguous record slices (torch.distributed P2P = RCCL over xGMI on "nccl"),

so a skewed integrand (sin(1/x), SURVEY H5: 4.7x imbalance under a static partition) keeps every
GPU busy. The run ends when the all-gathered sizes sum to zero (the farmer's `!is_empty(bag) ||
idle_count != workers`, :166). Every decision is the reference's arithmetic on the interval's own
endpoints, so the tree -- task and accepted counts -- is the reference's whatever the moves.

The per-rank accumulators {area (double-double), tasks, accepted, error bits, deepest level} stay
on the device; the final combine is one all-gather of them, folded on the host in double-double.

Backends: the product stepper is HipStepper (the C ABI). Tests pass the oracle's CPU restatement
(oracle/pyoracle.py: level_step) with the gloo backend to cover the multi-rank protocol on CPU.
"""
import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .aquad import AquadError, Problem, _check

REC = 4  # doubles per record {l, r, F(l), F(r)}
ERR_NAMES = {1: "on-device wait timed out", 2: "frontier capacity exceeded", 4: "maximum refinement depth reached"}


def plan_moves(counts: List[int]) -> List[Tuple[int, int, int]]:
    """Deterministic transfer plan (identical on every rank): (src, dst, n) moves that bring every
    rank to floor/ceil of the mean, taking from the largest surplus first. Ranks < total % N get
    the extra record."""
    n = len(counts)
    total = int(sum(counts))
    target = [total // n + (1 if i < total % n else 0) for i in range(n)]
    surplus = [[i, int(counts[i]) - target[i]] for i in range(n) if counts[i] > target[i]]
    deficit = [[i, target[i] - int(counts[i])] for i in range(n) if counts[i] < target[i]]
    surplus.sort(key=lambda e: (-e[1], e[0]))
    deficit.sort(key=lambda e: (-e[1], e[0]))
    moves = []
    si = di = 0
    while si < len(surplus) and di < len(deficit):
        k = min(surplus[si][1], deficit[di][1])
        moves.append((surplus[si][0], deficit[di][0], k))
        surplus[si][1] -= k
        deficit[di][1] -= k
        if surplus[si][1] == 0:
            si += 1
        if deficit[di][1] == 0:
            di += 1
    return moves


def dd_add(hi: float, lo: float, h2: float, l2: float) -> Tuple[float, float]:
    s = hi + h2
    bb = s - hi
    e = (hi - (s - bb)) + (h2 - bb) + lo + l2
    s2 = s + e
    return s2, e - (s2 - s)


class HipStepper:
    """The product path: one aq_level_step launch per level on the context's stream."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.device = torch.device("cuda", ctx.device)

    def root(self, integrand: int, a: float, b: float, out: torch.Tensor):
        _check(self.ctx.L.aq_frontier_root(self.ctx._h, integrand, float(a), float(b), out.data_ptr()),
               "aq_frontier_root")

    def step(self, integrand, fin, n_in, fout, cap, eps, depth, max_depth, nout, acc):
        _check(self.ctx.L.aq_level_step(self.ctx._h, integrand, fin.data_ptr(), int(n_in), fout.data_ptr(), int(cap),
                                        float(eps), int(depth), int(max_depth), nout.data_ptr(), acc.data_ptr()),
               "aq_level_step")

    def chain_step(self, integrand, fin, counts, depth, n_max, fout, cap, eps, max_depth, acc):
        """The level step reading its input count from counts[depth] on the device and appending to
        counts[depth + 1]: levels chain on the stream with no host round trip."""
        base = counts.data_ptr()
        _check(self.ctx.L.aq_level_step_chained(self.ctx._h, integrand, fin.data_ptr(), base + 4 * depth, int(n_max),
                                                fout.data_ptr(), int(cap), float(eps), int(depth), int(max_depth),
                                                base + 4 * (depth + 1), acc.data_ptr()),
               "aq_level_step_chained")

    def narrow(self, integrand, fronts, counts, depth, levels, cap, eps, max_depth, acc):
        """`levels` levels from `depth` in ONE single-workgroup launch (aq_level_narrow): level depth + k
        reads fronts[k % 2] and writes fronts[(k + 1) % 2]."""
        base = counts.data_ptr()
        _check(self.ctx.L.aq_level_narrow(self.ctx._h, integrand, fronts[0].data_ptr(), fronts[1].data_ptr(), int(cap),
                                          base, int(depth), int(levels), float(eps), int(max_depth), acc.data_ptr()),
               "aq_level_narrow")

    def integrate_one_gpu(self, problem, capacity, sync_every=4):
        """The whole single-GPU frontier run with its host loop in C (aq_frontier_integrate)."""
        from .aquad import _up
        r = _lib.aq_result()
        t = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
        lv = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
        _check(self.ctx.L.aq_frontier_integrate(self.ctx._h, ctypes.byref(problem.c()), int(capacity), int(sync_every),
                                                ctypes.byref(r), _up(t), _up(lv), _lib.AQ_MAX_LEVELS),
               "aq_frontier_integrate")
        per = [int(v) for v in t[:int(r.levels)]]
        return FrontierResult(area=r.area, tasks=int(r.tasks), accepted=int(r.accepted), levels=int(r.levels),
                              tasks_per_rank=[int(r.tasks)], accepted_per_rank=[int(r.accepted)], tasks_per_level=per,
                              rebalances=0, moved_records=0, max_frontier=max(per) if per else 0)

    def defer_folds(self, enable: bool):
        """Level steps leave their partial rows for one fold at the next sync (aq_level_defer_fold)."""
        _check(self.ctx.L.aq_level_defer_fold(self.ctx._h, 1 if enable else 0), "aq_level_defer_fold")

    def sync(self):
        self.ctx.synchronize()   # (also folds the deferred rows into the accumulator)


@dataclass
class FrontierResult:
    area: float
    tasks: int
    accepted: int
    levels: int
    tasks_per_rank: List[int]
    accepted_per_rank: List[int]
    tasks_per_level: List[int] = field(default_factory=list)
    rebalances: int = 0
    moved_records: int = 0
    max_frontier: int = 0


CHAIN_LEVELS = 4   # one GPU: levels chained on the device between host looks at the frontier size
NARROW_LEVELS = 13  # the tree's first levels (<= 2^12 records each) in one single-workgroup launch


def n_levels_narrow(max_depth: int) -> int:
    return max(0, min(NARROW_LEVELS, max_depth - 1))


def integrate(problem: Optional[Problem] = None, stepper=None, group=None, rebalance_every: int = 1,
              capacity: int = 1 << 22, c_loop: bool = True) -> FrontierResult:
    """One integral over every rank of `group` (torch.distributed, initialised by the caller; a
    single process runs without one). Collective: every rank calls it with the same arguments.

    A stepper with `chain_step` (HipStepper) keeps the per-level counts on the device and chains the
    levels between sync points -- every `rebalance_every` levels with several ranks (where the sizes
    are exchanged and records moved), every CHAIN_LEVELS levels on one -- so the host reads the
    frontier size once per sync point instead of once per level. Steppers without it (the CPU
    restatement in the tests) sync every level. With one GPU and c_loop (the default) the same levels
    run with their host loop in C (aq_frontier_integrate); c_loop=False keeps the Python loop."""
    problem = problem or Problem()
    if stepper is None:
        raise AquadError("frontier.integrate needs a stepper (HipStepper(ctx) on the GPU)")
    if rebalance_every < 1:
        raise AquadError("rebalance_every must be >= 1")
    integrand = problem.integrand if isinstance(problem.integrand, int) else {"cosh4": 0, "sin_recip": 1}[problem.integrand]
    max_depth = problem.max_depth or 96
    distributed = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if distributed else 0
    world = dist.get_world_size(group) if distributed else 1
    dev = stepper.device
    comm_dev = dev if (distributed and dist.get_backend(group) == "nccl") else torch.device("cpu")

    chain = getattr(stepper, "chain_step", None) if dev.type == "cuda" else None
    one_gpu = getattr(stepper, "integrate_one_gpu", None) if (c_loop and chain is not None and world == 1) else None
    if one_gpu is not None:
        # one GPU: no exchange to make -- the same levels with the host loop in C (aq_frontier_integrate)
        try:
            return one_gpu(problem, capacity, CHAIN_LEVELS)
        except AquadError as e:
            raise AquadError(f"frontier: {e}")
    sync_every = rebalance_every if world > 1 else CHAIN_LEVELS
    fronts = [torch.empty((capacity, REC), dtype=torch.float64, device=dev) for _ in range(2)]
    nout = torch.zeros(1, dtype=torch.int32, device=dev)
    acc = torch.zeros(8, dtype=torch.float64, device=dev)
    n = 1 if rank == 0 else 0
    counts = None
    if chain is not None:
        counts = torch.zeros(max_depth + 3, dtype=torch.int32, device=dev)   # counts[d]: records at level d
        counts[0] = n
    if dev.type == "cuda":
        # the zeroing ran on torch's stream, the level steps run on the engine's own stream: order them
        torch.cuda.synchronize(dev)
    cur = 0
    if rank == 0:
        stepper.root(integrand, problem.a, problem.b, fronts[cur])
    depth = 0
    rebalances = moved = 0
    max_front = 1
    per_level = []
    bound = n   # chained: an upper bound of this rank's current frontier (children <= 2 x parents)
    defer = getattr(stepper, "defer_folds", None) if chain is not None else None
    if defer is not None:
        defer(True)   # one fold per host look instead of one per level (aq_level_defer_fold)
    try:
        # one GPU: the narrow top in one launch (several ranks keep their per-level rebalancing from level 0)
        narrow = getattr(stepper, "narrow", None) if (chain is not None and world == 1) else None
        if narrow is not None and n_levels_narrow(max_depth) > 0:
            # levels 0 .. NARROW_LEVELS-1 (at most 2^(NARROW_LEVELS-1) records each) in one launch
            L0 = n_levels_narrow(max_depth)
            try:
                narrow(integrand, fronts, counts, 0, L0, capacity, problem.eps, max_depth, acc)
            except AquadError as e:
                raise AquadError(f"frontier: {e}")
            depth = L0
            cur = L0 % 2
            bound = min(1 << L0, capacity)
        while True:
            nxt = 1 - cur
            # a local failure is carried through the size exchange as a negative count, so every rank
            # raises together instead of the others waiting in the collective (one all-gather per level)
            err = ""
            synced = True
            if depth >= max_depth + 1:
                err = "maximum refinement depth reached"
                produced = 0
            elif chain is not None:
                try:
                    chain(integrand, fronts[cur], counts, depth, bound, fronts[nxt], capacity, problem.eps, max_depth, acc)
                except AquadError as e:
                    err = str(e)
                bound = min(2 * bound, capacity)
                synced = bool(err) or (depth + 1) % sync_every == 0
                produced = 0
                if synced and not err:
                    stepper.sync()
                    produced = int(counts[depth + 1].item())
                    if produced > capacity:
                        err = f"capacity exceeded: {produced} > {capacity}"
            else:
                try:
                    stepper.step(integrand, fronts[cur], n, fronts[nxt], capacity, problem.eps, depth, max_depth, nout,
                                 acc)
                    stepper.sync()
                    produced = int(nout.item())
                except AquadError as e:
                    err, produced = str(e), 0
                if not err and produced > capacity:
                    err = f"capacity exceeded: {produced} > {capacity}"
                per_level.append(n)
            cur, depth = nxt, depth + 1
            if not synced:
                continue
            n = 0 if err else produced
            bound = n
            mysize = torch.tensor([-1 if err else n], dtype=torch.int64, device=comm_dev)
            if distributed:
                gathered = [torch.zeros(1, dtype=torch.int64, device=comm_dev) for _ in range(world)]
                dist.all_gather(gathered, mysize, group=group)
                sizes = [int(g.item()) for g in gathered]
            else:
                sizes = [-1 if err else n]
            failed = [r for r, v in enumerate(sizes) if v < 0]
            if failed:
                raise AquadError(f"frontier: rank {failed[0]} failed" + (f" ({err})" if err else ""))
            total = sum(sizes)
            max_front = max(max_front, total)
            if total == 0:
                break
            if world > 1 and depth % rebalance_every == 0:
                moves = plan_moves(sizes)
                if moves:
                    rebalances += 1
                    ops = []
                    staged = []        # (device slice, host buffer): a CPU backend (gloo) with device records
                    send_end = n
                    recv_at = n
                    for src, dst, k in moves:
                        moved += k
                        if src == rank:
                            buf = fronts[cur][send_end - k:send_end]
                            if buf.device != comm_dev:
                                buf = buf.to(comm_dev)
                            ops.append(dist.P2POp(dist.isend, buf, dst, group))
                            send_end -= k
                        elif dst == rank:
                            if recv_at + k > capacity:   # every rank computes the same plan: all raise together
                                raise AquadError(f"frontier capacity exceeded on rank {rank} while receiving")
                            buf = fronts[cur][recv_at:recv_at + k]
                            if buf.device != comm_dev:
                                host = torch.empty((k, REC), dtype=torch.float64, device=comm_dev)
                                staged.append((buf, host))
                                buf = host
                            ops.append(dist.P2POp(dist.irecv, buf, src, group))
                            recv_at += k
                    if ops:
                        for req in dist.batch_isend_irecv(ops):
                            req.wait()
                    for dst_slice, host in staged:
                        dst_slice.copy_(host)
                    n = send_end + (recv_at - n)      # a rank only sends or only receives
                    bound = n
                    if counts is not None:
                        counts[depth] = n             # the next chained step reads it on the device
                    if dev.type == "cuda":
                        torch.cuda.synchronize(dev)   # the next level runs on the engine's own stream
        stepper.sync()
        if counts is not None:
            per_level = [int(v) for v in counts[:depth].cpu()]
        mine = acc.to(comm_dev)
        if distributed:
            accs = [torch.zeros(8, dtype=torch.float64, device=comm_dev) for _ in range(world)]
            dist.all_gather(accs, mine, group=group)
            lv = torch.tensor(per_level, dtype=torch.int64, device=comm_dev)
            # per-level task counts: ranks ran the same number of levels (one collective per level)
            dist.all_reduce(lv, op=dist.ReduceOp.SUM, group=group)
            per_level = [int(v) for v in lv.cpu()]
        else:
            accs = [mine]
        while per_level and per_level[-1] == 0:   # chained levels past the last sync point
            per_level.pop()
        rows = [a.cpu().numpy() for a in accs]
        hi = lo = 0.0
        for r in rows:
            hi, lo = dd_add(hi, lo, float(r[0]), float(r[1]))
        err = 0
        for r in rows:
            err |= int(r[4])
        if err:
            msg = "; ".join(v for k, v in ERR_NAMES.items() if err & k)
            raise AquadError(f"frontier: {msg}")
        tasks = [int(r[2]) for r in rows]
        leaves = [int(r[3]) for r in rows]
        return FrontierResult(area=hi + lo, tasks=sum(tasks), accepted=sum(leaves), levels=int(max(r[5] for r in rows)),
                              tasks_per_rank=tasks, accepted_per_rank=leaves, tasks_per_level=per_level,
                              rebalances=rebalances, moved_records=moved, max_frontier=max_front)
    finally:
        if defer is not None:
            defer(False)
