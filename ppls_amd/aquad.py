"""Host-side mirror of the reference's interface for the quadrature path.

Reference: /root/reference/aquadPartA.c
  - EPSILON / F / A / B macros (:45-48)          -> Problem
  - double farmer(int numprocs) (:125-173)         -> farmer(numprocs, problem) -> (area, tasks_per_process)
  - the numprocs < 2 error (:86-90)                -> AquadError with the same message
  - main()'s printout (:107-117)                   -> format_reference()
Everything here calls the HIP engine through the C ABI (include/aquad.h). There is no CPU path.
"""
import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _lib

COSH4 = 0
SIN_RECIP = 1
USER = 2        # the AQ_F_USER plug-in compiled into the library (default: exp(-x*x))
INTEGRANDS = {"cosh4": COSH4, "sin_recip": SIN_RECIP, "user": USER}

# aquadPartA.c:45-48
DEFAULT_EPSILON = 1e-3
DEFAULT_A = 0.0
DEFAULT_B = 5.0

ERR_NUMPROCS = "ERROR: Must have at least 2 processes to run"  # aquadPartA.c:87


class AquadError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


@dataclass
class Problem:
    integrand: int = COSH4
    a: float = DEFAULT_A
    b: float = DEFAULT_B
    eps: float = DEFAULT_EPSILON
    max_depth: int = 0
    n_gpus: int = 0

    def c(self):
        f = self.integrand if isinstance(self.integrand, int) else INTEGRANDS[self.integrand]
        return _lib.aq_problem(f, int(self.max_depth), float(self.a), float(self.b), float(self.eps),
                               int(self.n_gpus), 0)


@dataclass
class Result:
    area: float
    tasks: int
    accepted: int
    levels: int
    n_cu: int
    spilled: int = 0
    tasks_per_cu: Dict[int, int] = field(default_factory=dict)
    tasks_per_level: List[int] = field(default_factory=list)
    leaves_per_level: List[int] = field(default_factory=list)
    tasks_per_gpu: List[int] = field(default_factory=list)


def _check(rc, what):
    if rc != 0:
        msg = _lib.load().aq_strerror(rc).decode()
        raise AquadError(f"{what}: {msg} (code {rc})", rc)


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _up(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def exact_round(limbs) -> float:
    """Correctly rounded double of AQ_XS_LIMBS exact-accumulator limbs (e.g. summed over shards)."""
    v = np.ascontiguousarray(np.asarray(limbs)[:_lib.AQ_XS_LIMBS], np.int64)
    return _lib.load().aq_exact_round(v.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))


def user_integrand_name() -> str:
    return _lib.load().aq_user_integrand_name().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    _lib.load().aq_device_count(ctypes.byref(n))
    return n.value


class Context:
    """One GPU: owns device memory, the stream and the on-device work queue (aq_ctx)."""

    def __init__(self, device: int = 0):
        self.L = _lib.load()
        self._h = ctypes.c_void_p()
        _check(self.L.aq_ctx_create(int(device), ctypes.byref(self._h)), "aq_ctx_create")
        self.device = device
        self.num_cus = self.L.aq_ctx_num_cus(self._h)

    @property
    def num_workers(self) -> int:
        """Shares a lone integral is split into (the oracle partition's G): workgroups x waves."""
        return self.L.aq_ctx_num_workers(self._h)

    @property
    def device_bytes(self) -> int:
        """Device memory this context holds."""
        v = ctypes.c_uint64(0)
        _check(self.L.aq_ctx_device_bytes(self._h, ctypes.byref(v)), "aq_ctx_device_bytes")
        return v.value

    def set_stall_timeout(self, ms: float):
        """Fail a launch whose on-device work queue makes no progress for `ms` (not a run-time cap)."""
        _check(self.L.aq_set_stall_timeout(self._h, float(ms)), "aq_set_stall_timeout")

    def close(self):
        if self._h:
            self.L.aq_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_level_histograms(self, enable: bool):
        _check(self.L.aq_set_level_histograms(self._h, 1 if enable else 0), "aq_set_level_histograms")

    # -- results ---------------------------------------------------------------------------
    def _result(self, r, with_detail=True) -> Result:
        out = Result(r.area, int(r.tasks), int(r.accepted), int(r.levels), int(r.n_cu), int(r.spilled))
        out.tasks_per_gpu = [int(r.tasks)]
        if with_detail:
            cu = np.zeros(_lib.AQ_CU_SLOTS, np.uint64)
            self.L.aq_tasks_per_cu(self._h, _up(cu), _lib.AQ_CU_SLOTS)
            out.tasks_per_cu = {int(i): int(cu[i]) for i in np.nonzero(cu)[0]}
            t = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
            lv = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
            self.L.aq_level_histogram(self._h, _up(t), _up(lv), _lib.AQ_MAX_LEVELS)
            n = out.levels
            out.tasks_per_level = [int(v) for v in t[:n]]
            out.leaves_per_level = [int(v) for v in lv[:n]]
        return out

    # -- the hot path ----------------------------------------------------------------------
    def integrate(self, problem: Problem) -> Result:
        r = _lib.aq_result()
        _check(self.L.aq_integrate(self._h, ctypes.byref(problem.c()), ctypes.byref(r)), "aq_integrate")
        return self._result(r)

    def integrate_shard(self, problem: Problem, shard: int, nshards: int) -> Result:
        r = _lib.aq_result()
        _check(self.L.aq_integrate_shard(self._h, ctypes.byref(problem.c()), shard, nshards, ctypes.byref(r)),
               "aq_integrate_shard")
        return self._result(r)

    def integrate_shard_exact(self, problem: Problem, shard: int, nshards: int) -> np.ndarray:
        """This shard's exact row (int64[AQ_EXACT_ROW], as fetch_exact), run in the internal slot: no
        async slot of the caller is touched."""
        row = np.zeros(_lib.AQ_EXACT_ROW, np.int64)
        _check(self.L.aq_integrate_shard_exact(self._h, ctypes.byref(problem.c()), int(shard), int(nshards),
                                               row.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))),
               "aq_integrate_shard_exact")
        return row

    def integrate_levels(self, problem: Problem) -> Result:
        r = _lib.aq_result()
        t = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
        lv = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
        _check(self.L.aq_integrate_levels(self._h, ctypes.byref(problem.c()), ctypes.byref(r), _up(t), _up(lv),
                                          _lib.AQ_MAX_LEVELS), "aq_integrate_levels")
        return self._result(r)

    # -- async (bench) -----------------------------------------------------------------------
    @property
    def async_slots(self) -> int:
        return self.L.aq_async_slots()

    def integrate_async(self, problem: Problem, slot: int, shard: int = 0, nshards: int = 1):
        _check(self.L.aq_integrate_async(self._h, ctypes.byref(problem.c()), shard, nshards, slot),
               "aq_integrate_async")

    @property
    def max_integrals_per_launch(self) -> int:
        return self.L.aq_max_integrals_per_launch()

    def integrate_many_async(self, a, b, eps, first_slot=0, integrand=COSH4, max_depth=0, shard=0, nshards=1):
        """Enqueue len(a) integrals in one persistent launch; integral i lands in slot first_slot+i."""
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        _check(self.L.aq_integrate_many_async(self._h, integrand, a.size, _dp(a), _dp(b), float(eps), max_depth,
                                              shard, nshards, first_slot), "aq_integrate_many_async")

    def integrate_mixed_async(self, a, b, shards, nshards, eps, first_slot=0, integrand=COSH4, max_depth=0):
        """One launch of len(a) integral shards: integral i is shard shards[i] of nshards."""
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        sh = np.ascontiguousarray(shards, np.int32)
        _check(self.L.aq_integrate_mixed_async(self._h, integrand, a.size, _dp(a), _dp(b),
                                               sh.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(nshards),
                                               float(eps), max_depth, first_slot), "aq_integrate_mixed_async")

    def fetch(self, slot: int, detail=False) -> Result:
        r = _lib.aq_result()
        _check(self.L.aq_fetch(self._h, slot, ctypes.byref(r)), "aq_fetch")
        return self._result(r, with_detail=detail)

    def fetch_exact(self, slot: int) -> np.ndarray:
        """The slot's exact row: int64[AQ_EXACT_ROW] = area limbs, tasks, accepted, spilled, levels | error << 32."""
        row = np.zeros(_lib.AQ_EXACT_ROW, np.int64)
        _check(self.L.aq_fetch_exact(self._h, slot, row.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))),
               "aq_fetch_exact")
        return row

    def gather_exact(self, first_slot: int, n: int, device_ptr: int):
        """Enqueue n slots' exact int64 rows (AQ_EXACT_ROW each) into a device buffer."""
        _check(self.L.aq_gather_exact(self._h, first_slot, n, ctypes.c_void_p(device_ptr)), "aq_gather_exact")

    def gather_results(self, first_slot: int, n: int, device_ptr: int):
        """Enqueue slots' {area, tasks, accepted, error} rows into a device buffer (e.g. a torch tensor)."""
        _check(self.L.aq_gather_results(self._h, first_slot, n, ctypes.c_void_p(device_ptr)), "aq_gather_results")

    def synchronize(self):
        _check(self.L.aq_synchronize(self._h), "aq_synchronize")

    def kernel_timing(self, enable: bool):
        _check(self.L.aq_kernel_timing(self._h, 1 if enable else 0), "aq_kernel_timing")

    def kernel_time(self):
        ms = ctypes.c_double(0)
        n = ctypes.c_uint64(0)
        _check(self.L.aq_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n)), "aq_kernel_time")
        return ms.value, n.value

    DIAG_FIELDS = ("t_start", "t_seeded", "t_first_lead", "t_exit", "rounds", "tasks", "chunks_out", "chunks_in",
                   "records_out", "t_wait", "leads", "seeds", "pool_push", "cu", "records_in", "active_lanes",
                   "c_round", "c_eval", "pool_take", "lock_spins", "t_last_round", "spill_records", "max_ring", "c_seed",
                   "seed_calls", "c_seed_resolve", "max_cellar", "c_idle", "c_seed_pass1", "c_seed_pass2", "give", "cellar_in",
                   "cellar_out", "c_refill", "c_loop", "active_tasks", "prefetch", "t_init", "t_done", "t_fold",
                   "t_broke", "t_flushed", "c_p1_class", "c_p1_walk", "c_p1_f", "t_seed_in", "t_class", "polls")
    DIAG_WORDS = 48

    def set_diagnostics(self, enable: bool):
        _check(self.L.aq_set_diagnostics(self._h, 1 if enable else 0), "aq_set_diagnostics")

    def diagnostics(self):
        """Per-workgroup timeline of the last persistent launch: numpy (n_wg, DIAG_WORDS) uint64 + field names."""
        w = self.DIAG_WORDS
        out = np.zeros(w * 2048, np.uint64)
        n = self.L.aq_diagnostics(self._h, _up(out), out.size)
        if n < 0:
            _check(n, "aq_diagnostics")
        return out[:w * n].reshape(n, w), self.DIAG_FIELDS

    def cu_task_counters(self, reset: bool = False) -> Dict[int, int]:
        """Tasks per hardware CU slot over every persistent launch since the last reset (any launch
        shape: the farmer's tasks_per_process, aquadPartA.c:162, per CU). Waits for the stream."""
        cu = np.zeros(_lib.AQ_CU_SLOTS, np.uint64)
        n = self.L.aq_cu_task_counters(self._h, _up(cu), _lib.AQ_CU_SLOTS, 1 if reset else 0)
        if n < 0:
            _check(n, "aq_cu_task_counters")
        return {int(i): int(cu[i]) for i in np.nonzero(cu)[0]}

    # -- batch / libm ------------------------------------------------------------------------
    def integrate_batch(self, a, b, eps, integrand=COSH4, out=None):
        """(area, tasks, accepted) per integral. out: optional (area f64, tasks u64, accepted u64)
        contiguous arrays of n to write into (a caller that reuses them skips the first-touch page
        faults of three fresh arrays)."""
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        n = a.size
        if out is None:
            area = np.empty(n, np.float64)
            tasks = np.empty(n, np.uint64)
            acc = np.empty(n, np.uint64)
        else:
            area, tasks, acc = out
            for x, dt in ((area, np.float64), (tasks, np.uint64), (acc, np.uint64)):
                if x.dtype != dt or x.shape != (n,) or not x.flags.c_contiguous or not x.flags.writeable:
                    raise ValueError("out arrays must be writeable contiguous (f64, u64, u64) of the batch's size")
        _check(self.L.aq_integrate_batch(self._h, n, _dp(a), _dp(b), float(eps), integrand, _dp(area), _up(acc),
                                         _up(tasks)), "aq_integrate_batch")
        return area, tasks, acc

    def eval_cosh(self, x):
        x = np.ascontiguousarray(x, np.float64)
        out = np.empty_like(x)
        _check(self.L.aq_eval_cosh(self._h, x.size, _dp(x), _dp(out)), "aq_eval_cosh")
        return out

    def eval_integrand(self, x, integrand=COSH4):
        x = np.ascontiguousarray(x, np.float64)
        out = np.empty_like(x)
        _check(self.L.aq_eval_integrand(self._h, integrand, x.size, _dp(x), _dp(out)), "aq_eval_integrand")
        return out


class Group:
    """GPUs that combine one integral's shards over RCCL (aq_group): one process driving several
    contexts (Group([ctx0, ctx1, ...])), or one process per GPU (Group.join(ctx, nranks, rank, uid)
    with uid = Group.unique_id() from rank 0, broadcast by the caller)."""

    def __init__(self, contexts=None, _handle=None):
        self.L = _lib.load()
        self._h = ctypes.c_void_p()
        self.contexts = list(contexts or [])
        if _handle is not None:
            self._h = _handle
        else:
            arr = (ctypes.c_void_p * len(self.contexts))(*[c._h.value for c in self.contexts])
            _check(self.L.aq_group_create(arr, len(self.contexts), ctypes.byref(self._h)), "aq_group_create")

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(_lib.AQ_GROUP_ID_BYTES)
        _check(_lib.load().aq_group_unique_id(buf), "aq_group_unique_id")
        return buf.raw

    @classmethod
    def join(cls, ctx, nranks: int, rank: int, uid: bytes):
        L = _lib.load()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), _lib.AQ_GROUP_ID_BYTES)
        _check(L.aq_group_join(ctx._h, int(nranks), int(rank), buf, ctypes.byref(h)), "aq_group_join")
        return cls([ctx], _handle=h)

    @property
    def size(self) -> int:
        return self.L.aq_group_size(self._h)

    def integrate(self, problem: "Problem") -> Result:
        n = self.size
        ncu = self.contexts[0].num_cus
        per_gpu = np.zeros(n, np.uint64)
        per_cu = np.zeros(n * ncu, np.uint64)
        r = _lib.aq_result()
        r.tasks_per_gpu = _up(per_gpu)
        r.tasks_per_cu = _up(per_cu)
        _check(self.L.aq_integrate_group(self._h, ctypes.byref(problem.c()), ctypes.byref(r)), "aq_integrate_group")
        out = Result(r.area, int(r.tasks), int(r.accepted), int(r.levels), int(r.n_cu), int(r.spilled))
        out.tasks_per_gpu = [int(v) for v in per_gpu]
        out.tasks_per_cu = {(g, k): int(per_cu[g * ncu + k]) for g in range(n) for k in range(ncu) if per_cu[g * ncu + k]}
        t = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
        lv = np.zeros(_lib.AQ_MAX_LEVELS, np.uint64)
        self.L.aq_level_histogram(self.contexts[0]._h, _up(t), _up(lv), _lib.AQ_MAX_LEVELS)
        out.tasks_per_level = [int(v) for v in t[:out.levels]]
        out.leaves_per_level = [int(v) for v in lv[:out.levels]]
        return out

    def close(self):
        if self._h:
            self.L.aq_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def integrate(integrand="cosh4", a=DEFAULT_A, b=DEFAULT_B, eps=DEFAULT_EPSILON, device=0, ctx=None) -> Result:
    p = Problem(INTEGRANDS[integrand] if isinstance(integrand, str) else integrand, a, b, eps)
    if ctx is not None:
        return ctx.integrate(p)
    with Context(device) as c:
        return c.integrate(p)


def group_tasks(tasks_per_cu: Dict[int, int], workers: int) -> List[int]:
    """Map per-CU counters onto `workers` worker slots (CU k -> worker k mod workers, CUs in slot order)."""
    out = [0] * workers
    for k, slot in enumerate(sorted(tasks_per_cu)):
        out[k % workers] += tasks_per_cu[slot]
    return out


def farmer(numprocs: int, problem: Optional[Problem] = None, ctx: Optional[Context] = None):
    """Mirror of `double farmer(int numprocs)` + main()'s guard (aquadPartA.c:86-90, :125-173).

    Returns (area, tasks_per_process) where tasks_per_process[0] is the farmer's 0 and entries
    1..numprocs-1 are the on-device workers' task counts (the GPU's CUs grouped into numprocs-1 workers).
    """
    if numprocs < 2:
        raise AquadError(ERR_NUMPROCS)
    problem = problem or Problem()
    own = ctx is None
    ctx = ctx or Context(0)
    try:
        r = ctx.integrate(problem)
    finally:
        if own:
            ctx.close()
    return r.area, [0] + group_tasks(r.tasks_per_cu, numprocs - 1)


def format_reference(area: float, tasks_per_process: List[int]) -> str:
    """Exactly main()'s stdout (aquadPartA.c:107-117)."""
    n = len(tasks_per_process)
    s = "Area=%f\n" % area
    s += "\nTasks Per Process\n"
    s += "".join("%d\t" % i for i in range(n)) + "\n"
    s += "".join("%d\t" % t for t in tasks_per_process) + "\n"
    return s
