"""ctypes loader for libaquad.so (the C ABI declared in include/aquad.h).

There is no CPU fallback: if the HIP extension cannot be loaded, every entry point raises.
The library is built in-tree (ppls_amd/_build/) so the GPU box loads exactly the file built here.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AQ_LIB") or os.path.join(HERE, "_build", "libaquad.so")

# Every symbol include/aquad.h declares (tests check the library exports all of them).
EXPORTS = (
    "aq_device_count", "aq_ctx_create", "aq_ctx_destroy", "aq_strerror", "aq_ctx_num_cus", "aq_ctx_num_workers",
    "aq_ctx_device_bytes", "aq_set_level_histograms", "aq_set_stall_timeout", "aq_user_integrand_name",
    "aq_integrate", "aq_integrate_shard", "aq_integrate_shard_exact", "aq_async_slots", "aq_integrate_async", "aq_fetch", "aq_fetch_exact",
    "aq_exact_round", "aq_max_integrals_per_launch", "aq_integrate_many_async", "aq_integrate_mixed_async",
    "aq_synchronize", "aq_gather_results", "aq_gather_exact", "aq_integrate_levels", "aq_level_histogram",
    "aq_tasks_per_cu", "aq_cu_task_counters", "aq_integrate_batch", "aq_eval_integrand", "aq_eval_cosh", "aq_kernel_timing",
    "aq_kernel_time", "aq_set_diagnostics", "aq_diagnostics", "aq_frontier_root", "aq_level_step", "aq_level_step_chained", "aq_level_narrow", "aq_level_defer_fold", "aq_frontier_integrate",
    "aq_group_create", "aq_group_unique_id", "aq_group_join", "aq_group_destroy", "aq_group_size",
    "aq_integrate_group", "aq_print_reference", "aq_print_reference_procs",
)

AQ_MAX_LEVELS = 128
AQ_CU_SLOTS = 2048
AQ_XS_LIMBS = 68
AQ_EXACT_ROW = AQ_XS_LIMBS + 4
AQ_GROUP_ID_BYTES = 128


class aq_problem(ctypes.Structure):
    _fields_ = [("integrand", ctypes.c_int32), ("max_depth", ctypes.c_int32), ("a", ctypes.c_double),
                ("b", ctypes.c_double), ("eps", ctypes.c_double), ("n_gpus", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class aq_result(ctypes.Structure):
    _fields_ = [("area", ctypes.c_double), ("tasks", ctypes.c_uint64), ("accepted", ctypes.c_uint64),
                ("levels", ctypes.c_uint32), ("n_cu", ctypes.c_uint32), ("spilled", ctypes.c_uint64),
                ("n_gpus", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("tasks_per_gpu", ctypes.POINTER(ctypes.c_uint64)), ("tasks_per_cu", ctypes.POINTER(ctypes.c_uint64))]


_lib = None


def load(build_if_missing=True):
    """Load libaquad.so (building it with hipcc if absent). Raises OSError if that is impossible."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH) and build_if_missing:
        from . import build as _build
        _build.build()
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    dp = ctypes.POINTER(ctypes.c_double)
    up = ctypes.POINTER(ctypes.c_uint64)
    P = ctypes.POINTER(aq_problem)
    R = ctypes.POINTER(aq_result)
    ip = ctypes.POINTER(ctypes.c_int32)
    lp = ctypes.POINTER(ctypes.c_int64)
    c_int, c_dbl = ctypes.c_int, ctypes.c_double
    sig = {
        "aq_device_count": ([ctypes.POINTER(c_int)], c_int),
        "aq_ctx_create": ([c_int, ctypes.POINTER(vp)], c_int),
        "aq_ctx_destroy": ([vp], None),
        "aq_strerror": ([c_int], ctypes.c_char_p),
        "aq_ctx_num_cus": ([vp], c_int),
        "aq_ctx_num_workers": ([vp], c_int),
        "aq_ctx_device_bytes": ([vp, up], c_int),
        "aq_set_level_histograms": ([vp, c_int], c_int),
        "aq_set_stall_timeout": ([vp, c_dbl], c_int),
        "aq_user_integrand_name": ([], ctypes.c_char_p),
        "aq_integrate": ([vp, P, R], c_int),
        "aq_integrate_shard": ([vp, P, c_int, c_int, R], c_int),
        "aq_integrate_shard_exact": ([vp, P, c_int, c_int, lp], c_int),
        "aq_async_slots": ([], c_int),
        "aq_integrate_async": ([vp, P, c_int, c_int, c_int], c_int),
        "aq_fetch": ([vp, c_int, R], c_int),
        "aq_fetch_exact": ([vp, c_int, lp], c_int),
        "aq_exact_round": ([lp], c_dbl),
        "aq_max_integrals_per_launch": ([], c_int),
        "aq_integrate_many_async": ([vp, c_int, c_int, dp, dp, c_dbl, c_int, c_int, c_int, c_int], c_int),
        "aq_integrate_mixed_async": ([vp, c_int, c_int, dp, dp, ip, c_int, c_dbl, c_int, c_int], c_int),
        "aq_synchronize": ([vp], c_int),
        "aq_gather_results": ([vp, c_int, c_int, vp], c_int),
        "aq_gather_exact": ([vp, c_int, c_int, vp], c_int),
        "aq_integrate_levels": ([vp, P, R, up, up, c_int], c_int),
        "aq_level_histogram": ([vp, up, up, c_int], c_int),
        "aq_cu_task_counters": ([vp, up, c_int, c_int], c_int),
        "aq_level_defer_fold": ([vp, c_int], c_int),
        "aq_frontier_integrate": ([vp, P, ctypes.c_uint32, c_int, R, up, up, c_int], c_int),
        "aq_level_narrow": ([vp, c_int, vp, vp, ctypes.c_uint32, vp, c_int, c_int, c_dbl, c_int, vp], c_int),
        "aq_tasks_per_cu": ([vp, up, c_int], c_int),
        "aq_integrate_batch": ([vp, ctypes.c_size_t, dp, dp, c_dbl, c_int, dp, up, up], c_int),
        "aq_eval_integrand": ([vp, c_int, ctypes.c_size_t, dp, dp], c_int),
        "aq_eval_cosh": ([vp, ctypes.c_size_t, dp, dp], c_int),
        "aq_kernel_timing": ([vp, c_int], c_int),
        "aq_kernel_time": ([vp, dp, up], c_int),
        "aq_set_diagnostics": ([vp, c_int], c_int),
        "aq_diagnostics": ([vp, up, c_int], c_int),
        "aq_print_reference": ([vp, R], None),
        "aq_print_reference_procs": ([vp, c_dbl, up, c_int], None),
        "aq_frontier_root": ([vp, c_int, c_dbl, c_dbl, vp], c_int),
        "aq_level_step": ([vp, c_int, vp, ctypes.c_uint32, vp, ctypes.c_uint32, c_dbl, c_int, c_int, vp, vp], c_int),
        "aq_level_step_chained": ([vp, c_int, vp, vp, ctypes.c_uint32, vp, ctypes.c_uint32, c_dbl, c_int, c_int, vp, vp],
                                  c_int),
        "aq_group_create": ([ctypes.POINTER(vp), c_int, ctypes.POINTER(vp)], c_int),
        "aq_group_unique_id": ([vp], c_int),
        "aq_group_join": ([vp, c_int, c_int, vp, ctypes.POINTER(vp)], c_int),
        "aq_group_destroy": ([vp], None),
        "aq_group_size": ([vp], c_int),
        "aq_integrate_group": ([vp, P, R], c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L
