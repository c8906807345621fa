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
    "aq_set_level_histograms", "aq_set_engine",
    "aq_integrate", "aq_integrate_shard", "aq_async_slots", "aq_integrate_async", "aq_fetch",
    "aq_max_integrals_per_launch", "aq_integrate_many_async",
    "aq_synchronize", "aq_gather_results", "aq_integrate_levels", "aq_level_histogram", "aq_tasks_per_cu",
    "aq_integrate_batch", "aq_eval_integrand", "aq_eval_cosh", "aq_kernel_timing", "aq_kernel_time",
    "aq_set_diagnostics", "aq_diagnostics", "aq_frontier_root", "aq_level_step",
    "aq_print_reference",
)

AQ_MAX_LEVELS = 128
AQ_CU_SLOTS = 2048


class aq_problem(ctypes.Structure):
    _fields_ = [("integrand", ctypes.c_int32), ("max_depth", ctypes.c_int32), ("a", ctypes.c_double),
                ("b", ctypes.c_double), ("eps", ctypes.c_double)]


class aq_result(ctypes.Structure):
    _fields_ = [("area", ctypes.c_double), ("tasks", ctypes.c_uint64), ("accepted", ctypes.c_uint64),
                ("levels", ctypes.c_uint32), ("n_cu", ctypes.c_uint32), ("spilled", ctypes.c_uint64)]


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
    sig = {
        "aq_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "aq_ctx_create": ([ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "aq_ctx_destroy": ([vp], None),
        "aq_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "aq_ctx_num_cus": ([vp], ctypes.c_int),
        "aq_ctx_num_workers": ([vp], ctypes.c_int),
        "aq_set_level_histograms": ([vp, ctypes.c_int], ctypes.c_int),
        "aq_set_engine": ([vp, ctypes.c_int], ctypes.c_int),
        "aq_integrate": ([vp, P, R], ctypes.c_int),
        "aq_integrate_shard": ([vp, P, ctypes.c_int, ctypes.c_int, R], ctypes.c_int),
        "aq_async_slots": ([], ctypes.c_int),
        "aq_integrate_async": ([vp, P, ctypes.c_int, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "aq_fetch": ([vp, ctypes.c_int, R], ctypes.c_int),
        "aq_max_integrals_per_launch": ([], ctypes.c_int),
        "aq_integrate_many_async": ([vp, ctypes.c_int, ctypes.c_int, dp, dp, ctypes.c_double, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "aq_synchronize": ([vp], ctypes.c_int),
        "aq_gather_results": ([vp, ctypes.c_int, ctypes.c_int, vp], ctypes.c_int),
        "aq_integrate_levels": ([vp, P, R, up, up, ctypes.c_int], ctypes.c_int),
        "aq_level_histogram": ([vp, up, up, ctypes.c_int], ctypes.c_int),
        "aq_tasks_per_cu": ([vp, up, ctypes.c_int], ctypes.c_int),
        "aq_integrate_batch": ([vp, ctypes.c_int, ctypes.c_size_t, dp, dp, ctypes.c_double, dp, up, up], ctypes.c_int),
        "aq_eval_integrand": ([vp, ctypes.c_int, ctypes.c_size_t, dp, dp], ctypes.c_int),
        "aq_eval_cosh": ([vp, ctypes.c_size_t, dp, dp], ctypes.c_int),
        "aq_kernel_timing": ([vp, ctypes.c_int], ctypes.c_int),
        "aq_kernel_time": ([vp, dp, up], ctypes.c_int),
        "aq_set_diagnostics": ([vp, ctypes.c_int], ctypes.c_int),
        "aq_diagnostics": ([vp, up, ctypes.c_int], ctypes.c_int),
        "aq_print_reference": ([vp, ctypes.c_double, up, ctypes.c_int], None),
        "aq_frontier_root": ([vp, ctypes.c_int, ctypes.c_double, ctypes.c_double, vp], ctypes.c_int),
        "aq_level_step": ([vp, ctypes.c_int, vp, ctypes.c_uint32, vp, ctypes.c_uint32, ctypes.c_double, ctypes.c_int,
                           ctypes.c_int, vp, vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L
