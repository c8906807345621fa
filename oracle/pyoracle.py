"""ctypes binding of the CPU oracle (oracle/aq_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker (or the timed CPU baseline). The product package ppls_amd never imports this.
"""
import ctypes
import os
import subprocess
from dataclasses import dataclass, field
from typing import List

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")

COSH4 = 0
SIN_RECIP = 1
USER = 2        # exp(-x*x): the library's default AQ_F_USER plug-in

RESTATED_FMA = 0
RESTATED_NOFMA = 1
HOST_LIBM = 2


class _Res(ctypes.Structure):
    _fields_ = [
        ("area_lifo", ctypes.c_double),
        ("area_quad_hi", ctypes.c_double),
        ("area_quad_lo", ctypes.c_double),
        ("tasks", ctypes.c_uint64),
        ("leaves", ctypes.c_uint64),
        ("levels", ctypes.c_int32),
        ("pad", ctypes.c_int32),
    ]


@dataclass
class OracleResult:
    area_lifo: float
    area_quad_hi: float
    area_quad_lo: float
    area_quad_str: str
    tasks: int
    leaves: int
    levels: int
    tasks_per_level: List[int] = field(default_factory=list)
    leaves_per_level: List[int] = field(default_factory=list)

    @property
    def area(self) -> float:
        return self.area_quad_hi + self.area_quad_lo


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "_build/liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        up = ctypes.POINTER(ctypes.c_uint64)
        L.aqo_integrate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_int, ctypes.POINTER(_Res), up, up]
        L.aqo_integrate.restype = ctypes.c_int
        for name in ("aqo_cosh_array", "aqo_exp_array", "aqo_expm1_array", "aqo_sin_array"):
            getattr(L, name).argtypes = [ctypes.c_int, ctypes.c_long, dp, dp]
            getattr(L, name).restype = None
        L.aqo_integrate_shard.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(_Res), up, up]
        L.aqo_integrate_shard.restype = ctypes.c_int
        L.aqo_F_array.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, dp, dp]
        L.aqo_F_array.restype = None
        L.aqo_F.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.aqo_F.restype = ctypes.c_double
        L.aqo_quad_to_string.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
        L.aqo_batch_bounds.argtypes = [ctypes.c_long, dp, dp]
        L.aqo_batch_bounds.restype = None
        L.aqo_integrate_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, dp, dp,
                                          ctypes.c_double, ctypes.c_int, dp, up, up]
        L.aqo_integrate_batch.restype = ctypes.c_int
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _up(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def integrate(integrand=COSH4, a=0.0, b=5.0, eps=1e-3, mode=RESTATED_FMA, maxlev=256) -> OracleResult:
    L = lib()
    r = _Res()
    tpl = np.zeros(maxlev, np.uint64)
    lpl = np.zeros(maxlev, np.uint64)
    rc = L.aqo_integrate(integrand, mode, a, b, eps, maxlev, ctypes.byref(r), _up(tpl), _up(lpl))
    if rc != 0:
        raise RuntimeError(f"oracle aqo_integrate failed rc={rc}")
    buf = ctypes.create_string_buffer(64)
    L.aqo_quad_to_string(r.area_quad_hi, r.area_quad_lo, buf, 64)
    n = r.levels
    return OracleResult(r.area_lifo, r.area_quad_hi, r.area_quad_lo, buf.value.decode(), r.tasks, r.leaves,
                        r.levels, [int(v) for v in tpl[:n]], [int(v) for v in lpl[:n]])


def integrate_shard(shard, nshards, G=256, S=5, integrand=COSH4, a=0.0, b=5.0, eps=1e-3, mode=RESTATED_FMA,
                    maxlev=256) -> OracleResult:
    """Shard `shard` of `nshards` in the device's partition (G workgroups per GPU, 2^S seeds each)."""
    L = lib()
    r = _Res()
    tpl = np.zeros(maxlev, np.uint64)
    lpl = np.zeros(maxlev, np.uint64)
    rc = L.aqo_integrate_shard(integrand, mode, a, b, eps, maxlev, G, S, shard, nshards, ctypes.byref(r), _up(tpl),
                               _up(lpl))
    if rc != 0:
        raise RuntimeError(f"oracle aqo_integrate_shard failed rc={rc}")
    buf = ctypes.create_string_buffer(64)
    L.aqo_quad_to_string(r.area_quad_hi, r.area_quad_lo, buf, 64)
    n = r.levels
    return OracleResult(r.area_lifo, r.area_quad_hi, r.area_quad_lo, buf.value.decode(), r.tasks, r.leaves,
                        r.levels, [int(v) for v in tpl[:n]], [int(v) for v in lpl[:n]])


def cosh(x, mode=RESTATED_FMA):
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    lib().aqo_cosh_array(mode, x.size, _dp(x), _dp(out))
    return out


def exp(x, mode=RESTATED_FMA):
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    lib().aqo_exp_array(mode, x.size, _dp(x), _dp(out))
    return out


def expm1(x, mode=RESTATED_FMA):
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    lib().aqo_expm1_array(mode, x.size, _dp(x), _dp(out))
    return out


def sin(x, mode=RESTATED_FMA):
    """glibc 2.35 sin restated (aq_oracle.c aqo_sin), or the host libm's with HOST_LIBM."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    lib().aqo_sin_array(mode, x.size, _dp(x), _dp(out))
    return out


def F(x, integrand=COSH4, mode=RESTATED_FMA):
    """F at a scalar (returns float) or an array (returns an array), restated glibc (aq_oracle.c)."""
    if np.ndim(x) == 0:
        return lib().aqo_F(integrand, mode, float(x))
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    lib().aqo_F_array(integrand, mode, x.size, _dp(x), _dp(out))
    return out


def batch_bounds(n):
    a = np.empty(n, np.float64)
    b = np.empty(n, np.float64)
    lib().aqo_batch_bounds(n, _dp(a), _dp(b))
    return a, b


def integrate_batch(a, b, eps, integrand=COSH4, mode=RESTATED_FMA, maxlev=256):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    n = a.size
    area = np.empty(n, np.float64)
    tasks = np.empty(n, np.uint64)
    leaves = np.empty(n, np.uint64)
    rc = lib().aqo_integrate_batch(integrand, mode, n, _dp(a), _dp(b), eps, maxlev, _dp(area), _up(tasks), _up(leaves))
    if rc != 0:
        raise RuntimeError(f"oracle aqo_integrate_batch failed rc={rc}")
    return area, tasks, leaves


def level_step(fin, eps, depth, max_depth, integrand=COSH4, mode=RESTATED_FMA):
    """CPU restatement of one frontier level (the HIP aq_level_step; aquadPartA.c:183-202 applied
    to every record {l, r, F(l), F(r)} of fin, shape (n, 4)). Returns (children (m, 4), leaf areas,
    tasks, error bits): refining records emit [l, mid] and [mid, r] (:192-197)."""
    fin = np.asarray(fin, np.float64).reshape(-1, 4)
    l, r, fl, fr = fin[:, 0], fin[:, 1], fin[:, 2], fin[:, 3]
    mid = (l + r) / 2                                   # :187
    fmid = F(mid, integrand, mode)                      # :188
    lrarea = (fl + fr) * (r - l) / 2                    # :185
    larea = (fl + fmid) * (mid - l) / 2                 # :189
    rarea = (fmid + fr) * (r - mid) / 2                 # :190
    ref = np.abs((larea + rarea) - lrarea) > eps        # :191
    err = 0
    if depth + 1 >= max_depth and ref.any():
        err |= 4
        ref = np.zeros_like(ref)
        leaf = np.abs((larea + rarea) - lrarea) <= eps
    else:
        leaf = ~ref
    kids = np.empty((2 * int(ref.sum()), 4), np.float64)
    kids[0::2] = np.stack([l[ref], mid[ref], fl[ref], fmid[ref]], axis=1)
    kids[1::2] = np.stack([mid[ref], r[ref], fmid[ref], fr[ref]], axis=1)
    return kids, (larea + rarea)[leaf], fin.shape[0], err


class FrontierStepper:
    """Test-only stepper for ppls_amd.frontier on CPU torch tensors (gloo), backed by level_step."""

    def __init__(self, integrand=COSH4, mode=RESTATED_FMA):
        import torch
        self.device = torch.device("cpu")
        self.mode = mode

    def root(self, integrand, a, b, out):
        out[0, 0] = a
        out[0, 1] = b
        out[0, 2] = F(float(a), integrand, self.mode)
        out[0, 3] = F(float(b), integrand, self.mode)

    def step(self, integrand, fin, n_in, fout, cap, eps, depth, max_depth, nout, acc):
        kids, leaves, tasks, err = level_step(fin[:n_in].numpy(), eps, depth, max_depth, integrand, self.mode)
        if kids.shape[0] > cap:
            err |= 2
            kids = kids[:cap]
        fout[:kids.shape[0]] = __import__("torch").from_numpy(kids)
        nout[0] = kids.shape[0]
        hi, lo = float(acc[0]), float(acc[1])
        for v in leaves.tolist():
            s = hi + v
            bb = s - hi
            lo += (hi - (s - bb)) + (v - bb)
            hi = s
        acc[0], acc[1] = hi, lo
        acc[2] += tasks
        acc[3] += leaves.size
        acc[4] = float(int(acc[4]) | err)
        if tasks:
            acc[5] = max(float(acc[5]), depth + 1)

    def sync(self):
        pass
