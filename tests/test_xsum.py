"""The exact area accumulator (ppls_amd/csrc/aq_xsum.h) on the CPU: the header the kernels use is
compiled with g++ into a tiny shared library and checked against Python's math.fsum, which returns
the correctly rounded sum of its inputs -- the property the device gathers rely on (the per-integral
area is the correctly rounded sum of the waves' partials, whatever order they were added in)."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SRC = r"""
#include <algorithm>
#include "aq_xsum.h"
extern "C" double xs_sum(const double* x, long n) {
    aq::XSum a;
    memset(&a, 0, sizeof(a));
    for (long i = 0; i < n; ++i) aq::xs_add(a, x[i]);
    return aq::xs_round(a);
}
// split the inputs over k accumulators, then add the accumulators limb-wise (the collective path)
extern "C" double xs_sum_split(const double* x, long n, int k) {
    aq::XSum acc[16];
    memset(acc, 0, sizeof(acc));
    for (long i = 0; i < n; ++i) aq::xs_add(acc[i % k], x[i]);
    for (int j = 1; j < k; ++j) aq::xs_add_xs(acc[0], acc[j]);
    return aq::xs_round(acc[0]);
}
// the batch gather's path (aquad.hip k_gather_reset): only the limb window the adds touched
// (SlotSums win_lo_not / win_hi, folded by max), rounded with xs_round_span<16> when it spans <= 16
// limbs; -1 in *used when the window was too wide (the full xs_round path)
extern "C" double xs_sum_window(const double* x, long n, int* used) {
    aq::XSum a;
    memset(&a, 0, sizeof(a));
    unsigned lo_not = 0, hi = 0;
    for (long i = 0; i < n; ++i) {
        aq::XDigits g;
        if (!aq::xs_digits(x[i], g)) continue;
        aq::xs_add(a, x[i]);
        lo_not = std::max(lo_not, aq::xs_win_lo(g.i));
        hi = std::max(hi, aq::xs_win_hi(g.i));
    }
    const int l = hi ? (int)~lo_not : 0, h = hi ? (int)hi : 0;
    if (h - l > 16) { *used = -1; return aq::xs_round(a); }
    *used = h - l;
    for (int i = 0; i < aq::XS_LIMBS; ++i)
        if ((i < l || i >= h) && a.limb[i] != 0) return -12345.0;   // a nonzero limb outside the window
    return aq::xs_round_span<16>(a.limb + l, h - l, aq::XS_E0 + 32 * l);
}
"""


@pytest.fixture(scope="module")
def xs(tmp_path_factory):
    d = tmp_path_factory.mktemp("xsum")
    src = d / "xs.cpp"
    src.write_text(SRC)
    so = d / "libxs.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                           "-I", os.path.join(ROOT, "ppls_amd", "csrc"), "-o", str(so), str(src)])
    L = ctypes.CDLL(str(so))
    dp = ctypes.POINTER(ctypes.c_double)
    L.xs_sum.argtypes = [dp, ctypes.c_long]
    L.xs_sum.restype = ctypes.c_double
    L.xs_sum_split.argtypes = [dp, ctypes.c_long, ctypes.c_int]
    L.xs_sum_split.restype = ctypes.c_double

    L.xs_sum_window.argtypes = [dp, ctypes.c_long, ctypes.POINTER(ctypes.c_int)]
    L.xs_sum_window.restype = ctypes.c_double

    def run(x, k=1):
        x = np.ascontiguousarray(x, np.float64)
        p = x.ctypes.data_as(dp)
        if k == "window":
            used = ctypes.c_int(0)
            return L.xs_sum_window(p, x.size, ctypes.byref(used)), used.value
        return L.xs_sum(p, x.size) if k == 1 else L.xs_sum_split(p, x.size, k)
    return run


def same(a, b):
    return np.float64(a).view(np.uint64) == np.float64(b).view(np.uint64)


def test_simple(xs):
    assert xs([]) == 0.0
    assert xs([1.0, 2.0]) == 3.0
    assert xs([1e308, 1e308, -1e308]) == 1e308          # exact intermediate beyond double range
    assert xs([1.0, 1e-300, -1.0]) == 1e-300
    assert xs([5e-324, 5e-324]) == 1e-323               # subnormals
    assert xs([0.1] * 10) == math.fsum([0.1] * 10)
    assert xs([1.7976931348623157e308, 1.7976931348623157e308]) == float("inf")


@pytest.mark.parametrize("seed", range(6))
def test_random_matches_fsum(xs, seed):
    rng = np.random.default_rng(seed)
    n = 5000
    kind = seed % 3
    if kind == 0:    # the quadrature's case: many positive areas of mixed magnitude
        x = rng.uniform(0, 1, n) * 10.0 ** rng.integers(-12, 5, n)
    elif kind == 1:  # cancellation, both signs, wide exponents
        x = rng.standard_normal(n) * 2.0 ** rng.integers(-1000, 1000, n)
    else:            # ties and near-ties: halves of ulps
        base = rng.uniform(1, 2, n)
        x = np.concatenate([base, -base[:-1], [2.0 ** -53, 2.0 ** -105, 2.0 ** -106]])
    want = math.fsum(x.tolist())
    assert same(xs(x), want)
    assert same(xs(x, 7), want)                          # any partition, limb-wise combine
    assert same(xs(x[::-1]), want)                       # any order


def test_subnormal_results(xs):
    rng = np.random.default_rng(99)
    x = rng.integers(-2 ** 40, 2 ** 40, 200) * 5e-324
    x = np.concatenate([x, [2.0 ** -1022, -2.0 ** -1022 + 5e-324]])
    assert same(xs(x), math.fsum(x.tolist()))


@pytest.mark.parametrize("seed", range(6))
def test_window_rounding_matches_fsum(xs, seed):
    """The batch gather rounds only a slot's limb window (r05): the same correctly rounded sum, on
    quadrature-like partials (a narrow window: the short path) and on wide or cancelling ones (the
    full-accumulator fallback above 16 limbs)."""
    rng = np.random.default_rng(100 + seed)
    n = 4000
    if seed % 3 == 0:    # double-double partials of one integral: hi ~ 1e5, lo ~ 1e-12 of it
        hi = rng.uniform(1e4, 1e6, n)
        x = np.concatenate([hi, hi * rng.uniform(-1e-16, 1e-16, n)])
    elif seed % 3 == 1:  # ties and cancellation inside a narrow range
        base = rng.uniform(1, 2, n)
        x = np.concatenate([base, -base[:-1], [2.0 ** -53, 2.0 ** -60]])
    else:                # exponents across the whole range: the fallback
        x = rng.standard_normal(n) * 2.0 ** rng.integers(-1000, 1000, n)
    got, used = xs(x, "window")
    assert same(got, math.fsum(x.tolist()))
    assert (used == -1) if seed % 3 == 2 else (0 < used <= 16)
    assert xs(np.zeros(3), "window") == (0.0, 0)
