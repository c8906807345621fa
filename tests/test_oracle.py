"""The CPU oracle (oracle/aq_oracle.c) against the reference's golden vectors.

Pins: (1) the reference's header known answer (aquadPartA.c:31-36: Area=7583461.801486, 6567
tasks); (2) stdout of the reference binary compiled from /root/reference by oracle/Makefile
(recorded in tests/golden/trees.json by tests/golden/make_golden.py); (3) host glibc 2.35 libm
bit patterns (tests/golden/libm_bits.npz).
"""
import os
import platform
import re

import numpy as np
import pytest

from conftest import ROOT


def test_header_known_answer(oracle):
    # aquadPartA.c:31-36: mpirun -c 5 -> Area=7583461.801486, tasks 0 1679 1605 1682 1601 (sum 6567)
    r = oracle.integrate(eps=1e-3)
    assert "%f" % r.area == "7583461.801486"
    assert "%f" % r.area_lifo == "7583461.801486"
    assert r.tasks == 1679 + 1605 + 1682 + 1601
    assert r.leaves == (r.tasks + 1) // 2


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "cosh4_eps1e-6", "cosh4_eps1e-8", "cosh4_eps1e-10",
                                  "sin_recip_eps1e-9", "cosh4_eps1e3_root_leaf", "cosh4_empty_interval",
                                  "cosh4_neg_domain"])
def test_oracle_tree_fixture(oracle, trees, name):
    g = trees[name]
    f = oracle.COSH4 if g["integrand"] == "cosh4" else oracle.SIN_RECIP
    r = oracle.integrate(f, g["a"], g["b"], g["eps"])
    assert r.tasks == g["tasks"] and r.leaves == g["leaves"] and r.levels == g["levels"]
    assert r.tasks_per_level == g["tasks_per_level"]
    assert r.leaves_per_level == g["leaves_per_level"]
    assert r.area_quad_str == g["area_quad"]
    assert float(r.area_lifo).hex() == g["area_lifo_hex"]


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "cosh4_eps1e-10", "cosh4_eps1e-12", "sin_recip_eps1e-9"])
def test_fixture_matches_reference_stdout(trees, name):
    """The restatement's numbers are the reference binary's own output (recorded verbatim)."""
    g = trees[name]
    ref = g["reference"]
    assert ref["tasks_total"] == g["tasks"]
    assert ref["tasks_per_process"][0] == 0
    assert ref["area_printed"] == "%f" % float.fromhex(g["area_lifo_hex"]) or ref["area_printed"] == \
        "%f" % float(g["area_quad"])
    assert "%f" % float(g["area_quad"]) == ref["area_printed"]
    p2 = g["reference_p2"]
    assert p2["area_printed"] == g["area_lifo_printed"]  # one worker = LIFO order exactly
    assert p2["tasks_per_process"] == [0, g["tasks"]]


def test_fixture_histogram_consistency(trees):
    for name, g in trees.items():
        assert sum(g["tasks_per_level"]) == g["tasks"], name
        assert sum(g["leaves_per_level"]) == g["leaves"], name
        if g["tasks"]:
            assert g["tasks"] == 2 * g["leaves"] - 1, name
        # a level's tasks are the previous level's refined tasks times two
        for d in range(1, len(g["tasks_per_level"])):
            assert g["tasks_per_level"][d] == 2 * (g["tasks_per_level"][d - 1] - g["leaves_per_level"][d - 1])


def test_oracle_cosh_bits_fixture(oracle, libm_bits):
    x = libm_bits["x"].view(np.float64)
    got = oracle.cosh(x).view(np.uint64)
    assert np.array_equal(got, libm_bits["cosh"])
    ex = libm_bits["exp_x"].view(np.float64)
    assert np.array_equal(oracle.exp(ex).view(np.uint64), libm_bits["exp"])


def _host_is_glibc_235():
    try:
        return platform.libc_ver()[1] == "2.35"
    except Exception:
        return False


@pytest.mark.skipif(not _host_is_glibc_235(), reason="host libm is not glibc 2.35")
def test_oracle_vs_host_libm_random(oracle):
    rng = np.random.default_rng(7)
    x = rng.uniform(0.0, 5.0, 1_000_000)
    assert np.array_equal(oracle.cosh(x).view(np.uint64), oracle.cosh(x, oracle.HOST_LIBM).view(np.uint64))
    xs = rng.uniform(2.0 ** -54, 0.34657359027997264, 200_000)  # |x| < 0.5 ln2: cosh's expm1 range
    assert np.array_equal(oracle.expm1(xs).view(np.uint64), oracle.expm1(xs, oracle.HOST_LIBM).view(np.uint64))
    big = rng.uniform(0.35, 700.0, 200_000)
    assert np.array_equal(oracle.exp(big).view(np.uint64), oracle.exp(big, oracle.HOST_LIBM).view(np.uint64))


def test_oracle_sin_bits_fixture(oracle, sin_bits):
    """Config 4's F = sin(1.0/x) restated (glibc 2.35 s_sin.c, FMA form) against the committed host
    libm bits (tests/golden/sin_bits.npz)."""
    x = sin_bits["x"].view(np.float64)
    assert np.array_equal(oracle.F(x, oracle.SIN_RECIP).view(np.uint64), sin_bits["F"])


@pytest.mark.skipif(not _host_is_glibc_235(), reason="host libm is not glibc 2.35")
def test_oracle_sin_vs_host_libm_random(oracle):
    """Every s_sin.c range below 105414350 (the Taylor and table paths, the 0.855..2.426 cosine
    path, the Cody-Waite reduction), both signs, bit for bit against the host libm."""
    rng = np.random.default_rng(8)
    x = np.concatenate([1.0 / rng.uniform(1e-4, 1.0, 1_000_000), rng.uniform(-4.0, 4.0, 500_000),
                        rng.uniform(-1.05e8, 1.05e8, 300_000), rng.uniform(-0.2, 0.2, 100_000),
                        rng.uniform(-1e-7, 1e-7, 10_000)])
    assert np.array_equal(oracle.sin(x).view(np.uint64), oracle.sin(x, oracle.HOST_LIBM).view(np.uint64))


def test_sincos_tables_agree():
    """Oracle table (mpmath) == product table (decimal): two independent generators of glibc's
    __sincostab."""
    pat = r"-?0x[0-9a-f.]+p[-+]?\d+"
    a = [float.fromhex(v) for v in re.findall(pat, open(os.path.join(ROOT, "oracle", "glibc_sincos_table.h")).read())]
    b = [float.fromhex(v) for v in re.findall(pat, open(os.path.join(ROOT, "ppls_amd", "csrc", "aq_sincos_table.h")).read())]
    assert len(a) == 444 and a == b


def test_exp_tables_agree():
    """Oracle table (mpmath) == product table (decimal): two independent generators of glibc's data."""
    a = re.findall(r"0x[0-9a-f]{16}", open(os.path.join(ROOT, "oracle", "glibc_exp_table.h")).read())
    b = re.findall(r"0x[0-9a-f]{16}", open(os.path.join(ROOT, "ppls_amd", "csrc", "aq_exp_table.h")).read())
    assert len(a) == 256 and a == b


def test_shard_partition_sums_to_total(oracle):
    tot = oracle.integrate(eps=1e-8)
    for n in (1, 2, 3, 4, 8):
        parts = [oracle.integrate_shard(s, n, G=256, eps=1e-8) for s in range(n)]
        assert sum(p.tasks for p in parts) == tot.tasks
        assert sum(p.leaves for p in parts) == tot.leaves
        assert max(p.levels for p in parts) == tot.levels
        assert [sum(col) for col in zip(*[p.tasks_per_level + [0] * (tot.levels - p.levels) for p in parts])] == \
            tot.tasks_per_level
        assert abs(sum(p.area for p in parts) - tot.area) <= 1e-13 * tot.area


@pytest.mark.parametrize("G", [1, 7, 64, 304])
def test_shard_partition_any_grid(oracle, G):
    tot = oracle.integrate(oracle.SIN_RECIP, 1e-4, 1.0, 1e-6)
    parts = [oracle.integrate_shard(s, 2, G=G, integrand=oracle.SIN_RECIP, a=1e-4, b=1.0, eps=1e-6)
             for s in range(2)]
    assert sum(p.tasks for p in parts) == tot.tasks and sum(p.leaves for p in parts) == tot.leaves


def test_batch_bounds_and_kat(oracle, batch_golden):
    a, b = oracle.batch_bounds(10000)
    assert [[float(x).hex(), float(y).hex()] for x, y in zip(a[:16], b[:16])] == batch_golden["first_bounds_hex"]
    assert (a <= b).all() and (a >= 0).all() and (b < 5).all()
    ar, t, lv = oracle.integrate_batch(a[:256], b[:256], 1e-3)
    assert [int(v) for v in lv] == batch_golden["leaves_eps1e-3_first256"]
    assert [float(v).hex() for v in ar] == batch_golden["area_eps1e-3_first256_hex"]
    assert (t == 2 * lv - 1).all()
    # SURVEY §8d KAT: first 10 000 draws -> mean leaves 711.5 at eps=1e-3
    assert abs(batch_golden["mean_leaves_eps1e-3"] - 711.5) < 0.05


def test_oracle_deep_eps(oracle):
    # eps=1e-14 -> T=30 870 291, L=15 435 146, measured there by a
    # verbatim replay of the reference's task arithmetic (it reproduced every MPI total)
    r = oracle.integrate(eps=1e-14)
    assert (r.tasks, r.leaves) == (30870291, 15435146)


def test_plugin_fixture_pinned_by_reference(trees, plugin_bits):
    """The AQ_F_USER plug-in's fixtures: the reference binary built with `#define F(arg)
    exp(-(arg)*(arg))` printed the same task totals and Area= as the oracle's restatement."""
    from oracle import pyoracle as O
    for name in ["gauss_eps1e-10", "gauss_eps1e-13"]:
        g = trees[name]
        r = O.integrate(O.USER, g["a"], g["b"], g["eps"])
        assert (r.tasks, r.leaves, r.levels) == (g["tasks"], g["leaves"], g["levels"])
        assert g["reference"]["tasks_total"] == r.tasks == g["reference_p2"]["tasks_total"]
        assert g["reference"]["area_printed"] == "%f" % r.area
        assert g["reference_p2"]["area_printed"] == "%f" % r.area_lifo   # P=2: deterministic LIFO order
    x = plugin_bits["x"].view(np.float64)
    assert (O.F(x, O.USER).view(np.uint64) == plugin_bits["F"]).all()
    assert (O.F(x, O.USER, O.HOST_LIBM).view(np.uint64) == plugin_bits["F"]).all()


def test_exp_restatement_every_path_vs_host_libm():
    """glibc exp restated for every path the plug-in surface exposes: tiny arguments, the main
    range, |x| >= 512 with k > 0 and k < 0 (subnormal results), |x| >= 1024."""
    from oracle import pyoracle as O
    rng = np.random.default_rng(17)
    x = np.concatenate([rng.uniform(-745.2, -700, 100000), rng.uniform(-1100, -500, 50000),
                        rng.uniform(-30, 30, 100000), rng.uniform(-1e-15, 1e-15, 5000), rng.uniform(500, 709.7, 50000),
                        [0.0, -0.0, -708.39, -745.13, -745.14, -1024.0, -1e300, 2.0 ** -55, 5e-324, 709.78, 1e300]])
    assert (O.exp(x).view(np.uint64) == O.exp(x, O.HOST_LIBM).view(np.uint64)).all()


def test_deep_fixture_pinned_by_reference(deep_golden):
    """eps=1e-14 (31 M tasks): the oracle reproduces the reference binary's task total (deep.json)."""
    from oracle import pyoracle as O
    g = deep_golden["cosh4_eps1e-14"]
    r = O.integrate(eps=g["eps"], maxlev=128)
    assert r.tasks == g["tasks"] == g["reference"]["tasks_total"]
    assert (r.leaves, r.levels) == (g["leaves"], g["levels"])
    assert abs(float(g["reference"]["area_printed"]) - r.area) <= 5e-7 + 1e-12 * r.area


def test_device_seed_depth_rule():
    """tests' device_seed_S restates aq_stream.h seed_depth_job: one level deeper only where the
    seeding's 64-node fast path holds it (the bench's adaptive jobs, whole-integral jobs), never for a
    lone launch's 3072 shares or the sharded launches' 32 virtual workers."""
    from conftest import device_seed_S
    assert device_seed_S(3072, 1) == 2       # lone: 14 levels x 3 positions; deeper = 15 x 6 = 90 nodes
    assert device_seed_S(3072, 2) == 2
    assert device_seed_S(16, 2) == 2         # sharded multi-integral: V = 32, deeper = 9 x 8 = 72
    assert device_seed_S(24, 1) == 3         # adaptive jobs: 8 levels x 6 = 48 nodes
    assert device_seed_S(1, 1) == 3          # whole-integral jobs: 4 levels x 8 = 32 nodes
