"""GPU parity: the HIP engine (through the C ABI, include/aquad.h) against the oracle and the
reference's golden vectors. Bar: interval counts (tasks, accepted, per-level histograms) bit-exact;
area within 1e-12 relative of the quad-precision Σ of leaf areas (BASELINE.json north_star);
device cosh bit-identical to host glibc 2.35."""
import math
import os
import subprocess

import numpy as np
import pytest
from conftest import device_seed_S

pytestmark = pytest.mark.gpu

AREA_RTOL = 1e-12  # BASELINE.json north_star: "its area to a stated relative tolerance of 1e-12"

TREE_CASES = ["cosh4_eps1e-3", "cosh4_eps1e-6", "cosh4_eps1e-8", "cosh4_eps1e-10", "cosh4_eps1e-12",
              "sin_recip_eps1e-9", "cosh4_eps1e3_root_leaf", "cosh4_empty_interval", "cosh4_neg_domain",
              "gauss_eps1e-10", "gauss_eps1e-13"]


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


FIDS = {"cosh4": 0, "sin_recip": 1, "gauss": 2}


def _problem(g):
    from ppls_amd import Problem
    return Problem(FIDS[g["integrand"]], g["a"], g["b"], g["eps"])


def _area_ok(got, quad_str):
    want = float(quad_str)
    if want == 0.0:
        return got == 0.0
    return abs(got - want) <= AREA_RTOL * abs(want)


def test_native_library_is_loaded(ctx):
    from ppls_amd import _lib
    maps = open("/proc/self/maps").read()
    assert _lib.LIB_PATH in maps
    assert ctx.num_cus > 0


def test_device_cosh_bit_exact_fixture(ctx, libm_bits):
    x = libm_bits["x"].view(np.float64)
    got = ctx.eval_cosh(x).view(np.uint64)
    bad = np.nonzero(got != libm_bits["cosh"])[0]
    assert bad.size == 0, [(float(x[i]), hex(int(got[i])), hex(int(libm_bits['cosh'][i]))) for i in bad[:10]]


def test_device_cosh_bit_exact_random(ctx, oracle):
    rng = np.random.default_rng(11)
    x = np.concatenate([rng.uniform(0.0, 5.0, 2_000_000), rng.uniform(0.0, 0.35, 200_000),
                        rng.uniform(5.0, 30.0, 100_000), -rng.uniform(0.0, 5.0, 100_000)])
    got = ctx.eval_cosh(x).view(np.uint64)
    want = oracle.cosh(x).view(np.uint64)  # restated glibc (pinned to libm by test_oracle)
    assert int((got != want).sum()) == 0


def test_device_integrand_bit_exact(ctx, oracle):
    rng = np.random.default_rng(12)
    x = rng.uniform(0.0, 5.0, 500_000)
    want = np.array([oracle.F(v) for v in x[:20000]])
    got = ctx.eval_integrand(x[:20000])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_device_batched_integrand_bit_exact(ctx, oracle, libm_bits):
    """F through the persistent kernel's batched path (aq_eval_integrand: integrand_k, two points per
    lane, computed as 16 F from 2 cosh as the rounds do, /16 exact) against the restated glibc cosh^4, on the
    committed libm fixture points and 8 M random points: the main range, both sides of its ends, and
    lanes whose two points fall on different paths."""
    rng = np.random.default_rng(14)
    x = np.concatenate([libm_bits["x"].view(np.float64), rng.uniform(0.0, 5.0, 4_000_000),
                        rng.uniform(0.3, 0.4, 1_000_000), rng.uniform(21.5, 22.5, 1_000_000),
                        rng.uniform(-30.0, 30.0, 2_000_000)])
    c = oracle.cosh(x)
    want = ((c * c) * c) * c          # the reference macro's ((c*c)*c)*c (aquadPartA.c:46)
    got = ctx.eval_integrand(x)
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, [(float(x[i]), float(got[i]), float(want[i])) for i in bad[:10]]


def test_device_sin_recip_bit_exact(ctx, oracle, sin_bits):
    """Config 4's F = sin(1.0/x) on the device (aq_libm.h sin_glibc, glibc 2.35 s_sin.c restated)
    against the committed host-libm bits and against the restated oracle on 4 M points: every range
    of 1/x below 105414350, both signs. Beyond it (|x| < 9.5e-9) the device's faithful sin answers
    (glibc's __branred is not restated): within 1 ulp there."""
    xf = sin_bits["x"].view(np.float64)
    inside = np.abs(1.0 / xf) < 105414350.0
    got = ctx.eval_integrand(xf, integrand=1)
    bad = np.nonzero(inside & (got.view(np.uint64) != sin_bits["F"]))[0]
    assert bad.size == 0, [(float(xf[i]), float(got[i])) for i in bad[:10]]
    want = sin_bits["F"].view(np.float64)
    assert (np.abs(got.view(np.int64) - want.view(np.int64))[~inside] <= 1).all()
    rng = np.random.default_rng(13)
    x = np.concatenate([rng.uniform(1e-4, 1.0, 2_000_000), 1.0 / rng.uniform(-4.0, 4.0, 1_000_000),
                        np.exp(rng.uniform(np.log(9.5e-9), np.log(1e4), 1_000_000)) * rng.choice([-1.0, 1.0], 1_000_000)])
    got = ctx.eval_integrand(x, integrand=1)
    want = oracle.F(x, oracle.SIN_RECIP)
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, [(float(x[i]), float(got[i]), float(want[i])) for i in bad[:10]]


@pytest.mark.parametrize("name", TREE_CASES)
def test_persistent_tree_parity(ctx, trees, name):
    g = trees[name]
    r = ctx.integrate(_problem(g))
    assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"])
    assert r.tasks_per_level == g["tasks_per_level"]
    assert r.leaves_per_level == g["leaves_per_level"]
    assert _area_ok(r.area, g["area_quad"]), (r.area, g["area_quad"])
    # F bit-exact (cosh^4 and sin(1/x) restate glibc): leaf areas are the reference's; lanes sum
    # their own few leaves in double, everything above is double-double, so the area is within 1 ulp
    # of the correctly rounded sum of the leaf areas
    want = float(g["area_quad"])
    assert abs(r.area - want) <= math.ulp(want), (r.area.hex(), want.hex())
    assert sum(r.tasks_per_cu.values()) == r.tasks
    assert r.n_cu == len(r.tasks_per_cu) >= 1


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "cosh4_eps1e-8", "cosh4_eps1e-10", "sin_recip_eps1e-9",
                                  "cosh4_eps1e3_root_leaf", "cosh4_empty_interval", "cosh4_neg_domain",
                                  "gauss_eps1e-13"])
def test_level_path_parity(ctx, trees, name):
    g = trees[name]
    r = ctx.integrate_levels(_problem(g))
    assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"])
    assert r.tasks_per_level == g["tasks_per_level"]
    assert r.leaves_per_level == g["leaves_per_level"]
    assert _area_ok(r.area, g["area_quad"])


def test_reference_known_answer_printout(ctx, trees):
    """aquadPartA.c:31-32: Area=7583461.801486 at EPSILON=1e-3; Σ tasks = 6567."""
    from ppls_amd import farmer, format_reference
    area, tpp = farmer(5, ctx=ctx)
    out = format_reference(area, tpp)
    ref = trees["cosh4_eps1e-3"]["reference"]["stdout"]
    assert out.splitlines()[0] == ref.splitlines()[0] == "Area=7583461.801486"
    assert out.splitlines()[2:4] == ref.splitlines()[2:4]
    assert tpp[0] == 0 and sum(tpp) == 6567 and len(tpp) == 5


@pytest.mark.parametrize("nshards", [2, 3, 8])
@pytest.mark.parametrize("name", ["cosh4_eps1e-10", "cosh4_eps1e-12", "sin_recip_eps1e-9", "gauss_eps1e-13"])
def test_shards_match_oracle_partition(ctx, trees, oracle, name, nshards):
    g = trees[name]
    p = _problem(g)
    tot_t = tot_l = 0
    area = 0.0
    for s in range(nshards):
        r = ctx.integrate_shard(p, s, nshards)
        o = oracle.integrate_shard(s, nshards, G=ctx.num_workers, S=device_seed_S(ctx.num_workers, nshards),
                                   integrand=p.integrand, a=p.a, b=p.b,
                                   eps=p.eps)
        assert (r.tasks, r.accepted) == (o.tasks, o.leaves)
        assert r.tasks_per_level == o.tasks_per_level
        tot_t += r.tasks
        tot_l += r.accepted
        area += r.area
    assert (tot_t, tot_l) == (g["tasks"], g["leaves"])
    assert _area_ok(area, g["area_quad"])


def test_async_slots_back_to_back(ctx, trees):
    from ppls_amd import Problem
    g = trees["cosh4_eps1e-10"]
    k = 12
    for s in range(k):
        ctx.integrate_async(Problem(eps=1e-10), s)
    ctx.synchronize()
    for s in range(k):
        r = ctx.fetch(s)
        assert (r.tasks, r.accepted) == (g["tasks"], g["leaves"])
        assert _area_ok(r.area, g["area_quad"])


def test_repeatable_counts(ctx, trees):
    from ppls_amd import Problem
    g = trees["cosh4_eps1e-12"]
    for _ in range(3):
        r = ctx.integrate(Problem(eps=1e-12))
        assert (r.tasks, r.accepted) == (g["tasks"], g["leaves"])


def test_errors(ctx):
    from ppls_amd import AquadError, Problem
    with pytest.raises(AquadError):
        ctx.integrate(Problem(a=1.0, b=0.0))
    with pytest.raises(AquadError):
        ctx.integrate(Problem(eps=float("nan")))
    with pytest.raises(AquadError, match="depth"):
        ctx.integrate(Problem(eps=1e-10, max_depth=10))
    # the domain (include/aquad.h AQ_EINVAL): bounds 0 or 2^-900 <= |x| <= 2^900, |x| <= 170 for cosh^4
    for a, b, f in [(1e-300, 1.0, 1), (0.0, 2.0 ** 901, 1), (0.0, 171.0, 0)]:
        with pytest.raises(AquadError):
            ctx.integrate(Problem(a=a, b=b, eps=1e-3, integrand=f))
    assert ctx.integrate(Problem(a=2.0 ** -900, b=1.0, eps=1e-3, integrand=1)).tasks > 0
    # the context is still usable after an error
    assert ctx.integrate(Problem(eps=1e-3)).tasks == 6567


def test_batch_front_end(ctx, batch_golden, oracle):
    a, b = oracle.batch_bounds(64)
    area, tasks, acc = ctx.integrate_batch(a, b, 1e-3)
    assert [int(v) for v in acc] == batch_golden["leaves_eps1e-3_first256"][:64]
    assert (tasks == 2 * acc - 1).all()
    want = np.array([float.fromhex(h) for h in batch_golden["area_eps1e-3_first256_hex"][:64]])
    assert np.all(np.abs(area - want) <= AREA_RTOL * np.abs(want))


def test_batch_front_end_multi_chunk(ctx, batch_golden, oracle):
    """A batch of three launches' worth (2 x MAXK + 1000 integrals): the rows of every chunk are
    unpacked while the next one runs; the first 256 against the golden fixture, the last chunk's
    against the oracle. A bad bound in the second chunk fails the call and leaves the context usable."""
    from ppls_amd import AquadError
    mk = ctx.max_integrals_per_launch
    n = 2 * mk + 1000
    a, b = oracle.batch_bounds(n)
    before = ctx.device_bytes
    area, tasks, acc = ctx.integrate_batch(a, b, 1e-3)
    # the device keeps two chunks' bounds, rows and size order and one chunk's size keys (140 B per row
    # of a chunk, at most MAXK rows; plus 4 KiB of size-class counters on a context's first batch), not
    # the whole batch: a third chunk reuses the first's
    assert ctx.device_bytes - before <= 140 * mk + 8192, (before, ctx.device_bytes)
    assert [int(v) for v in acc[:256]] == batch_golden["leaves_eps1e-3_first256"]
    assert (tasks == 2 * acc - 1).all()
    oa, ot, ol = oracle.integrate_batch(a[-200:], b[-200:], 1e-3)
    assert list(acc[-200:]) == list(ol) and list(tasks[-200:]) == list(ot)
    bad_a = a.copy()
    bad_a[mk + 4464] = np.nan
    with pytest.raises(AquadError):
        ctx.integrate_batch(bad_a, b, 1e-3)
    area2, _, acc2 = ctx.integrate_batch(a[:64], b[:64], 1e-3)
    assert list(acc2) == list(acc[:64])


def test_cli_reference_output(trees):
    from ppls_amd import build
    build.build()
    out = subprocess.run([build.CLI, "-n", "5"], capture_output=True, text=True, timeout=120, check=True).stdout
    lines = out.splitlines()
    assert lines[0] == "Area=7583461.801486"
    assert lines[2] == "Tasks Per Process"
    assert lines[3] == "0\t1\t2\t3\t4\t"
    counts = [int(v) for v in lines[4].split()]
    assert counts[0] == 0 and sum(counts) == 6567


def test_many_integrals_one_launch(ctx, oracle, trees):
    """K integrals with different bounds share one persistent launch; each slot is its own tree."""
    a, b = oracle.batch_bounds(7)
    a = np.concatenate([[0.0], a, [0.0]])
    b = np.concatenate([[5.0], b, [5.0]])
    ctx.integrate_many_async(a, b, 1e-8, first_slot=3)
    for i in range(a.size):
        r = ctx.fetch(3 + i, detail=True)
        o = oracle.integrate(a=a[i], b=b[i], eps=1e-8)
        assert (r.tasks, r.accepted, r.levels) == (o.tasks, o.leaves, o.levels)
        assert r.tasks_per_level == o.tasks_per_level and r.leaves_per_level == o.leaves_per_level
        assert abs(r.area - o.area) <= AREA_RTOL * abs(o.area)


@pytest.mark.parametrize("k", [2, 11, 12, 15, 16])
def test_few_integrals_static_jobs(ctx, oracle, trees, k):
    """Launches of fewer than 12 integrals (the per-CU instance) seed one share per wave with a static,
    rotated stride; from 12 on (r06: from 16) they claim jobs filled to one per wave. Every integral is
    its own exact tree; the cosh4 [0,5] ones match the golden counts."""
    g = trees["cosh4_eps1e-8"]
    a, b = oracle.batch_bounds(k)
    a[0], b[0] = 0.0, 5.0
    a[-1], b[-1] = 0.0, 5.0
    ctx.integrate_many_async(a, b, 1e-8, first_slot=100)
    for i in range(k):
        r = ctx.fetch(100 + i)
        o = oracle.integrate(a=a[i], b=b[i], eps=1e-8)
        assert (r.tasks, r.accepted) == (o.tasks, o.leaves), (k, i)
        assert abs(r.area - o.area) <= AREA_RTOL * abs(o.area)
    for i in (0, k - 1):
        assert (ctx.fetch(100 + i).tasks, ctx.fetch(100 + i).accepted) == (g["tasks"], g["leaves"])


def test_sync_call_leaves_async_slots_alone(ctx, trees):
    """aq_integrate runs in an internal slot: a pending async slot keeps its own result."""
    from ppls_amd import Problem
    g3, g10 = trees["cosh4_eps1e-3"], trees["cosh4_eps1e-10"]
    ctx.integrate_async(Problem(eps=1e-3), 0)
    r = ctx.integrate(Problem(eps=1e-10))
    assert (r.tasks, r.accepted) == (g10["tasks"], g10["leaves"])
    r0 = ctx.fetch(0)
    assert (r0.tasks, r0.accepted) == (g3["tasks"], g3["leaves"])
    r = ctx.integrate(Problem(eps=1e-3))      # the internal slot starts from zero again
    assert (r.tasks, r.accepted) == (g3["tasks"], g3["leaves"])


def test_cu_task_counters_every_launch(ctx, trees):
    """per-CU task counters on every launch shape (the farmer's tasks_per_process,
    aquadPartA.c:162). A pipelined bench-shape batch: the counters over all its launches sum to the
    tasks of every integral, and every CU ran some; a lone integral: they equal its per-CU row."""
    from ppls_amd import Problem
    g8, g10 = trees["cosh4_eps1e-8"], trees["cosh4_eps1e-10"]
    ctx.set_level_histograms(False)
    try:
        ctx.cu_task_counters(reset=True)
        k = 4096
        for _ in range(3):                     # three pipelined launches, no host sync between them
            ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-8, first_slot=0)
        cu = ctx.cu_task_counters(reset=True)
        assert sum(cu.values()) == 3 * k * g8["tasks"]
        assert len(cu) == ctx.num_cus
        r = ctx.integrate(Problem(eps=1e-10))
        cu1 = ctx.cu_task_counters(reset=True)
        assert sum(cu1.values()) == r.tasks == g10["tasks"]
        assert cu1 == r.tasks_per_cu
    finally:
        ctx.set_level_histograms(True)


def test_small_launches_in_high_slots(ctx, trees):
    """launches of fewer than 12 integrals run the per-CU instance only while their
    slots lie below NPARTS = 16384 (the per-workgroup words exist for those; 65536 before r06); at
    first_slot 16373 with 11 integrals (the last per-CU slots), 16380 with 11 (straddling the boundary),
    65531, 200000 and the last slot, they run the bulk instance with a static job stride. Counts exact and
    areas within 1e-12 everywhere -- the per-CU instance's area through its per-workgroup words
    (PCU_AREA, folded by k_fold_parts) -- and within one ulp of the leaf sum for the per-CU ones; the
    per-CU row is kept below NPARTS and documented as absent above (n_cu = 0, include/aquad.h) -- the
    context's per-CU counters (aq_cu_task_counters) count every launch either way."""
    g = trees["cosh4_eps1e-8"]
    nparts = 16384
    ctx.set_level_histograms(False)
    try:
        for first, k in [(0, 3), (16373, 11), (16380, 11), (65531, 1), (65531, 11), (200000, 1), (200000, 11),
                         (ctx.async_slots - 1, 1)]:
            ctx.cu_task_counters(reset=True)
            ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-8, first_slot=first)
            for i in range(k):
                r = ctx.fetch(first + i, detail=True)
                assert (r.tasks, r.accepted) == (g["tasks"], g["leaves"]), (first, k, i)
                assert _area_ok(r.area, g["area_quad"]), (first, k, i)
                if first + k <= nparts:
                    assert r.n_cu >= 1 and sum(r.tasks_per_cu.values()) == r.tasks
                    want = float(g["area_quad"])
                    assert abs(r.area - want) <= math.ulp(want), (first, k, i, r.area.hex(), want.hex())
                else:
                    assert r.n_cu == 0 and r.tasks_per_cu == {}
            assert sum(ctx.cu_task_counters(reset=True).values()) == k * g["tasks"]
    finally:
        ctx.set_level_histograms(True)


def _gather(ctx, n):
    """Rows {area, tasks, accepted, error} of slots 0..n-1 (aq_gather_results into a device buffer)."""
    import torch
    out = torch.empty((n, 4), dtype=torch.float64, device="cuda")
    ctx.gather_results(0, n, out.data_ptr())
    ctx.synchronize()
    return out.cpu().numpy()


def test_batch_order_and_host_threads_do_not_change_results(ctx, oracle, monkeypatch):
    """Size-ordered chunks (the default) against input order (AQ_BATCH_SORT=0), and host work on
    one thread against several (AQ_HOST_THREADS): every integral's counts identical, its area
    within 2 ulp (another schedule of the same tree), over a two-chunk batch."""
    n = 131072 + 5000
    a, b = oracle.batch_bounds(n)
    ref_area, ref_tasks, ref_acc = ctx.integrate_batch(a, b, 1e-3)
    for env in ({"AQ_BATCH_SORT": "0"}, {"AQ_HOST_THREADS": "1"}, {"AQ_BATCH_SORT": "0", "AQ_HOST_THREADS": "3"}):
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            area, tasks, acc = ctx.integrate_batch(a, b, 1e-3)
        assert (tasks == ref_tasks).all() and (acc == ref_acc).all(), env
        assert np.all(np.abs(area - ref_area) <= 2 * np.spacing(np.abs(ref_area))), env


def test_max_integrals_per_launch_batch(ctx, oracle, batch_golden):
    """MAXK (262144) integrals with random bounds in ONE persistent launch (the launch shape of the
    N-GPU bench); the first 256 against the committed golden fixture, 4096 more drawn across the launch
    against the oracle, every integral T = 2L - 1."""
    k = ctx.max_integrals_per_launch
    assert k == 262144
    a, b = oracle.batch_bounds(k)
    ctx.set_level_histograms(False)
    try:
        ctx.integrate_many_async(a, b, 1e-3, first_slot=0)
        rows = _gather(ctx, k)
    finally:
        ctx.set_level_histograms(True)
    assert (rows[:, 3] == 0).all()
    assert [int(v) for v in rows[:256, 2]] == batch_golden["leaves_eps1e-3_first256"]
    want = np.array([float.fromhex(h) for h in batch_golden["area_eps1e-3_first256_hex"]])
    assert np.all(np.abs(rows[:256, 0] - want) <= AREA_RTOL * np.abs(want))
    assert (rows[:, 1] == 2 * rows[:, 2] - 1).all()
    pick = np.sort(np.random.default_rng(3).choice(np.arange(256, k), 4096, replace=False))
    oa, ot, ol = oracle.integrate_batch(a[pick], b[pick], 1e-3)
    assert (rows[pick, 2] == ol).all() and (rows[pick, 1] == ot).all()
    assert np.all(np.abs(rows[pick, 0] - oa) <= AREA_RTOL * np.abs(oa))


def test_many_sharded(ctx, oracle, trees):
    """Sharded multi-integral launches: per-shard counts match the oracle partition (one share per wave worker)."""
    g = trees["cosh4_eps1e-10"]
    tot_t = tot_l = 0
    for s in range(2):
        ctx.integrate_many_async(np.zeros(3), np.full(3, 5.0), 1e-10, first_slot=10, shard=s, nshards=2)
        rs = [ctx.fetch(10 + i) for i in range(3)]
        assert len({(r.tasks, r.accepted) for r in rs}) == 1
        tot_t += rs[0].tasks
        tot_l += rs[0].accepted
    assert (tot_t, tot_l) == (g["tasks"], g["leaves"])


def test_large_jobs_and_cellar(trees, monkeypatch):
    """Jobs of 8 waves' shares (deep per-wave subtrees, claimed dynamically): ring overflow goes
    through the per-wave HBM cellars and every integral still matches the golden tree."""
    from ppls_amd import Context
    monkeypatch.setenv("AQ_GSPLIT", "8")
    c = Context(0)
    try:
        c.set_level_histograms(False)
        c.set_diagnostics(True)
        g = trees["cosh4_eps1e-12"]
        k = 32
        c.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-12, first_slot=0)
        d, f = c.diagnostics()
        for i in range(k):
            r = c.fetch(i)
            assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"])
            assert _area_ok(r.area, g["area_quad"])
        col = dict(zip(f, d.T))
        assert col["cellar_out"].sum() > 0
        assert col["cellar_out"].sum() == col["cellar_in"].sum() + col["prefetch"].sum()
    finally:
        c.close()


def test_back_to_back_launches_same_slots(ctx, oracle, batch_golden, trees):
    """Launches queued without a host sync reuse the same slots; each gathers its own results
    (bounds staging must not be overwritten while a previous copy is pending)."""
    import torch
    a1, b1 = oracle.batch_bounds(8)
    out = torch.zeros((3, 8, 4), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ctx.set_level_histograms(False)
    try:
        for rep in range(3):
            if rep == 1:
                ctx.integrate_many_async(np.zeros(8), np.full(8, 5.0), 1e-3, first_slot=0)
            else:
                ctx.integrate_many_async(a1, b1, 1e-3, first_slot=0)
            ctx.gather_results(0, 8, out[rep].data_ptr())
        ctx.synchronize()
    finally:
        ctx.set_level_histograms(True)
    o = out.cpu().numpy()
    want = batch_golden["leaves_eps1e-3_first256"][:8]
    assert [int(v) for v in o[0, :, 2]] == want and [int(v) for v in o[2, :, 2]] == want
    assert (o[1, :, 2] == trees["cosh4_eps1e-3"]["leaves"]).all()
    assert (o[:, :, 3] == 0).all()


def test_mixed_bounds_and_shards(ctx, oracle, trees):
    """Lone integrals of every golden tree, a 40-integral launch of mixed bounds, and a 5-way sharded
    integral (the seeding's many-node path) -- counts bit-exact, areas within 1e-12."""
    for name in ["cosh4_eps1e-3", "cosh4_eps1e-10", "cosh4_eps1e-12", "sin_recip_eps1e-9", "cosh4_empty_interval"]:
        g = trees[name]
        r = ctx.integrate(_problem(g))
        assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"]), name
        assert r.tasks_per_level == g["tasks_per_level"]
        assert _area_ok(r.area, g["area_quad"])
    a, b = oracle.batch_bounds(32)
    a = np.concatenate([a, np.zeros(8)])
    b = np.concatenate([b, np.full(8, 5.0)])
    ctx.integrate_many_async(a, b, 1e-8, first_slot=100)
    oa, ot, ol = oracle.integrate_batch(a, b, 1e-8)
    for i in range(a.size):
        r = ctx.fetch(100 + i, detail=True)
        assert (r.tasks, r.accepted) == (int(ot[i]), int(ol[i])), i
        assert abs(r.area - oa[i]) <= AREA_RTOL * abs(oa[i])
    g = trees["cosh4_eps1e-10"]
    tot = [0, 0]
    for s in range(5):
        r = ctx.integrate_shard(_problem(g), s, 5)
        o = oracle.integrate_shard(s, 5, G=ctx.num_workers, S=device_seed_S(ctx.num_workers, 5), integrand=0, a=0.0, b=5.0, eps=1e-10)
        assert (r.tasks, r.accepted) == (o.tasks, o.leaves)
        tot[0] += r.tasks
        tot[1] += r.accepted
    assert tot == [g["tasks"], g["leaves"]]


def test_adaptive_job_size_keeps_counts(ctx, oracle, trees):
    """Multi-integral launches size their jobs from the previous launch of the same workload (a
    device-side hint); switching workload (tiny random trees <-> the eps=1e-10 tree, sharded or
    not) changes the shares per integral, never the counts."""
    g10 = trees["cosh4_eps1e-10"]
    a, b = oracle.batch_bounds(64)
    oa, ot, ol = oracle.integrate_batch(a, b, 1e-3)
    ctx.set_level_histograms(False)
    phase_shard_checked = [False, False]
    try:
        for phase in ["big", "big", "small", "small", "big", "shard", "shard", "big"]:
            if phase == "big":
                ctx.integrate_many_async(np.zeros(64), np.full(64, 5.0), 1e-10, first_slot=0)
                rs = [ctx.fetch(i) for i in range(64)]
                assert all((r.tasks, r.accepted) == (g10["tasks"], g10["leaves"]) for r in rs), phase
                assert all(_area_ok(r.area, g10["area_quad"]) for r in rs)
            elif phase == "small":
                ctx.integrate_many_async(a, b, 1e-3, first_slot=0)
                rs = [ctx.fetch(i) for i in range(64)]
                assert [(r.tasks, r.accepted) for r in rs] == [(int(t), int(l)) for t, l in zip(ot, ol)]
            else:
                tot = np.zeros((64, 2), np.int64)
                for s in range(2):
                    ctx.integrate_many_async(np.zeros(64), np.full(64, 5.0), 1e-10, first_slot=0, shard=s, nshards=2)
                    rs = [ctx.fetch(i) for i in range(64)]
                    tot += np.array([(r.tasks, r.accepted) for r in rs], np.int64)
                    if phase_shard_checked[s]:
                        continue
                    phase_shard_checked[s] = True
                    # each shard's partition against the oracle's: every integral of a sharded launch
                    # at AQ_GSPLIT_DEFAULT (192) waves per share and shard -- the last ones too (no
                    # end-of-launch tail for shards: all shards of an integral share its partition)
                    Gm = ctx.num_workers // (192 * 2)
                    for i, G in ((0, Gm), (63, Gm)):
                        o = oracle.integrate_shard(s, 2, G=G, S=device_seed_S(G, 2), integrand=0, a=0.0, b=5.0,
                                                   eps=1e-10)
                        assert (rs[i].tasks, rs[i].accepted) == (o.tasks, o.leaves), (s, i)
                assert (tot == np.array([g10["tasks"], g10["leaves"]])).all()
    finally:
        ctx.set_level_histograms(True)


@pytest.mark.parametrize("k", [16, 64, 700])
def test_few_integrals_fill_the_waves(ctx, trees, k):
    """Launches of fewer integrals than the GPU's waves (16 .. W - 1, unsharded) run the few-integral /
    batch instance, which raises the job-size hint's shares per integral to fill the waves (up to one
    job per wave, none below 2 k tasks; DESIGN §2.1 *Few integrals*). Its first launch (no hint), its
    hinted launches, and a switch to and from a launch of more integrals than waves (the bench's
    instance, which leaves no per-integral task count in the hint) keep every count exact and every
    area within the tolerance of the golden tree's quad sum -- for the skewed sin(1/x) tree and cosh4."""
    from ppls_amd import SIN_RECIP
    big = ctx.num_workers + 64
    ctx.set_level_histograms(False)
    try:
        for name, integrand, a0, b0, eps in (("sin_recip_eps1e-9", SIN_RECIP, 1e-4, 1.0, 1e-9),
                                             ("cosh4_eps1e-8", 0, 0.0, 5.0, 1e-8)):
            g = trees[name]
            for n in (k, k, big, k):
                ctx.integrate_many_async(np.full(n, a0), np.full(n, b0), eps, first_slot=0, integrand=integrand)
                rs = [ctx.fetch(i) for i in (0, n // 2, n - 1)]
                assert all((r.tasks, r.accepted) == (g["tasks"], g["leaves"]) for r in rs), (name, n)
                assert all(_area_ok(r.area, g["area_quad"]) for r in rs), (name, n)
    finally:
        ctx.set_level_histograms(True)


def test_random_batches_match_oracle_across_launch_shapes(ctx, oracle):
    """The r06 launch shapes against the CPU restatement on random bounds at tolerances no golden
    fixture holds: a one-chunk sorted batch (size classes, the pre-pass stream, the host pool, the
    batch instance's fill rule) at eps=1e-6, few-integral launches (static per-CU deal, claimed filled
    jobs; first and hinted) of cosh4 at 1e-7 and of sin(1/x) at 1e-8. Counts exact, areas within the
    per-tree tolerance of the oracle's."""
    from ppls_amd import SIN_RECIP
    a, b = oracle.batch_bounds(3000)
    area, tasks, acc = ctx.integrate_batch(a, b, 1e-6)
    oa, ot, ol = oracle.integrate_batch(a, b, 1e-6)
    assert (tasks == ot).all() and (acc == ol).all()
    assert np.all(np.abs(area - oa) <= AREA_RTOL * np.abs(oa))
    ctx.set_level_histograms(False)
    try:
        for k in (5, 14, 40):
            ak, bk = a[:k], b[:k]
            oa, ot, ol = oracle.integrate_batch(ak, bk, 1e-7)
            for _ in range(2):   # the first launch of the workload, then a hinted one
                ctx.integrate_many_async(ak, bk, 1e-7, first_slot=0)
                rs = [ctx.fetch(i) for i in range(k)]
                assert [(r.tasks, r.accepted) for r in rs] == [(int(t), int(l)) for t, l in zip(ot, ol)], k
                assert all(abs(r.area - w) <= AREA_RTOL * abs(w) for r, w in zip(rs, oa)), k
        k = 24
        sa, sb = 1e-4 + a[:k] / 5.0, 1e-4 + b[:k] / 5.0 + 1e-3
        oa, ot, ol = oracle.integrate_batch(sa, sb, 1e-8, integrand=oracle.SIN_RECIP)
        for _ in range(2):
            ctx.integrate_many_async(sa, sb, 1e-8, first_slot=0, integrand=SIN_RECIP)
            rs = [ctx.fetch(i) for i in range(k)]
            assert [(r.tasks, r.accepted) for r in rs] == [(int(t), int(l)) for t, l in zip(ot, ol)]
            assert all(abs(r.area - w) <= AREA_RTOL * abs(w) for r, w in zip(rs, oa))
    finally:
        ctx.set_level_histograms(True)


# Deep trees (up to 150 M tasks, depth 31, in one launch), pinned by the reference binary's own task
# totals (tests/golden/deep.json, make_golden.py deep): alone and as a small batch.
@pytest.mark.parametrize("name", ["cosh4_eps1e-14", "cosh4_eps1e-15", "cosh4_eps1e-16"])
def test_deep_trees(ctx, deep_golden, name):
    from ppls_amd import Problem
    g = deep_golden[name]
    assert g["reference"]["tasks_total"] == g["tasks"]
    ctx.set_level_histograms(True)
    r = ctx.integrate(Problem(eps=g["eps"]))
    assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"])
    assert r.tasks_per_level == g["tasks_per_level"] and r.leaves_per_level == g["leaves_per_level"]
    assert abs(r.area - float(g["area_quad"])) <= math.ulp(float(g["area_quad"]))
    assert sum(r.tasks_per_cu.values()) == r.tasks
    ctx.set_level_histograms(False)
    try:
        ctx.integrate_many_async(np.zeros(4), np.full(4, 5.0), g["eps"], first_slot=0)
        got = [ctx.fetch(i) for i in range(4)]
        assert all((x.tasks, x.accepted) == (g["tasks"], g["leaves"]) for x in got)
        assert all(_area_ok(x.area, g["area_quad"]) for x in got)
    finally:
        ctx.set_level_histograms(True)


@pytest.mark.parametrize("eps", [1e-10, 1e-12])
def test_sin_recip_deeper(ctx, oracle, eps):
    """Config 4's integrand past the fixture's eps=1e-9: the device's glibc sin makes every leaf the
    oracle's, so counts, histograms and the area (within 1 ulp of the exact leaf sum) all agree."""
    from ppls_amd import Problem
    o = oracle.integrate(integrand=1, a=1e-4, b=1.0, eps=eps)
    r = ctx.integrate(Problem(1, 1e-4, 1.0, eps))
    assert (r.tasks, r.accepted, r.levels) == (o.tasks, o.leaves, o.levels)
    assert r.tasks_per_level == o.tasks_per_level
    want = o.area_quad_hi + o.area_quad_lo
    assert abs(r.area - want) <= math.ulp(want), (r.area.hex(), want.hex())


def test_c3_eps1e10_max_launch(ctx, oracle, batch_golden):
    """SURVEY config 3 at its throughput tolerance in ONE launch of the maximum size (262144 random
    bounds, splitmix64): the first 200 against the fixture the oracle committed (tests/golden/
    batch.json), 48 more drawn across the launch against the oracle live, every integral T = 2L - 1,
    and a second launch of the same integrals in reverse order (another schedule) agreeing."""
    k = ctx.max_integrals_per_launch
    a, b = oracle.batch_bounds(k)
    ctx.set_level_histograms(False)
    try:
        ctx.integrate_many_async(a, b, 1e-10, first_slot=0)
        rows = _gather(ctx, k)
        ctx.integrate_many_async(a[::-1].copy(), b[::-1].copy(), 1e-10, first_slot=0)
        rev = _gather(ctx, k)[::-1]
    finally:
        ctx.set_level_histograms(True)
    assert (rows[:, 3] == 0).all() and (rev[:, 3] == 0).all()
    n10 = batch_golden["n_eps1e-10"]
    assert [int(v) for v in rows[:n10, 2]] == batch_golden["leaves_eps1e-10"]
    want = [float.fromhex(h) for h in batch_golden["area_eps1e-10_hex"]]
    assert all(abs(r - w) <= math.ulp(w) for r, w in zip(rows[:n10, 0], want))
    assert (rows[:, 1] == 2 * rows[:, 2] - 1).all()
    # the exact KAT of the first 10 000 draws (tests/golden/batch.json, the oracle's own 3e9 tasks)
    kn = batch_golden["kat_n_eps1e-10"]
    assert int(rows[:kn, 2].sum()) == batch_golden["kat_sum_leaves_eps1e-10"]
    assert int(rows[:kn, 1].sum()) == batch_golden["kat_sum_tasks_eps1e-10"]
    assert (rev[:, 1:3] == rows[:, 1:3]).all()
    assert all(abs(x - y) <= 2 * math.ulp(y) for x, y in zip(rev[:, 0], rows[:, 0]))
    pick = np.random.default_rng(7).choice(np.arange(n10, k), 48, replace=False)
    oa, ot, ol = oracle.integrate_batch(a[pick], b[pick], 1e-10)
    for j, i in enumerate(pick):
        assert (rows[i, 1], rows[i, 2]) == (int(ot[j]), int(ol[j])), i
        assert abs(rows[i, 0] - oa[j]) <= AREA_RTOL * abs(oa[j])


def test_fresh_context_first_tiny_batch(oracle, batch_golden):
    """A fresh context's first batch of tiny trees (C3 at eps=1e-3, 65536 integrals): the size
    pre-pass sets the first launch's job size (whole-integral jobs here) instead of the default 16
    shares per integral, with which ~90-task jobs had made it seeding-bound (13 ms where a sized launch
    takes ~0.5, profiles/r05w). Counts exact, and -- deterministically, not by the clock -- the
    launch ran whole-integral jobs: one seeding pass per integral (the DIAG instance's seed_calls), where
    the unsized default seeds 16 shares of each."""
    from ppls_amd import Context
    k = 65536
    a, b = oracle.batch_bounds(k)
    with Context(0) as c:
        c.set_level_histograms(False)
        c.set_diagnostics(True)   # the DIAG instance: same partition and job sizing, per-workgroup counters
        area, tasks, acc = c.integrate_batch(a, b, 1e-3)
        dg, names = c.diagnostics()
    assert (tasks == 2 * acc - 1).all()
    first = batch_golden["leaves_eps1e-3_first256"]
    assert [int(v) for v in acc[:len(first)]] == first
    kn = batch_golden["n_eps1e-3"]
    assert int(acc[:kn].sum()) == batch_golden["sum_leaves_eps1e-3"]
    assert int(tasks[:kn].sum()) == batch_golden["sum_tasks_eps1e-3"]
    assert dg.shape[0] > 0 and int(dg[:, list(names).index("seed_calls")].sum()) == k


def test_stall_bound_is_not_a_run_time_cap(ctx, deep_golden):
    """A launch far longer than the stall bound (50 ms here; 1024 integrals at eps=1e-16, 1.5e11
    tasks) completes with exact counts: the on-device wait is bounded by time without progress only."""
    g = deep_golden["cosh4_eps1e-16"]
    k = 1024
    ctx.set_level_histograms(False)
    ctx.set_stall_timeout(50.0)
    try:
        ctx.kernel_timing(True)
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-16, first_slot=0)
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        got = [ctx.fetch(i) for i in range(k)]
    finally:
        ctx.set_stall_timeout(10000.0)
        ctx.set_level_histograms(True)
    assert ms > 200.0   # the launch really outlived the bound several times over
    assert all((x.tasks, x.accepted) == (g["tasks"], g["leaves"]) for x in got)


def test_plugin_integrand_bit_exact(ctx, plugin_bits):
    """AQ_F_USER (the default plug-in, exp(-x*x)) on the device equals the host libm bit for bit,
    including exp's tiny-argument and subnormal-result paths."""
    from ppls_amd import USER, user_integrand_name
    assert user_integrand_name().startswith("gauss")
    x = plugin_bits["x"].view(np.float64)
    got = ctx.eval_integrand(x, integrand=USER).view(np.uint64)
    bad = np.nonzero(got != plugin_bits["F"])[0]
    assert bad.size == 0, [(float(x[i]), hex(int(got[i])), hex(int(plugin_bits["F"][i]))) for i in bad[:8]]


def test_plugin_reference_printout(ctx, trees):
    """The plug-in tree against the reference binary built with that F (its printed Area= and task total)."""
    for name in ["gauss_eps1e-10", "gauss_eps1e-13"]:
        g = trees[name]
        r = ctx.integrate(_problem(g))
        assert r.tasks == g["reference"]["tasks_total"]
        assert "%f" % r.area == g["reference"]["area_printed"]


def test_context_footprint():
    """No per-wave area partials or second engine: a fresh context holds ~1.2 GiB -- 262144 result
    slots (738 MB, r04: 8 x 32768 per launch), the wave cellars (302 MB: 2048 pairs each since r05,
    from 4096), the per-CU count and area words of the first 16384 slots (134 MB; r05: counts of 65536,
    268 MB) and the HBM queue -- of the GPU's
    288 GB (round 1: ~7 GiB; the level path's two 512 MiB frontiers are allocated only when
    aq_integrate_levels first runs)."""
    from ppls_amd import Context
    with Context(0) as c:
        assert c.device_bytes < 1.45 * 2 ** 30, c.device_bytes


def test_exact_rows_sum_over_shards(ctx, trees):
    """Exact rows (int64 limbs) summed over the shards of a partition round to the whole area within
    one ulp of the correctly rounded leaf sum, and the counts add up."""
    from ppls_amd import Problem, exact_round
    g = trees["cosh4_eps1e-12"]
    tot = np.zeros(72, np.int64)
    for s in range(8):
        ctx.integrate_async(Problem(eps=1e-12), slot=s, shard=s, nshards=8)
    ctx.synchronize()
    for s in range(8):
        row = ctx.fetch_exact(s)
        assert row[71] >> 32 == 0   # no error bits
        tot[:71] += row[:71]
    assert (int(tot[68]), int(tot[69])) == (g["tasks"], g["leaves"])
    want = float(g["area_quad"])
    assert abs(exact_round(tot) - want) <= math.ulp(want)


def test_mixed_shard_launch(ctx, oracle, trees):
    """One launch holding different shards of different integrals (the rebalanced batch's launch
    shape): every entry equals the oracle's shard, and each integral's shards sum to its tree."""
    g = trees["sin_recip_eps1e-9"]
    N = 8
    shards = np.array([s for s in range(N) for _ in range(3)], np.int32)[::-1].copy()
    a = np.full(shards.size, 1e-4)
    b = np.ones(shards.size)
    ctx.set_level_histograms(False)
    try:
        ctx.integrate_mixed_async(a, b, shards, N, 1e-9, first_slot=0, integrand=1)
        got = [ctx.fetch(i) for i in range(shards.size)]
    finally:
        ctx.set_level_histograms(True)
    want = {}
    for s in range(N):
        G = ctx.num_workers // (192 * N)   # aq_stream.h AQ_GSPLIT_DEFAULT waves per share and shard (V = 16: deeper seeding)
        o = oracle.integrate_shard(s, N, G=G, S=device_seed_S(G, N), integrand=1, a=1e-4, b=1.0, eps=1e-9)
        want[s] = (o.tasks, o.leaves)
    for i, s in enumerate(shards):
        assert (got[i].tasks, got[i].accepted) == want[int(s)], (i, int(s))
    assert sum(want[s][0] for s in range(N)) == g["tasks"]


def test_rccl_group_single_process(ctx, trees):
    """aq_integrate_group over an in-library RCCL communicator (one GPU here: a group of one runs the
    same grouped all-reduce / all-gather the 8-GPU node runs)."""
    from ppls_amd import Group
    with Group([ctx]) as grp:
        assert grp.size == 1
        for name in ["cosh4_eps1e-10", "sin_recip_eps1e-9", "gauss_eps1e-13"]:
            g = trees[name]
            r = grp.integrate(_problem(g))
            assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"]), name
            assert r.tasks_per_level == g["tasks_per_level"]
            assert r.tasks_per_gpu == [g["tasks"]]
            assert sum(r.tasks_per_cu.values()) == g["tasks"]
            assert _area_ok(r.area, g["area_quad"])


def test_group_call_leaves_async_slots_alone(ctx, trees):
    """aq_integrate_group runs its shard in the internal slot, like aq_integrate: a
    pending async slot-0 result survives a Group.integrate, and so does one around integrate_shard_exact."""
    from ppls_amd import Group, Problem
    g3, g10 = trees["cosh4_eps1e-3"], trees["cosh4_eps1e-10"]
    with Group([ctx]) as grp:
        ctx.integrate_async(Problem(eps=1e-3), 0)
        r = grp.integrate(Problem(eps=1e-10))
        assert (r.tasks, r.accepted) == (g10["tasks"], g10["leaves"])
        r0 = ctx.fetch(0)
        assert (r0.tasks, r0.accepted) == (g3["tasks"], g3["leaves"])
        r = grp.integrate(Problem(eps=1e-3))   # the internal slot starts from zero again
        assert (r.tasks, r.accepted) == (g3["tasks"], g3["leaves"])
    ctx.integrate_async(Problem(eps=1e-3), 0)
    row = ctx.integrate_shard_exact(Problem(eps=1e-10), 0, 1)
    assert (int(row[68]), int(row[69])) == (g10["tasks"], g10["leaves"])
    r0 = ctx.fetch(0)
    assert (r0.tasks, r0.accepted) == (g3["tasks"], g3["leaves"])
    r = ctx.integrate(Problem(eps=1e-3))
    assert (r.tasks, r.accepted) == (g3["tasks"], g3["leaves"])


def test_rccl_group_join(ctx, trees):
    """The one-process-per-GPU form (aq_group_unique_id + aq_group_join), as an MPI rank would use it."""
    from ppls_amd import Group, Problem
    uid = Group.unique_id()
    with Group.join(ctx, 1, 0, uid) as grp:
        r = grp.integrate(Problem(eps=1e-10, n_gpus=1))
    g = trees["cosh4_eps1e-10"]
    assert (r.tasks, r.accepted) == (g["tasks"], g["leaves"])


@pytest.mark.gpu
@pytest.mark.parametrize("hist", [False, True])
def test_depth_cap_boundary(ctx, trees, hist):
    """The depth cap (max_depth) at its exact boundary. The bench instance checks it once per burst
    (AQ_BURST_CAP: the deepest pushed pair against max_depth at the burst's end), the histogram
    instance per round; both must agree with the reference's refinement to the level: cosh4 at
    eps=1e-10 has levels L = 23 (its deepest tasks at depth 22), so max_depth = L runs exactly and
    max_depth = L - 1 fails with AQ_EDEPTH -- for a lone launch (per-CU instance) and a 64-integral
    launch; the context stays usable."""
    from ppls_amd import AquadError, Problem
    g = trees["cosh4_eps1e-10"]
    L = g["levels"]
    ctx.set_level_histograms(hist)
    try:
        r = ctx.integrate(Problem(eps=1e-10, max_depth=L))
        assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], L)
        with pytest.raises(AquadError, match="depth"):
            ctx.integrate(Problem(eps=1e-10, max_depth=L - 1))
        k = 64
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-10, first_slot=0, max_depth=L)
        for i in range(k):
            r = ctx.fetch(i)
            assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], L)
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-10, first_slot=0, max_depth=L - 1)
        with pytest.raises(AquadError, match="depth"):
            ctx.fetch(0)
    finally:
        ctx.set_level_histograms(True)   # the context's default
    assert ctx.integrate(Problem(eps=1e-3)).tasks == 6567


def test_grid_that_cannot_be_resident_is_refused(trees, monkeypatch):
    """the persistent grid's workgroups wait on each other, so a grid larger than the
    device can hold at once is refused before launch with AQ_ERESIDENT (-9) -- not a 10 s stall. A
    smaller grid (AQ_GRID) is resident and exact; so is the cooperative launch (AQ_COOP=1)."""
    from ppls_amd import AquadError, Context, Problem
    g = trees["cosh4_eps1e-10"]
    with Context(0) as c0:
        ncu = c0.num_cus
    monkeypatch.setenv("AQ_GRID", str(2 * ncu))   # one workgroup per CU is all k_stream's LDS allows
    c = Context(0)
    try:
        with pytest.raises(AquadError) as e:
            c.integrate(Problem(eps=1e-10))
        assert e.value.code == -9
        with pytest.raises(AquadError) as e:
            c.integrate_many_async(np.zeros(64), np.full(64, 5.0), 1e-10, first_slot=0)
        assert e.value.code == -9
    finally:
        c.close()
    for env in ({"AQ_GRID": str(ncu // 2)}, {"AQ_GRID": "", "AQ_COOP": "1"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        c = Context(0)
        try:
            r = c.integrate(Problem(eps=1e-10))
            assert (r.tasks, r.accepted, r.levels) == (g["tasks"], g["leaves"], g["levels"]), env
            assert _area_ok(r.area, g["area_quad"])
            c.set_level_histograms(False)
            c.integrate_many_async(np.zeros(64), np.full(64, 5.0), 1e-10, first_slot=0)
            for i in (0, 63):
                r = c.fetch(i)
                assert (r.tasks, r.accepted) == (g["tasks"], g["leaves"]), env
        finally:
            c.close()
