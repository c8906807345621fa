"""Sanitizer runs of the CPU-side code (SURVEY §5 "sanitizers"; no GPU sanitizers exist on this pool).

`make -C oracle san` builds the restatement (aq_oracle.c, driven by oracle/san_check.c) under
AddressSanitizer + UndefinedBehaviorSanitizer, and the threaded bag of tasks (aq_bag.c, the CPU
baseline) under ASan + UBSan and under ThreadSanitizer -- its lock-free mailboxes are the only
shared-memory protocol on the CPU side. Every run must exit 0 with no sanitizer report AND reproduce
the golden counts the reference binary pinned (tests/golden/), so a sanitizer build that changed
the arithmetic would fail too."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "oracle", "_build", "san")
REPORT_MARKERS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")


@pytest.fixture(scope="module")
def san():
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], capture_output=True, text=True)
    if r.returncode:
        pytest.skip("sanitizer runtimes unavailable: " + r.stderr[-400:])
    return SAN


def _run(args, timeout=120):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    for m in REPORT_MARKERS:
        assert m not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    return r.stdout


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "cosh4_eps1e-8", "sin_recip_eps1e-9", "gauss_eps1e-10",
                                  "cosh4_empty_interval", "cosh4_neg_domain"])
def test_oracle_tree_under_asan_ubsan(san, trees, name):
    g = trees[name]
    fid = {"cosh4": 0, "sin_recip": 1, "gauss": 2}[g["integrand"]]
    out = _run([os.path.join(san, "san_check"), "tree", str(fid), repr(g["a"]), repr(g["b"]), repr(g["eps"])]).split()
    assert (int(out[0]), int(out[1]), int(out[2])) == (g["tasks"], g["leaves"], g["levels"])
    want = float(g["area_quad"])
    got = float.fromhex(out[3])
    assert abs(got - want) <= 2e-16 * abs(want)


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_oracle_shard_partition_under_asan_ubsan(san, trees, nshards):
    g = trees["cosh4_eps1e-8"]
    out = _run([os.path.join(san, "san_check"), "shards", "0", "0.0", "5.0", "1e-08", str(nshards)]).split()
    assert (int(out[0]), int(out[1]), int(out[2])) == (g["tasks"], g["leaves"], g["levels"])


def test_oracle_batch_under_asan_ubsan(san, batch_golden):
    out = _run([os.path.join(san, "san_check"), "batch", "256", "1e-3"]).split()
    assert int(out[1]) == sum(batch_golden["leaves_eps1e-3_first256"])


@pytest.mark.parametrize("binary", ["aq_bag_asan", "aq_bag_tsan"])
@pytest.mark.parametrize("nprocs", [2, 5])
def test_bag_of_tasks_under_sanitizers(san, trees, binary, nprocs):
    g = trees["cosh4_eps1e-3"]
    out = _run([os.path.join(san, binary), "-n", str(nprocs), "-e", "0.001"])
    lines = out.splitlines()
    assert lines[0] == "Area=7583461.801486"
    assert sum(int(v) for v in lines[-1].split()) == g["tasks"]
    if nprocs == 2:
        assert out == g["reference_p2"]["stdout"]
