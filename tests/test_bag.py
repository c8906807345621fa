"""The bag of tasks on threads (oracle/aq_bag.c): the CPU baseline's port of
aquadPartA.c's farmer/worker. With one worker (P=2) the farmer's arrival order is deterministic,
so its stdout must equal the reference binary's P=2 stdout byte for byte (tests/golden/trees.json,
recorded by tests/golden/make_golden.py); with more workers the task totals are exact and the
printed area is the reference's up to the arrival-order rounding of `result += buff[0]` (:149)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BAG = os.path.join(ROOT, "oracle", "_build", "aq_bag")


@pytest.fixture(scope="module")
def bag():
    if not os.path.exists(BAG) or os.path.getmtime(BAG) < os.path.getmtime(os.path.join(ROOT, "oracle", "aq_bag.c")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_build/aq_bag"])
    return BAG


def _args(g, nprocs):
    a = ["-n", str(nprocs), "-e", repr(g["eps"]), "-a", repr(g["a"]), "-b", repr(g["b"])]
    if g["integrand"] != "cosh4":
        a += ["-f", "sin"]
    return a


def _run(bag, g, nprocs):
    return subprocess.run([bag] + _args(g, nprocs), capture_output=True, text=True, timeout=300, check=True).stdout


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "cosh4_eps1e-10", "sin_recip_eps1e-9"])
def test_one_worker_matches_reference_stdout(bag, trees, name):
    g = trees[name]
    assert _run(bag, g, 2) == g["reference_p2"]["stdout"]


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "sin_recip_eps1e-9", "cosh4_neg_domain", "cosh4_empty_interval",
                                  "cosh4_eps1e3_root_leaf"])
@pytest.mark.parametrize("nprocs", [3, 5, 8])
def test_many_workers_totals(bag, trees, name, nprocs):
    g = trees[name]
    lines = _run(bag, g, nprocs).split("\n")
    assert lines[1] == "" and lines[2] == "Tasks Per Process"
    assert lines[3].split() == [str(i) for i in range(nprocs)]
    counts = [int(v) for v in lines[4].split()]
    assert len(counts) == nprocs and counts[0] == 0 and sum(counts) == g["tasks"]
    area = float(lines[0][len("Area="):])
    # the printed 6th decimal may flip with the arrival order (as the reference's does)
    assert abs(area - float(g["area_quad"])) <= 2e-6 + 1e-12 * abs(float(g["area_quad"]))


def test_needs_two_processes(bag):
    r = subprocess.run([bag, "-n", "1"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 1
    assert r.stderr.strip() == "ERROR: Must have at least 2 processes to run"
