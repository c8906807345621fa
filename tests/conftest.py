import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def trees():
    with open(os.path.join(GOLDEN, "trees.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def batch_golden():
    with open(os.path.join(GOLDEN, "batch.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def deep_golden():
    with open(os.path.join(GOLDEN, "deep.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def plugin_bits():
    z = np.load(os.path.join(GOLDEN, "plugin_bits.npz"))  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def sin_bits():
    z = np.load(os.path.join(GOLDEN, "sin_bits.npz"))  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def libm_bits():
    z = np.load(os.path.join(GOLDEN, "libm_bits.npz"))  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


def device_seed_S(G, nshards):
    """The seed depth offset S for oracle.integrate_shard() that reproduces the device's partition
    (ppls_amd/csrc/aq_stream.h seed_depth / seed_depth_job): V = G * nshards, D = floor(log2 V) + 2,
    one level deeper where (D + 2) levels x ceil(2^(D+1) / V) positions still fit 64 nodes."""
    V = G * nshards
    D = V.bit_length() - 1 + 2
    nb = -(-(1 << (D + 1)) // V)
    return 3 if (D + 2) * nb <= 64 else 2


def exact_row(values, tasks=0, accepted=0, spilled=0, levels=0, error=0):
    """An exact row (include/aquad.h AQ_EXACT_ROW) of the given doubles, built with Python integers:
    limbs whose weighted sum is exactly sum(values) (the CPU shard backends of the dist tests)."""
    import math
    X = 0
    for v in values:
        if v == 0.0:
            continue
        m, e = math.frexp(v)
        X += int(m * 2 ** 53) << (e - 53 + 1088)
    row = np.zeros(72, np.int64)
    for i in range(67):
        row[i] = X & 0xffffffff
        X >>= 32
    row[67] = X
    row[68], row[69], row[70] = tasks, accepted, spilled
    row[71] = levels | (error << 32)
    return row
