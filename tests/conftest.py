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
def libm_bits():
    z = np.load(os.path.join(GOLDEN, "libm_bits.npz"))  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle
