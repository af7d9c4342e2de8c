import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.join(ROOT, "tests")
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "murmur3_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_var():
    z = np.load(os.path.join(GOLDEN_DIR, "murmur3_var.npz"))  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle_py import Oracle

    return Oracle()


@pytest.fixture(scope="session")
def hb():
    """The product library (C ABI) bound through ctypes."""
    import sharedhashfile_amd

    sharedhashfile_amd.load()
    return sharedhashfile_amd
