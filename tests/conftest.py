import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def engine():
    """Initialised engine (GPU tests only)."""
    import eges_amd
    n = eges_amd.init()
    assert n >= 1
    return eges_amd


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
