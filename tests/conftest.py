import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built library")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.fixture(scope="session")
def gpu():
    """Skip unless a HIP device is present; the library must then load (no fallback)."""
    from movie_recommender_amd import _lib
    L = _lib.lib()
    if L.mr_device_count() < 1:
        pytest.skip("no HIP device")
    return L
