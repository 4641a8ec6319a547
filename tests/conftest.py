import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ssl-vit-video-analytics_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long CPU test")
    config.addinivalue_line("markers", "gpu_fresh: runs before every other test (a child process that needs the "
                                       "device memory this process has not touched yet)")


def pytest_collection_modifyitems(config, items):
    """gpu_fresh tests first: their child processes size the device-memory arena from the free
    HBM at start-up, which whatever the test process still holds after hundreds of GPU tests
    would shrink (tests/test_policy_gpu.py checks the policy bench.py's auto rule picks there)."""
    items.sort(key=lambda it: 0 if it.get_closest_marker("gpu_fresh") else 1)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
