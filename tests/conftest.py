import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def O():
    """The CPU oracle (checker only)."""
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def pkg():
    """The product package; on a GPU box a missing/broken liborbx.so fails loudly."""
    if not os.path.exists("/dev/kfd"):
        pytest.skip("no AMD GPU driver in this container")
    import orb_slam_cuda_amd
    assert orb_slam_cuda_amd.device_count() >= 1, "liborbx.so sees no HIP device"
    return orb_slam_cuda_amd


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
