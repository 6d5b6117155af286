import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line(
        "markers", "slow: larger CPU cases")


import subprocess  # noqa: E402

import pytest  # noqa: E402

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "conjugate-gradient_amd"
sys.path.insert(0, str(PKG))


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    """Build libcgx.so (hipcc, gfx950) and the oracle if they are missing or
    stale; both builds are incremental and take seconds."""
    subprocess.run(["make", "-s", "-C", str(PKG)], check=True)
    subprocess.run(["make", "-s", "-C", str(REPO / "oracle"), "liboracle.so"],
                   check=True)
    yield


def gpu_available():
    try:
        import cgx
        return cgx.lib().cgx_device_count() > 0
    except Exception:
        return False
