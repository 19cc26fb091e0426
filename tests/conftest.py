"""Shared test setup: registers the `gpu` marker and puts the product package
(rududu-image-codec_amd/) and the oracle on sys.path."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rududu-image-codec_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: full-size (8K) cases")


def gpu_available():
    try:
        import ric_amd
        return ric_amd.lib().ric_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def ric():
    # device buffers come from the library itself (ric_amd.DeviceArray): no
    # other HIP runtime is loaded into the test process
    import ric_amd
    if ric_amd.lib().ric_device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X (no CPU fallback exists)")
    return ric_amd


@pytest.fixture(scope="session")
def port():
    from oracle import oracle
    return oracle.port()


@pytest.fixture(scope="session")
def ref():
    from oracle import oracle
    return oracle.ref()
