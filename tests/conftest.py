import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (ROOT, os.path.join(ROOT, "fo-rma_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernel through the C ABI)")
    config.addinivalue_line("markers", "slow: full-size parity (1080p) cases")


@pytest.fixture(scope="session")
def fr():
    import forma_rt

    forma_rt.lib()
    return forma_rt


@pytest.fixture(scope="session")
def gpu(fr):
    """The product library with at least one HIP device. Fails (does not skip) when
    the device is missing: GPU tests must never pass on a fallback."""
    n = fr.device_count()
    assert n >= 1, "no HIP device visible to libforma_rt"
    return fr
