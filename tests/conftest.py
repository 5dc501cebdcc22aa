import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libMiniCVNative.so kernels)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) parity properties")


@pytest.fixture(scope="session")
def oracle():
    import _oracle
    _oracle.load()
    return _oracle


@pytest.fixture(scope="session")
def native():
    from minicv_amd import native as N
    N.lib()
    return N


@pytest.fixture(scope="session")
def gpu(native):
    n = native.lib().mcvDeviceCount()
    if n <= 0:
        pytest.fail("gpu test scheduled but no HIP device visible (the HIP path has no fallback)")
    return n
