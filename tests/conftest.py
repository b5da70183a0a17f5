import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def gpu_device():
    """Device ordinal for GPU tests; fails loudly (no CPU fallback) if none is visible."""
    import ctypes

    from dag_rider_amd import _lib

    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.dr_create(4, 1, 8, 0, ctypes.byref(h))
    if rc != 0:
        pytest.fail(f"no usable HIP device: {L.dr_last_error(None).decode()}")
    L.dr_destroy(h)
    return 0
