import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = os.path.join(ROOT, "opencv_amd", "lib", "libtbdk.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "opencv_amd", "csrc")])
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def gpu():
    """The HIP context for device 0; a GPU test FAILS (not skips) if the
    native library cannot be used, so a silent fallback can never pass."""
    import torch

    assert torch.cuda.is_available(), "gpu-marked test run without a visible HIP device"
    from opencv_amd import klt

    return klt.Context.get(0)
