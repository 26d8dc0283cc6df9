import os
import sys

import pytest

# torch first: its bundled HIP runtime (soname libamdhip64.so.7, like
# /opt/rocm's) is then the process's one runtime, as in bench.py and the
# tools.  Loading librtamd.so first and torch later inside a test aborted
# the process at exit (heap corruption in runtime teardown) on the GPU box.
try:
    import torch  # noqa: F401
except ImportError:
    pass

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = os.path.join(REPO, "raytracing-project_amd", "python")
if PY not in sys.path:
    sys.path.insert(0, PY)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def rt():
    import rtamd

    rtamd.host_lib()
    return rtamd


@pytest.fixture(scope="session")
def gpu(rt):
    """The HIP renderer; fails loudly when the extension or device is missing."""
    rt.amd_lib()
    n = rt.device_count()
    assert n > 0, "no HIP device visible: the -m gpu tests must run on an MI355X"
    return rt
