import os
import sys

import pytest

# No torch in the test process: librtamd.so runs on /opt/rocm's HIP runtime
# (the one the `ray` CLI and the INTEGRATION binding use), and every GPU test
# gets its device buffers and streams from the library itself
# (rtamd.DeviceBuffer / rtamd.Stream).  rtamd.amd_lib() refuses a process
# with torch's bundled runtime mapped (two runtimes aborted at exit).

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
