"""One HIP runtime per process, and the one the product ships on.

librtamd.so links /opt/rocm's libamdhip64 (what `bin/ray` and the INTEGRATION
binding load) and dlopens /opt/rocm's librccl on its first collective
(csrc/device/rccl_dyn.hpp: the one-GPU CLI never maps it).  The GPU tests therefore run without torch (whose
wheel bundles its own HIP runtime under the same soname) and get device
buffers and streams from the library (rt_device_alloc, rt_stream_create), so
the kernels are validated on the runtime the CLI uses."""
import os
import sys

import pytest


@pytest.mark.gpu
def test_single_runtime_is_opt_rocm(gpu):
    assert gpu.device_count() > 0
    assert "torch" not in sys.modules, "the GPU test process must not import torch"
    for stem in ("libamdhip64.so", "libhsa-runtime64.so"):
        paths = gpu.mapped_libraries(stem)
        assert len(paths) == 1, (stem, paths)
        assert paths[0].startswith(gpu.ROCM_DIR + os.sep), (stem, paths)
    # RCCL: loaded on the first collective call (an RCCL unique id here)
    import ctypes as C

    uid = (C.c_uint8 * 128)()
    assert gpu.amd_lib().rt_dist_get_id(uid) == 0, gpu.last_error()
    paths = gpu.mapped_libraries("librccl.so")
    assert len(paths) == 1 and paths[0].startswith(gpu.ROCM_DIR + os.sep), paths
    assert gpu.check_one_hip_runtime().startswith(gpu.ROCM_DIR + os.sep)


@pytest.mark.gpu
def test_cli_uses_the_same_runtime(gpu):
    """bin/ray resolves the same libamdhip64 file (ldd) and does not link
    librccl at all (the library dlopens it for collectives only)."""
    import subprocess

    ray = os.path.join(gpu.BIN_DIR, "ray")
    out = subprocess.run(["ldd", ray], capture_output=True, text=True, check=True).stdout
    libs = {}
    for line in out.splitlines():
        parts = line.split("=>")
        if len(parts) == 2 and parts[1].strip().startswith("/"):
            libs[parts[0].strip()] = os.path.realpath(parts[1].split()[0])
    cli = [p for n, p in libs.items() if n.startswith("libamdhip64.so")]
    assert cli and cli == gpu.mapped_libraries("libamdhip64.so"), (cli, gpu.mapped_libraries("libamdhip64.so"))
    assert not [n for n in libs if n.startswith("librccl.so")], libs


@pytest.mark.gpu
def test_device_buffers_round_trip(gpu):
    import numpy as np

    v = np.arange(1000, dtype=np.float64) * 0.25
    b = gpu.DeviceBuffer(v.nbytes)
    assert not b.to_host(np.float64).any()   # zero-filled
    b.from_host(v)
    assert np.array_equal(b.to_host(np.float64), v)
    b.free()
    s = gpu.Stream()
    s.destroy()
