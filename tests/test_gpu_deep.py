"""Scenes beyond the common kernels' stacks run on the big-stack kernels
(rt_kernels_big.hip, rt_launch.hpp kBig*) instead of being refused: the
reference recurses without a limit through trace_recursive
(tracer.cpp:22-73), the transform wrappers (transform.cpp:18-255) and binary
csg nodes (json_loader.cpp:354-366).  Each deep scene must match the oracle
(pinned to the reference by tests/golden/deep.npz) to 1e-5 with equal ray
counts, paper mode bit-exact.  Scenes beyond even the big stacks, and the
FP32 fast path on a deep scene, must be refused with RT_ERR_UNSUPPORTED and
a message naming the limit."""
import ctypes as C
import json

import numpy as np
import pytest

import scenes

TOL = 1e-5
RT_ERR_UNSUPPORTED = -6


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(scenes.deep_scenes()))
@pytest.mark.parametrize("mode", [0, 1])
def test_deep_scene_matches_oracle(gpu, name, mode):
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.deep_scenes(dpi=16)[name]))
    W, H = sc.width, sc.height
    st = gpu.Stats()
    fb = gpu.Tracer(sc, W, H, mode).render(st)
    ref, ost = gpu.oracle_render(sc, W, H, mode, threads=8)
    d = float(np.abs(fb - ref).max())
    print(f"  {name} {W}x{H} mode={mode} max|d|={d:.3g} rays=({st.rays_intersect},{st.rays_occluded})")
    assert d <= TOL
    assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded)
    if mode == 1:
        assert np.array_equal(fb, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(scenes.deep_scenes()))
def test_deep_scene_uses_big_stacks(gpu, name):
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.deep_scenes()[name]))
    lib = gpu.amd_lib()
    lib.rt_test_kernel_info.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int32)]
    out = (C.c_int32 * 8)()
    assert lib.rt_test_kernel_info(sc.handle, 0, 0, out) == 0
    assert out[1] > 16384, list(out)   # scratch-resident stacks
    cfg = gpu.load_scene_from_json_text(scenes.config_json(4, dpi=8)[0])
    assert lib.rt_test_kernel_info(cfg.handle, 0, 0, out) == 0
    assert out[1] < 4096, list(out)    # the bench scene keeps the lean kernel


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,mode", [(4, 0), (3, 0), (5, 1), (5, 0)])
def test_trace_kernels_carry_their_shading_pool(gpu, cfg, mode):
    """The light-geometry pool is dynamic LDS sized at launch (10 KiB per
    wave): the occupancy query sees it, and the trace kernels keep four waves
    per SIMD."""
    lib = gpu.amd_lib()
    lib.rt_test_kernel_info.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int32)]
    out = (C.c_int32 * 8)()
    sc = gpu.load_scene_from_json_text(scenes.config_json(cfg, dpi=8)[0])
    assert lib.rt_test_kernel_info(sc.handle, mode, 0, out) == 0
    waves_per_group = out[2] // 10240
    assert waves_per_group >= 1 and out[2] >= 10240 * waves_per_group, list(out)
    assert out[4] == 4, list(out)


def _refused(gpu, text, flags=0):
    sc = gpu.load_scene_from_json_text(text)
    with pytest.raises(gpu.RTError) as e:
        gpu.Tracer(sc, sc.width, sc.height, 0, flags=flags).render()
    assert e.value.code == RT_ERR_UNSUPPORTED
    return str(e.value)


@pytest.mark.gpu
def test_beyond_big_stacks_refused(gpu):
    d = scenes.deep_scenes(dpi=4)["mirrors_rec24"]
    d["medium"]["recursion"] = 400
    msg = _refused(gpu, json.dumps(d))
    assert "exceeds the device stacks" in msg and "medium.recursion 400" in msg
    leaves = [{"sphere": {"position": [0.01 * i, 0, -2], "radius": 0.5, "color": {"diffuse": [1, 1, 1]}}}
              for i in range(80)]
    node = leaves[-1]
    for leaf in reversed(leaves[:-1]):
        node = {"csg": {"operator": "union", "left": leaf, "right": node}}
    msg = _refused(gpu, json.dumps({"screen": {"dpi": 4, "dimensions": [2, 2], "position": [-1, -1, 0],
                                               "observer": [0, 0, 3]}, "objects": [node]}))
    assert "CSG operand depth 80" in msg


@pytest.mark.gpu
def test_fp32_fast_path_refuses_deep_scene(gpu):
    msg = _refused(gpu, json.dumps(scenes.deep_scenes(dpi=4)["csg_right12"]), flags=gpu.RT_FLAG_FP32)
    assert "FP32" in msg
