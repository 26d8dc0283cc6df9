"""Plain-kernel selection (rt_device.hpp CntPlain, rt_render.hip plain_scene):
scenes whose objects are all spheres, half-spaces and pokeballs run the lean /
recursion / paper kernels compiled without transform and CSG code; any
transform or CSG object keeps the general variants.  The choice is host logic
(rt_test_kernel_name compiles the scene and names the kernel a frame would
launch), so this runs without a GPU; the images of both kinds of kernel are
checked against the oracle by the -m gpu parity tests (configs 2, 3, 5 and the
recursion row on plain kernels, config 4 and the torture scenes on general
ones)."""
import ctypes as C
import json

import pytest

import scenes


def _kernel(rt, text, mode, flags=0):
    lib = rt.amd_lib()
    sc = rt.load_scene_from_json_text(text)
    buf = C.create_string_buffer(160)
    assert lib.rt_test_kernel_name(sc.handle, mode, flags, buf, 160) == 0
    return buf.value.decode()


def _args(name):
    return [a.strip() for a in name.split("<", 1)[1].rsplit(">", 1)[0].split(",")]


@pytest.mark.parametrize("cfg,mode,kernel", [
    (2, 0, "k_std_lean"),            # 3 spheres + half-space (per-lane culls)
    (3, 0, "k_std_lean"),            # pokeballs + half-space
    (5, 1, "k_paper_primary_lean"),  # 64 spheres + floor, paper mode
    (5, 0, "k_std_secw"),            # the recursion row: config 5's scene in standard mode
])
def test_plain_scenes_take_the_plain_kernels(rt, cfg, mode, kernel):
    text, _ = scenes.config_json(cfg, dpi=24)
    name = _kernel(rt, text, mode)
    assert name.startswith("rtd::" + kernel + "<"), name
    assert _args(name)[0] == "false" and _args(name)[-1] == "true", name
    # op-counting frames keep the counting (general) variant
    cnt = _kernel(rt, text, mode, rt.RT_FLAG_COUNT_OPS)
    assert _args(cnt)[0] == "true" and _args(cnt)[-1] == "false", cnt


@pytest.mark.parametrize("which", ["rotation_scaling", "csg_ops", "pokeball_csg", "xform_in_csg"])
@pytest.mark.parametrize("mode", [0, 1])
def test_transform_and_csg_scenes_keep_the_general_kernels(rt, which, mode):
    text = json.dumps(scenes.torture_scenes(dpi=12)[which])
    name = _kernel(rt, text, mode)
    if "_lean<" in name or "_secw<" in name:
        assert _args(name)[-1] == "false", name


def test_snorlax_keeps_the_csg_kernel(rt):
    text, _ = scenes.config_json(4, dpi=24)
    name = _kernel(rt, text, 0)
    assert name.startswith("rtd::k_std_lean<false, 1, false>"), name


def test_fp32_build_has_no_plain_variant(rt):
    text, _ = scenes.config_json(5, dpi=24)
    name = _kernel(rt, text, 1, rt.RT_FLAG_FP32)
    assert name.startswith("rtf::") and _args(name)[-1] == "false", name
