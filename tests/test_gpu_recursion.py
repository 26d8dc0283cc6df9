"""Reflection / refraction recursion at realistic sizes (Tracer::trace_recursive,
raytracer/src/tracer.cpp:22-73; reflect :38-48, refract :51-68).

No BASELINE config renders bounces in standard mode (the example scenes have
no reflected/refracted materials and config 5 is paper mode), so config 5's
scene (64 spheres, every third reflective, every fifth refractive, 8 lights,
recursion 6) is rendered in STANDARD mode:
  * 960x540 (dpi 240): the case SURVEY.md §6 measured on the reference itself:
    6,199,046 Scene::intersect + 28,798,014 Scene::occluded calls;
  * 3840x2160 (dpi 960): against the all-cores CPU oracle.
Bar: every channel within 1e-5 of the oracle, identical ray counts, culling
on (the shipped path) and off."""
import os

import numpy as np
import pytest

import scenes

TOL = 1e-5
THREADS = max(1, min(16, os.cpu_count() or 1))
REF_960 = (6199046, 28798014)   # SURVEY.md §6 "cfg5 at dpi 240 (extra), std, 960x540", measured on the reference

_ORACLE = {}


def _scene(rt, dpi):
    text, _ = scenes.config_json(5, dpi=dpi)
    return rt.load_scene_from_json_text(text)


def _oracle(rt, dpi):
    if dpi not in _ORACLE:
        sc = _scene(rt, dpi)
        fb, st = rt.oracle_render(sc, sc.width, sc.height, 0, threads=THREADS)
        _ORACLE[dpi] = (fb, int(st.rays_intersect), int(st.rays_occluded))
    return _ORACLE[dpi]


def _check(rt, dpi, flags):
    sc = _scene(rt, dpi)
    W, H = sc.width, sc.height
    st = rt.Stats()
    fb = rt.Tracer(sc, W, H, 0, flags=flags).render(st)
    ref, ni, no = _oracle(rt, dpi)
    d = np.abs(fb - ref)
    print(f"  cfg5 std {W}x{H} flags={flags} max|d|={d.max():.3g} exact={np.mean(fb == ref):.6f} "
          f"gpu=({st.rays_intersect},{st.rays_occluded}) oracle=({ni},{no}) kernel {st.ms_kernel:.3f} ms")
    assert np.isfinite(fb).all()
    assert float(d.max()) <= TOL, f"{int(np.count_nonzero(d > TOL))} channels above {TOL}"
    assert (int(st.rays_intersect), int(st.rays_occluded)) == (ni, no)
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 2], ids=["cull", "no_cull"])
def test_cfg5_standard_960x540_matches_oracle_and_reference_counts(gpu, flags):
    st = _check(gpu, 240, flags)
    assert (int(st.rays_intersect), int(st.rays_occluded)) == REF_960


@pytest.mark.gpu
def test_cfg5_standard_4k_matches_oracle(gpu):
    _check(gpu, 960, 0)


@pytest.mark.gpu
def test_cfg2_recursion6_640x480_matches_oracle(gpu):
    """Config 2's reflective + refractive spheres with recursion 6 at full size."""
    import json

    d = json.loads(scenes.config_json(2)[0])
    d["medium"]["recursion"] = 6
    sc = gpu.load_scene_from_json_text(json.dumps(d))
    W, H = sc.width, sc.height
    st = gpu.Stats()
    fb = gpu.Tracer(sc, W, H, 0).render(st)
    ref, ost = gpu.oracle_render(sc, W, H, 0, threads=THREADS)
    assert float(np.abs(fb - ref).max()) <= TOL
    assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded)
    assert st.ops[gpu.OP_NAMES.index("secondary")] == 0   # (not counted without RT_FLAG_COUNT_OPS)
