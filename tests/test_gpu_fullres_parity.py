"""Per-pixel parity at the BASELINE.json benchmark sizes (SURVEY.md §8d
configs 2-5 and the native example frames): every channel of the GPU frame,
rendered through the C-ABI (rt_render), against the CPU oracle over the
whole frame on the box's host cores.

Bar (north_star): |d| <= 1e-5 per channel on the FP64 framebuffer, identical
Scene::intersect / Scene::occluded counts, and paper mode bit-exact.  Config 4
(the bench frame, snorlax 3840x2160) is checked with the conservative culling
on (the shipped path) AND off (RT_FLAG_NO_CULL), so a mis-culled object at 4K
fails here even if the ray counts still matched.  Reference loop being
restated: raytracer/src/tracer.cpp:258-300.

Oracle runs take ~1-15 s each at 16 threads on the box; each is computed once
per module and shared by the tests that need it.
"""
import json
import os

import numpy as np
import pytest

import scenes

TOL = 1e-5
THREADS = max(1, min(16, os.cpu_count() or 1))   # the GPU box grants 16 cores to a job

_ORACLE = {}


def _scene(rt, key):
    if key.startswith("cfg"):
        text, mode = scenes.config_json(int(key[3:]))
    else:
        name, m = key.split(":")
        text, mode = json.dumps(scenes.load_example(name)), int(m)
    return rt.load_scene_from_json_text(text), mode


def _oracle(rt, key):
    if key not in _ORACLE:
        sc, mode = _scene(rt, key)
        fb, st = rt.oracle_render(sc, sc.width, sc.height, mode, threads=THREADS)
        _ORACLE[key] = (fb, int(st.rays_intersect), int(st.rays_occluded))
    return _ORACLE[key]


def _check(rt, key, flags=0):
    sc, mode = _scene(rt, key)
    W, H = sc.width, sc.height
    st = rt.Stats()
    fb = rt.Tracer(sc, W, H, mode, flags=flags).render(st)
    ref, ni, no = _oracle(rt, key)
    assert fb.shape == ref.shape == (H, W, 3)
    d = np.abs(fb - ref)
    dmax = float(d.max())
    bad = int(np.count_nonzero(d > TOL))
    exact = float(np.mean(fb == ref))
    print(f"  {key} {W}x{H} flags={flags} max|d|={dmax:.3g} channels>tol={bad} exact={exact:.6f} "
          f"gpu=({st.rays_intersect},{st.rays_occluded}) oracle=({ni},{no})")
    assert np.isfinite(fb).all()
    assert dmax <= TOL, f"{bad} channels above {TOL}, max {dmax}"
    assert (int(st.rays_intersect), int(st.rays_occluded)) == (ni, no)
    if mode == 1:
        assert np.array_equal(fb, ref), "paper mode must be bit-exact"
    return fb


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_config_full_size_matches_oracle(gpu, cfg):
    _check(gpu, f"cfg{cfg}")


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 2], ids=["cull", "no_cull"])
def test_config4_full_size_matches_oracle(gpu, flags):
    """The bench frame itself: snorlax 3840x2160, 5 lights, recursion 4."""
    _check(gpu, "cfg4", flags=flags)


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["penguin:0", "penguin:1", "pokeballs:0", "pokeballs:1", "snorlax:0", "snorlax:1"])
def test_native_example_matches_oracle(gpu, key):
    _check(gpu, key)


@pytest.mark.gpu
def test_config4_counting_pass_with_cull(gpu):
    """bench.py's executed-FLOP pass (RT_FLAG_COUNT_OPS, culling on) at the
    bench frame: the same image and ray counts as the timed kernel's frame."""
    sc, mode = _scene(gpu, "cfg4")
    W, H = sc.width, sc.height
    s0, s1 = gpu.Stats(), gpu.Stats()
    a = gpu.Tracer(sc, W, H, mode).render(s0)
    b = gpu.Tracer(sc, W, H, mode, flags=gpu.RT_FLAG_COUNT_OPS).render(s1)
    assert (s0.rays_intersect, s0.rays_occluded) == (s1.rays_intersect, s1.rays_occluded)
    assert np.array_equal(a, b)
