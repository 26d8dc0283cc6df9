"""Edge cases of the hot path against the CPU oracle (tracer.cpp:247-305,
shading.cpp:31-138): frames of one row / one column / one pixel (partial
waves and blocks on every edge, paper pixels with fewer than four
neighbours), a scene without objects (every ray misses: background, and in
paper mode the all-miss alphabet), a scene without lights (ambient only), a
scene of unbounded objects only (no cull records: the wave culls have
nothing to test), and distributed frames where some ranks own no rows
(H < world).  Bar as in test_gpu_parity.py: |d| <= 1e-5 per channel and
identical Scene::intersect / Scene::occluded counts; paper frames bit-exact.
"""
import json

import numpy as np
import pytest

import scenes

TOL = 1e-5


def _frame(text, w, h, dpi=16):
    """The scene's screen centre, a w x h frame at dpi."""
    d = json.loads(text)
    scr = d["screen"]
    dims = scr.get("dimensions", [1, 1])
    cx, cy = scr["position"][0] + dims[0] / 2, scr["position"][1] + dims[1] / 2
    scr["dpi"] = dpi
    scr["dimensions"] = [w / dpi, h / dpi]
    scr["position"] = [cx - w / dpi / 2, cy - h / dpi / 2, scr["position"][2]]
    return json.dumps(d)


def _check(rt, text, mode):
    sc = rt.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    st = rt.Stats()
    fb = rt.Tracer(sc, W, H, mode).render(st)
    ref, ost = rt.oracle_render(sc, W, H, mode, threads=4)
    assert fb.shape == ref.shape
    assert np.abs(fb - ref).max() <= TOL
    assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded)
    if mode == 1:
        assert np.array_equal(fb, ref)
    return sc, fb


def _cfg5():
    return scenes.config_json(5, dpi=24)[0]


def _cfg4():
    return scenes.config_json(4, dpi=24)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("wh", [(1, 1), (1, 9), (9, 1), (2, 2), (3, 17)])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("scene", ["cfg4", "cfg5"])
def test_tiny_frames(gpu, scene, mode, wh):
    w, h = wh
    text = _frame(_cfg4() if scene == "cfg4" else _cfg5(), w, h)
    sc, fb = _check(gpu, text, mode)
    assert (sc.width, sc.height) == (w, h)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_scene_without_objects(gpu, mode):
    d = json.loads(_cfg5())
    d["objects"] = []
    sc, fb = _check(gpu, json.dumps(d), mode)
    if mode == 0:
        # every sample misses: acc = bg + ... + bg (8 times, in order) * (1/8) (tracer.cpp:290-296)
        bg = np.array(d["background"], dtype=np.float64)
        acc = np.zeros(3)
        for _ in range(8):
            acc = acc + bg
        assert np.all(fb == acc * (1.0 / 8))
    else:
        assert np.all(fb == 1.0)   # every neighbour agrees (all miss), lum 1: no hatch


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("scene", ["cfg4", "cfg5"])
def test_scene_without_lights(gpu, scene, mode):
    d = json.loads(_cfg4() if scene == "cfg4" else _cfg5())
    d["sources"] = []
    _check(gpu, json.dumps(d), mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_unbounded_objects_only(gpu, mode):
    d = json.loads(_cfg5())
    d["objects"] = [o for o in d["objects"] if "halfSpace" in o] + [
        {"halfSpace": {"position": [0, 0, -9], "normal": [0, 0, 1], "color": {"diffuse": [0.3, 0.5, 0.7]}}}]
    _check(gpu, json.dumps(d), mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("world", [3, 8])
def test_dist_ranks_without_rows(gpu, mode, world):
    """H = 2 rows split over more ranks than rows: the empty ranks still take
    part in every collective, and the frame is rt_render's bit for bit."""
    text = _frame(_cfg5(), 13, 2)
    sc = gpu.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    want = gpu.Tracer(sc, W, H, mode).render()
    out, rc, _, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2)
    assert (rc == 0).all(), msg
    for f in range(2):
        assert np.array_equal(out[f], want), f"frame {f}"
