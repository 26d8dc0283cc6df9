"""Pin the CPU oracle (oracle/oracle.c) to the reference.

Fixtures in tests/golden/*.npz were produced by the reference's own hot-path
sources (oracle/_ref, script tests/golden/make_golden.py).  Everything here is
bit-exact.  Also restates the reference's Catch2 known-answer tests
(raytracer/tests/test_{core,camera,geometry,csg}.cpp) and the quirk values of
SURVEY.md §8c item 5.
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

_dp = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def frames():
    return np.load(os.path.join(GOLDEN, "frames.npz"))


def _scene_names(fr):
    return sorted({k.split("/")[0] for k in fr.files})


def test_frames_fixture_complete(frames):
    names = _scene_names(frames)
    for want in ("penguin", "pokeballs", "snorlax", "cfg2", "cfg5", "csg_ops", "reflect_refract", "xform_in_csg"):
        assert want in names


@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_frames_bit_exact(rt, frames, mode):
    for name in _scene_names(frames):
        text = bytes(frames[f"{name}/scene"]).decode()
        sc = rt.load_scene_from_json_text(text)
        fb, st = rt.oracle_render(sc, sc.width, sc.height, mode, threads=4)
        gold = frames[f"{name}/{mode}/fb"]
        cnt = frames[f"{name}/{mode}/counts"]
        assert np.array_equal(fb, gold), name
        assert (st.rays_intersect, st.rays_occluded) == (int(cnt[0]), int(cnt[1])), name


@pytest.fixture(scope="module")
def kats():
    return np.load(os.path.join(GOLDEN, "kats.npz"))


def _hit_row(h):
    return np.array([h.t, *h.p, *h.n, float(h.mat), float(h.front_face)])


def test_oracle_primitive_kats(rt, kats):
    lib = rt.oracle_lib()
    snames = sorted({k.split("/")[0] for k in kats.files})
    checked = 0
    for sname in snames:
        sc = rt.load_scene_from_json_text(bytes(kats[f"{sname}/scene"]).decode())
        for node in range(sc.desc.n_nodes):
            o = kats[f"{sname}/{node}/o"]
            d = kats[f"{sname}/{node}/d"]
            for tag in ("isect", "isect_win"):
                tmin, tmax = kats[f"{sname}/{node}/{tag}/range"]
                ok_g = kats[f"{sname}/{node}/{tag}/ok"]
                hit_g = kats[f"{sname}/{node}/{tag}/hit"]
                for i in range(len(o)):
                    h = rt.OracleHit()
                    ok = lib.oracle_node_intersect(sc.desc_ptr, node, np.ascontiguousarray(o[i]).ctypes.data_as(_dp),
                                                   np.ascontiguousarray(d[i]).ctypes.data_as(_dp), tmin, tmax,
                                                   C.byref(h))
                    assert ok == ok_g[i], (sname, node, tag, i)
                    if ok:
                        assert np.array_equal(_hit_row(h), hit_g[i]), (sname, node, tag, i)
                    checked += 1
            ok_g = kats[f"{sname}/{node}/ivl/ok"]
            t_g = kats[f"{sname}/{node}/ivl/t"]
            h0_g = kats[f"{sname}/{node}/ivl/h0"]
            h1_g = kats[f"{sname}/{node}/ivl/h1"]
            for i in range(len(o)):
                t0, t1 = C.c_double(), C.c_double()
                h0, h1 = rt.OracleHit(), rt.OracleHit()
                ok = lib.oracle_node_interval(sc.desc_ptr, node, np.ascontiguousarray(o[i]).ctypes.data_as(_dp),
                                              np.ascontiguousarray(d[i]).ctypes.data_as(_dp), C.byref(t0), C.byref(t1),
                                              C.byref(h0), C.byref(h1))
                assert ok == ok_g[i], (sname, node, "ivl", i)
                if ok:
                    assert np.array_equal([t0.value, t1.value], t_g[i]), (sname, node, i)
                    assert np.array_equal(_hit_row(h0), h0_g[i]), (sname, node, i)
                    assert np.array_equal(_hit_row(h1), h1_g[i]), (sname, node, i)
                checked += 1
    assert checked > 10000


def test_oracle_jitter_matches_libstdcxx(rt):
    g = np.load(os.path.join(GOLDEN, "jitter.npz"))
    lib = rt.oracle_lib()
    words = np.zeros(4096, dtype=np.uint32)
    lib.oracle_mt_words(0, 4096, words.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert np.array_equal(words, g["words0"])
    for p, want in zip(g["pixels"], g["draws"]):
        got = np.zeros(16)
        lib.oracle_jitter(16 * int(p), 16, got.ctypes.data_as(_dp))
        assert np.array_equal(got, want), int(p)


def test_oracle_camera_rays(rt):
    import scenes

    g = np.load(os.path.join(GOLDEN, "cameras.npz"))
    lib = rt.oracle_lib()
    for name in g.files:
        sc = rt.load_scene_from_json_text(json.dumps(scenes.load_example(name)))
        for row in g[name]:
            i, j, dx, dy, sub = int(row[0]), int(row[1]), row[2], row[3], int(row[4])
            o = np.zeros(3)
            d = np.zeros(3)
            lib.oracle_camera_ray(sc.desc_ptr, i, j, dx, dy, sub, o.ctypes.data_as(_dp), d.ctypes.data_as(_dp))
            assert np.array_equal(np.concatenate([o, d]), row[5:]), (name, i, j, sub)


# ------------------------------------------------------------------ KATs
MAT = {"diffuse": [1, 0, 0]}


def _scene(objects, **extra):
    s = {"screen": {"position": [-1, -1, 0], "dimensions": [2, 2], "dpi": 100, "observer": [0, 0, 1]},
         "objects": objects}
    s.update(extra)
    return json.dumps(s)


def _isect(rt, sc, node, o, d, tmin=0.001, tmax=1000.0):
    h = rt.OracleHit()
    ok = rt.oracle_lib().oracle_node_intersect(sc.desc_ptr, node, np.array(o, float).ctypes.data_as(_dp),
                                               np.array(d, float).ctypes.data_as(_dp), tmin, tmax, C.byref(h))
    return ok, h


def _ivl(rt, sc, node, o, d):
    t0, t1 = C.c_double(), C.c_double()
    h0, h1 = rt.OracleHit(), rt.OracleHit()
    ok = rt.oracle_lib().oracle_node_interval(sc.desc_ptr, node, np.array(o, float).ctypes.data_as(_dp),
                                              np.array(d, float).ctypes.data_as(_dp), C.byref(t0), C.byref(t1),
                                              C.byref(h0), C.byref(h1))
    return ok, t0.value, t1.value, h0, h1


def test_catch2_sphere(rt):   # test_geometry.cpp:10-46
    sc = rt.load_scene_from_json_text(_scene([{"sphere": {"position": [0, 0, 0], "radius": 1.0, "color": MAT}}]))
    ok, h = _isect(rt, sc, 0, [-2, 0, 0], [1, 0, 0])
    assert ok and h.t == pytest.approx(1.0) and h.p[0] == pytest.approx(-1.0)
    assert tuple(h.n) == pytest.approx((-1.0, 0.0, 0.0))
    ok, _ = _isect(rt, sc, 0, [-2, 2, 0], [1, 0, 0])
    assert not ok


def test_catch2_halfspace(rt):   # test_geometry.cpp:50-85
    sc = rt.load_scene_from_json_text(_scene([
        {"halfSpace": {"position": [0, 0, 0], "normal": [1, 0, 0], "color": MAT}},
        {"halfSpace": {"position": [0, 0, 0], "normal": [3, 4, 0], "color": MAT}}]))
    ok, h = _isect(rt, sc, 0, [-1, 0, 0], [1, 0, 0])
    assert ok and h.t == pytest.approx(1.0) and h.p[0] == pytest.approx(0.0)
    ok, _ = _isect(rt, sc, 0, [1, 0, 0], [0, 1, 0])
    assert not ok   # parallel
    n = np.array(sc.desc.nodes[1].v[3:6])
    assert np.linalg.norm(n) == pytest.approx(1.0)


def test_catch2_pokeball(rt):   # test_geometry.cpp:89-107
    sc = rt.load_scene_from_json_text(_scene([{"pokeball": {"position": [0, 0, 0], "radius": 1.0}}]))
    ok1, top = _isect(rt, sc, 0, [0, 2, 0], [0, -1, 0])
    ok2, bot = _isect(rt, sc, 0, [0, -2, 0], [0, 1, 0])
    assert ok1 and ok2 and top.mat != bot.mat
    assert np.linalg.norm(top.p) == pytest.approx(1.0) and np.linalg.norm(bot.p) == pytest.approx(1.0)


def test_catch2_csg(rt):   # test_csg.cpp:11-46
    sc = rt.load_scene_from_json_text(_scene([
        {"union": [{"sphere": {"position": [-0.5, 0, 0], "radius": 0.7, "color": MAT}},
                   {"sphere": {"position": [0.5, 0, 0], "radius": 0.7, "color": MAT}}]},
        {"difference": [{"sphere": {"position": [0, 0, 0], "radius": 1.0, "color": MAT}},
                        {"sphere": {"position": [0, 0, 0], "radius": 0.5, "color": MAT}}]}]))
    objs = list(sc.desc.objects[:2])
    ok, h = _isect(rt, sc, objs[0], [-2, 0, 0], [1, 0, 0])
    assert ok and h.t < 2.0
    ok, h = _isect(rt, sc, objs[1], [0, 0, -2], [0, 0, 1])
    assert ok


def test_survey_quirks(rt):   # SURVEY.md §8c item 5 (values observed on the reference)
    sc = rt.load_scene_from_json_text(_scene([
        {"difference": [{"sphere": {"position": [0, 0, 0], "radius": 1.0, "color": MAT}},
                        {"sphere": {"position": [0, 0, 0], "radius": 0.5, "color": MAT}}]},
        {"union": [{"sphere": {"position": [0, 0, 0], "radius": 1.0, "color": MAT}},
                   {"halfSpace": {"position": [0, -2, 0], "normal": [0, 1, 0], "color": MAT}}]},
        {"translation": {"factors": [0, 0, 0], "subject": {
            "halfSpace": {"position": [0, 0, 0], "normal": [0, 0, 1], "color": MAT}}}}]))
    diff, uni, trans = list(sc.desc.objects[:3])
    ok, h = _isect(rt, sc, diff, [0, 0, 0], [0, 0, 1], tmin=1e-4, tmax=math.inf)
    assert ok and h.t == 0.5 and h.front_face == 0          # from the centre: inner wall, flipped
    ok, h = _isect(rt, sc, diff, [0, 0, 0.75], [0, 0, -1], tmin=1e-4, tmax=math.inf)
    assert ok and h.t == pytest.approx(1e-4) and tuple(h.n) == (0.0, 0.0, 0.0)   # inside the shell, facing the hollow
    ok, _ = _isect(rt, sc, diff, [0, 0, 0.75], [0, 0, 1], tmin=1e-4, tmax=math.inf)
    assert not ok   # facing out: the sweep exits at a negative event (csg.cpp:136-151) -> no hit
    ok, _ = _isect(rt, sc, uni, [0, 0, 5], [0, 0, -1], tmin=1e-4, tmax=math.inf)
    assert not ok                                            # infinite exit -> no hit
    ok, t0, t1, _, _ = _ivl(rt, sc, trans, [0, 0, -2], [0, 0, 1])
    assert ok and t0 == pytest.approx(2.0) and t1 == pytest.approx(0.0, abs=1e-12)   # projected unbounded exit


def test_catch2_camera(rt):   # test_camera.cpp:9-45
    lib = rt.oracle_lib()
    sc = rt.load_scene_from_json_text(json.dumps(
        {"screen": {"position": [-1, -1, 0], "dimensions": [2, 2], "dpi": 100, "observer": [0, 0, 1]}}))
    W, H = sc.width, sc.height
    o = np.zeros(3)
    d = np.zeros(3)
    lib.oracle_camera_ray(sc.desc_ptr, W // 2, H // 2, 0.0, 0.0, 0, o.ctypes.data_as(_dp), d.ctypes.data_as(_dp))
    assert tuple(o) == pytest.approx((0, 0, 1)) and d[2] < 0
    lib.oracle_camera_ray(sc.desc_ptr, -1, -1, 0.0, 0.0, 0, o.ctypes.data_as(_dp), d.ctypes.data_as(_dp))
    assert d[2] == pytest.approx(-1.0)
    lib.oracle_camera_ray(sc.desc_ptr, 0, 0, 0.0, 0.0, 0, o.ctypes.data_as(_dp), d.ctypes.data_as(_dp))
    assert np.linalg.norm(d) == pytest.approx(1.0)
    sc2 = rt.load_scene_from_json_text(json.dumps({"screen": {"position": [0, 0, 0], "observer": [0, 0, 1]}}))
    assert sc2.desc.camera.dpi == 72


# Full-resolution checksums measured on the reference.
FULL = [
    ("penguin", 0, 1723305.7154781767, 8640000, 25508192),
    ("penguin", 1, 2106634.080000015, 6475800, 3188536),
    ("pokeballs", 0, 1004231.2312431693, 6291456, 21816264),
    ("pokeballs", 1, 1718591.3999999866, 4715008, 2727111),
    ("snorlax", 1, 2555288.6999998926, 6475800, 2943551),
]


@pytest.mark.parametrize("name,mode,checksum,ni,no", FULL)
def test_full_resolution_checksums(rt, name, mode, checksum, ni, no):
    import scenes

    sc = rt.load_scene_from_json_text(json.dumps(scenes.load_example(name)))
    fb, st = rt.oracle_render(sc, sc.width, sc.height, mode, threads=8)
    s = 0.0
    for v in fb.reshape(-1, 3):   # sequential sum over pixels of (r+g+b), as in the survey
        s += v[0] + v[1] + v[2]
    assert s == checksum
    assert (st.rays_intersect, st.rays_occluded) == (ni, no)


@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_dir_lights_bit_exact(rt, mode):
    """Directional lights (shading.cpp:45-76) against frames of the reference
    itself (tests/golden/dirlights.npz, made from oracle/_ref)."""
    import scenes

    gold = np.load(os.path.join(GOLDEN, "dirlights.npz"))
    for name, (text, lights) in scenes.dir_light_cases().items():
        assert np.array_equal(np.array(lights, dtype=np.float64), gold[f"{name}/lights"]), name
        sc = rt.with_dir_lights(rt.load_scene_from_json_text(text), lights)
        assert sc.desc.n_dir_lights == len(lights)
        fb, st = rt.oracle_render(sc, sc.width, sc.height, mode, threads=4)
        assert np.array_equal(fb, gold[f"{name}/{mode}/fb"]), name
        cnt = gold[f"{name}/{mode}/counts"]
        assert (st.rays_intersect, st.rays_occluded) == (int(cnt[0]), int(cnt[1])), name


@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_deep_scenes_bit_exact(rt, mode):
    """Scenes beyond the device's common stacks (scenes.deep_scenes:
    recursion 24, 12 nested transforms, a 12-leaf right-nested csg) against
    frames of the reference itself (tests/golden/deep.npz, make_golden.py)."""
    fr = np.load(os.path.join(GOLDEN, "deep.npz"))
    names = _scene_names(fr)
    assert set(names) == {"mirrors_rec24", "xform_nest12", "csg_right12"}
    for name in names:
        sc = rt.load_scene_from_json_text(bytes(fr[f"{name}/scene"]).decode())
        fb, st = rt.oracle_render(sc, sc.width, sc.height, mode, threads=4)
        assert np.array_equal(fb, fr[f"{name}/{mode}/fb"]), name
        cnt = fr[f"{name}/{mode}/counts"]
        assert (st.rays_intersect, st.rays_occluded) == (int(cnt[0]), int(cnt[1])), name


def test_oracle_cfg5_standard_960_counts_match_reference(rt):
    """SURVEY.md §6 measured the reference on config 5's scene in STANDARD mode
    at dpi 240 (960x540): 6,199,046 intersect + 28,798,014 occluded calls.
    The oracle (the GPU tests' checker for the recursive path at scale)
    reproduces them."""
    import scenes

    sc = rt.load_scene_from_json_text(scenes.config_json(5, dpi=240)[0])
    assert (sc.width, sc.height) == (960, 540)
    _, st = rt.oracle_render(sc, 960, 540, 0, threads=8)
    assert (int(st.rays_intersect), int(st.rays_occluded)) == (6199046, 28798014)
