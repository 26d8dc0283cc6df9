"""The wave BVH on the host (no GPU): CompiledScene::wobjs / worig / wctab /
wchunk of scenes with more than one wave's 64 objects (scene_compile.cpp
build_wave_bvh), and the reference fixtures of the BVH parity scenes.

Pinned to the reference: tests/golden/bvh.npz holds the frames and ray
counts of the reference's own hot-path code (oracle/_ref, made by
tests/golden/make_golden.py bvh) for scenes.bvh_scenes(16): a 576-sphere
lattice and a scene of exact closest-hit ties (Scene::intersect,
scene.cpp:10-24: spheres accept t == tmax, CSG does not)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import scenes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bvh.npz")
CHUNK = 64


def _gold(name, mode):
    z = np.load(GOLD)   # data only (allow_pickle stays False)
    return z[f"{name}/{mode}/fb"], tuple(int(v) for v in z[f"{name}/{mode}/counts"])


def _bvh(rt, scene):
    amd = rt.amd_lib()
    amd.rt_test_wave_bvh.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_float),
                                     C.c_int, C.POINTER(C.c_float), C.c_int]
    sc = rt.load_scene_from_json_text(json.dumps(scene) if isinstance(scene, dict) else scene)
    counts = (C.c_int32 * 2)()
    assert amd.rt_test_wave_bvh(sc.handle, counts, None, None, 0, None, 0) == 0
    n, nch = counts[0], counts[1]
    worig = (C.c_int32 * max(1, n))()
    wctab = (C.c_float * (8 * max(1, n)))()
    wchunk = (C.c_float * (8 * max(1, nch)))()
    assert amd.rt_test_wave_bvh(sc.handle, counts, worig, wctab, n, wchunk, nch) == 0
    info = (C.c_int32 * 8)()
    amd.rt_test_compile_info.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
    assert amd.rt_test_compile_info(sc.handle, info) == 0
    return {"n": n, "chunks": nch, "n_objs": info[0], "groups": info[1],
            "worig": np.array(worig[:n]), "wctab": np.frombuffer(bytes(wctab), dtype=np.float32).reshape(-1, 8)[:n],
            "wchunk": np.frombuffer(bytes(wchunk), dtype=np.float32).reshape(-1, 8)[:nch],
            "wtype": np.frombuffer(bytes(wctab), dtype=np.int32).reshape(-1, 8)[:n, 4],
            "ctype": np.frombuffer(bytes(wchunk), dtype=np.int32).reshape(-1, 8)[:nch, 4]}


@pytest.mark.parametrize("name", ["grid", "ties"])
@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_matches_reference_fixture(rt, name, mode):
    sc = rt.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(16)[name]))
    fb, ost = rt.oracle_render(sc, sc.width, sc.height, mode, threads=4)
    gfb, gcounts = _gold(name, mode)
    assert (ost.rays_intersect, ost.rays_occluded) == gcounts
    assert np.array_equal(fb, gfb)


def test_tie_order_matters_in_the_reference(rt):
    """The ties scene resolves ties by the reference's object order: reversing
    every pair changes the image (union vs union: the earlier wins; sphere vs
    sphere: the later wins), so the fixture pins the tie rule."""
    s = scenes.bvh_scenes(16)["ties"]
    objs = s["objects"]
    rev = [objs[0]]
    for k in range(1, len(objs), 2):
        rev += [objs[k + 1], objs[k]]
    sc = rt.load_scene_from_json_text(json.dumps(dict(s, objects=rev)))
    fb, _ = rt.oracle_render(sc, sc.width, sc.height, 0, threads=4)
    gfb, _ = _gold("ties", 0)
    assert not np.array_equal(fb, gfb)


@pytest.mark.parametrize("name", ["grid", "ties", "crowd1", "crowd2", "perf"])
def test_wave_bvh_structure(rt, name):
    scene = (scenes.bvh_scenes(16).get(name) or
             (scenes.crowd_scene(int(name[-1]), n_objects=400) if name.startswith("crowd")
              else scenes.bvh_perf_scene(1024, dpi=16)))
    b = _bvh(rt, scene)
    if b["n"] == 0:   # (eager programs: no BVH)
        pytest.skip("scene compiles to eager programs")
    # every object except group headers and never-hit ones, exactly once
    # (entries -1: never-hit padding)
    real = b["worig"][b["worig"] >= 0]
    assert len(real) == len(set(real.tolist())) > 4 * CHUNK
    assert len(real) <= b["n_objs"] - b["groups"]
    assert b["chunks"] == (b["n"] + CHUNK - 1) // CHUNK
    # unbounded objects (types 1, 3) first, padded (type 0) to a chunk
    # boundary, then the bounded ones (type 2)
    t = b["wtype"]
    assert set(t.tolist()) <= {0, 1, 2, 3}
    first_ball = int(np.argmax(t == 2))
    assert first_ball % CHUNK == 0
    assert np.all(t[first_ball:] == 2) and np.all(t[:first_ball] != 2)
    assert np.all(b["worig"][t == 0] == -1) and np.all(b["worig"][t != 0] >= 0)
    # each chunk record encloses its members' f32 balls (type 2), or is "always" (1)
    for c in range(b["chunks"]):
        mem = slice(c * CHUNK, min(b["n"], (c + 1) * CHUNK))
        if b["ctype"][c] == 1:
            assert np.all(t[mem] != 2)
            continue
        assert b["ctype"][c] == 2 and np.all(t[mem] == 2)
        cc, rc = b["wchunk"][c, :3].astype(np.float64), float(b["wchunk"][c, 3])
        m = b["wctab"][mem, :4].astype(np.float64)
        reach = np.linalg.norm(m[:, :3] - cc, axis=1) + m[:, 3]
        assert np.all(reach <= rc * (1 + 1e-6)), (c, float(reach.max()), rc)
    # ball records (objects and chunks) carry |x| + |y| + |z| + r in word 5,
    # rounded up, for the device tests' margins (rt_device.hpp record_touch)
    for rec, typ in ((b["wctab"], t), (b["wchunk"], b["ctype"])):
        balls = rec[typ == 2].astype(np.float64)
        mag = np.abs(balls[:, :3]).sum(axis=1) + balls[:, 3]
        assert np.all(balls[:, 5] >= mag) and np.all(balls[:, 5] <= mag * (1 + 1e-6))


def test_small_scenes_have_no_bvh(rt):
    """Up to four chunks (256 objects) the object test alone is as cheap."""
    assert _bvh(rt, scenes.config_json(4, dpi=8)[0])["n"] == 0      # 15 objects
    assert _bvh(rt, scenes.config_json(5, dpi=8)[0])["n"] == 0      # 65
