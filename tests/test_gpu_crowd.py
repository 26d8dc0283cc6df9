"""Parity on seeded random scenes with more top-level objects than one
transposed wave cull pass covers (64): every object kind, n-ary / binary CSG
with half-spaces, transforms over CSG, reflection and refraction, in both
modes (scenes.crowd_scene).

Pinned to the reference: tests/golden/crowd.npz holds the frames and ray
counts of the reference's own hot-path code (oracle/_ref, made by
tests/golden/make_golden.py crowd).  CPU: the oracle reproduces them bit for
bit.  GPU: the device matches the oracle and the fixture, per channel within
1e-5 (paper mode bit-exact), with identical ray counts."""
import json
import os

import numpy as np
import pytest

import scenes

TOL = 1e-5
SEEDS = [1, 2, 3]
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "crowd.npz")


def _gold(seed, mode):
    z = np.load(GOLD)   # data only (allow_pickle stays False)
    return z[f"{seed}/{mode}/fb"], tuple(int(v) for v in z[f"{seed}/{mode}/counts"])


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_matches_reference_fixture(rt, seed, mode):
    sc = rt.load_scene_from_json_text(json.dumps(scenes.crowd_scene(seed)))
    fb, ost = rt.oracle_render(sc, sc.width, sc.height, mode, threads=4)
    gfb, gcounts = _gold(seed, mode)
    assert (ost.rays_intersect, ost.rays_occluded) == gcounts
    assert np.array_equal(fb, gfb)


@pytest.mark.parametrize("seed", SEEDS)
def test_crowd_scene_loads(rt, seed):
    sc = rt.load_scene_from_json_text(json.dumps(scenes.crowd_scene(seed)))
    assert sc.width > 0 and sc.height > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("mode", [0, 1])
def test_crowd_matches_oracle(gpu, seed, mode):
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.crowd_scene(seed)))
    W, H = sc.width, sc.height
    st = gpu.Stats()
    fb = gpu.Tracer(sc, W, H, mode).render(st)
    ref, ost = gpu.oracle_render(sc, W, H, mode, threads=8)
    d = float(np.abs(fb - ref).max())
    print(f"  seed {seed} mode {mode} {W}x{H} max|d|={d:.3g} gpu=({st.rays_intersect},{st.rays_occluded}) "
          f"oracle=({ost.rays_intersect},{ost.rays_occluded})")
    gfb, gcounts = _gold(seed, mode)
    assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded) == gcounts
    if mode == 1:
        assert np.array_equal(fb, ref) and np.array_equal(fb, gfb)
    else:
        assert d <= TOL, d
        assert float(np.abs(fb - gfb).max()) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:1])
def test_crowd_no_cull_same_image(gpu, seed):
    """Culling never changes a result on the crowd scene either."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.crowd_scene(seed)))
    W, H = sc.width, sc.height
    a = gpu.Tracer(sc, W, H, 0).render(gpu.Stats())
    b = gpu.Tracer(sc, W, H, 0, flags=gpu.RT_FLAG_NO_CULL).render(gpu.Stats())
    assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5])
def test_crowd_midres_matches_oracle(gpu, seed):
    """320x240 (more waves per object, so more partial culls) against the
    oracle at run time (no fixture: the oracle is pinned above)."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.crowd_scene(seed, dpi=80)))
    W, H = sc.width, sc.height
    st = gpu.Stats()
    fb = gpu.Tracer(sc, W, H, 0).render(st)
    ref, ost = gpu.oracle_render(sc, W, H, 0, threads=16)
    assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded)
    assert float(np.abs(fb - ref).max()) <= TOL
