"""The wave BVH kernels (k_std_lean<C, 2, PL>, k_std_secw<C, 2, PL>,
k_paper_primary_lean<C, 2, T, PL>: Morton-ordered objects, one transposed test per
64 chunk records before the object tests, closest-hit ties resolved in the
reference's order; DESIGN.md §Wave BVH) against the reference fixtures
(tests/golden/bvh.npz, oracle/_ref), the CPU oracle and the same kernels
without the BVH (RT_FLAG_NO_BVH) and without culling.  Bar: per channel within
1e-5 (paper mode bit-exact), identical ray counts."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import scenes

TOL = 1e-5
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bvh.npz")


def _gold(name, mode):
    z = np.load(GOLD)   # data only (allow_pickle stays False)
    return z[f"{name}/{mode}/fb"], tuple(int(v) for v in z[f"{name}/{mode}/counts"])


def _kernel(rt, sc, mode, flags=0):
    lib = rt.amd_lib()
    buf = C.create_string_buffer(160)
    assert lib.rt_test_kernel_name(sc.handle, mode, flags, buf, 160) == 0
    return buf.value.decode()


def _wv(name):   # the kernel's wave-cull variant (its second template argument)
    return name.split("<", 1)[1].split(",")[1].strip()


def _render(rt, sc, mode, flags=0):
    st = rt.Stats()
    fb = rt.Tracer(sc, sc.width, sc.height, mode, flags=flags).render(st)
    return fb, (int(st.rays_intersect), int(st.rays_occluded))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["grid", "ties"])
@pytest.mark.parametrize("mode", [0, 1])
def test_bvh_matches_reference_fixture(gpu, name, mode):
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(16)[name]))
    k = _kernel(gpu, sc, mode)
    assert _wv(k) == "2", k   # the BVH variant is the one that runs
    fb, counts = _render(gpu, sc, mode)
    gfb, gcounts = _gold(name, mode)
    d = float(np.abs(fb - gfb).max())
    print(f"  {name} mode {mode} {sc.width}x{sc.height} {k} max|d|={d:.3g} rays {counts} ref {gcounts}")
    assert counts == gcounts
    if mode == 1:
        assert np.array_equal(fb, gfb)
    else:
        assert d <= TOL, d


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["grid", "ties"])
@pytest.mark.parametrize("mode", [0, 1])
def test_bvh_equals_no_bvh_and_no_cull(gpu, name, mode):
    """The BVH changes which objects a wave tests and in what order, never a
    result: bit for bit the same frame and ray counts as the wave culls over
    the reference's order, and as no culling at all."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(16)[name]))
    assert _wv(_kernel(gpu, sc, mode, gpu.RT_FLAG_NO_BVH)) == "1"
    a, ca = _render(gpu, sc, mode)
    b, cb = _render(gpu, sc, mode, gpu.RT_FLAG_NO_BVH)
    c, cc = _render(gpu, sc, mode, gpu.RT_FLAG_NO_CULL)
    assert ca == cb == cc
    assert np.array_equal(a, b) and np.array_equal(a, c)


@pytest.mark.gpu
@pytest.mark.parametrize("name,dpi", [("grid", 80), ("ties", 60)])
def test_bvh_midres_matches_oracle(gpu, name, dpi):
    """320x240 / 240x180: many waves per object and chunk, partial chunk culls."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(dpi)[name]))
    fb, counts = _render(gpu, sc, 0)
    ref, ost = gpu.oracle_render(sc, sc.width, sc.height, 0, threads=16)
    d = float(np.abs(fb - ref).max())
    print(f"  {name} {sc.width}x{sc.height} max|d|={d:.3g} exact={np.mean(fb == ref):.6f} rays {counts}")
    assert counts == (int(ost.rays_intersect), int(ost.rays_occluded))
    assert d <= TOL, d


@pytest.mark.gpu
def test_bvh_perf_scene_matches_oracle_small(gpu):
    """The 4096-sphere perf scene (tools/bvh_perf.py) at 64x48."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_perf_scene(4096, dpi=16)))
    assert _wv(_kernel(gpu, sc, 0)) == "2"
    fb, counts = _render(gpu, sc, 0)
    ref, ost = gpu.oracle_render(sc, sc.width, sc.height, 0, threads=16)
    assert counts == (int(ost.rays_intersect), int(ost.rays_occluded))
    assert float(np.abs(fb - ref).max()) <= TOL


@pytest.mark.gpu
def test_bvh_counting_pass_matches_plain(gpu):
    """The op-counting BVH kernel takes the timed kernel's control flow."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(16)["grid"]))
    a, ca = _render(gpu, sc, 0)
    b, cb = _render(gpu, sc, 0, gpu.RT_FLAG_COUNT_OPS)
    assert ca == cb and np.array_equal(a, b)


@pytest.mark.gpu
def test_unbounded_chunk_and_paper_mode(gpu):
    """A floor (unbounded) in its own padded chunk: paper mode of the grid at
    160x120 bit-exact against the oracle, through the BVH kernel."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(40)["grid"]))
    assert _wv(_kernel(gpu, sc, 1)) == "2"
    fb, counts = _render(gpu, sc, 1)
    ref, ost = gpu.oracle_render(sc, sc.width, sc.height, 1, threads=16)
    assert counts == (int(ost.rays_intersect), int(ost.rays_occluded))
    assert np.array_equal(fb, ref)


@pytest.mark.gpu
def test_bvh_counts_every_object_of_every_query(gpu):
    """Op counting with the BVH: every object of every closest-hit query is
    either culled (by its own test or its chunk's) or evaluated, so culled +
    evaluated = queries x objects, with and without the BVH.  (The grid
    without lights: Scene::occluded stops at its first hit, in an order the
    BVH changes, so shadow queries have no such invariant.)"""
    s = scenes.bvh_scenes(16)["grid"]
    s = dict(s, sources=[])
    sc = gpu.load_scene_from_json_text(json.dumps(s))
    n_obj = len(s["objects"])
    totals = []
    for flags in (gpu.RT_FLAG_COUNT_OPS, gpu.RT_FLAG_COUNT_OPS | gpu.RT_FLAG_NO_BVH):
        st = gpu.Stats()
        gpu.Tracer(sc, sc.width, sc.height, 0, flags=flags).render(st)
        ops = st.as_dict()["ops"]
        evaluated = ops["sphere_isect"] + ops["half_isect"]
        totals.append((ops["culled"] + evaluated, int(st.rays_intersect)))
    (t_bvh, q_bvh), (t_flat, q_flat) = totals
    assert q_bvh == q_flat
    assert t_bvh == t_flat == q_bvh * n_obj


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["grid", "ties"])
@pytest.mark.parametrize("mode", [0, 1])
def test_bvh_on_off_trial_frames_identical(gpu, name, mode):
    """Without RT_FLAG_FORCE_BVH / RT_FLAG_NO_BVH the first two frames of a
    frame shape try the BVH on and off and later frames take the faster
    (rt_render.hip SceneCache::bvh_trial): every frame across the switch is
    bit-identical to the forced-BVH and the flat-list frames."""
    sc = gpu.load_scene_from_json_text(json.dumps(scenes.bvh_scenes(40)[name]))
    want, cw = _render(gpu, sc, mode, gpu.RT_FLAG_FORCE_BVH)
    flat, cf = _render(gpu, sc, mode, gpu.RT_FLAG_NO_BVH)
    assert cw == cf and np.array_equal(want, flat)
    t = gpu.Tracer(sc, sc.width, sc.height, mode)
    for i in range(4):
        st = gpu.Stats()
        fb = t.render(st)
        assert np.array_equal(fb, want), i
        assert (int(st.rays_intersect), int(st.rays_occluded)) == cw
