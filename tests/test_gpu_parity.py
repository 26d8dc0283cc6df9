"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the
same scenes.  Bar (BASELINE.json north_star): per-channel |d| <= 1e-5 on the
FP64 framebuffer, identical Scene::intersect / Scene::occluded counts, and
bit-exact paper-mode output (it only takes the values {0, 0.2, h*(1-darken)})."""
import json

import numpy as np
import pytest

import scenes

TOL = 1e-5

SMALL = {
    "penguin": lambda: json.dumps(scenes.with_dpi(scenes.load_example("penguin"), 24)),
    "pokeballs": lambda: json.dumps(scenes.with_dpi(scenes.load_example("pokeballs"), 24)),
    "snorlax": lambda: json.dumps(scenes.with_dpi(scenes.load_example("snorlax"), 24)),
    "cfg2": lambda: scenes.config_json(2, dpi=24)[0],
    "cfg3": lambda: scenes.config_json(3, dpi=24)[0],
    "cfg4": lambda: scenes.config_json(4, dpi=24)[0],
    "cfg5": lambda: scenes.config_json(5, dpi=24)[0],
}
SMALL.update({k: (lambda v=v: json.dumps(v)) for k, v in scenes.torture_scenes(dpi=20).items()})


def _compare(rt, text, mode):
    sc = rt.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    st = rt.Stats()
    fb = rt.Tracer(sc, W, H, mode).render(st)
    ref, ost = rt.oracle_render(sc, W, H, mode, threads=8)
    d = np.abs(fb - ref)
    exact = float(np.mean(fb == ref))
    print(f"  {W}x{H} mode={mode} max|d|={d.max():.3g} exact={exact:.4f} "
          f"gpu=({st.rays_intersect},{st.rays_occluded}) oracle=({ost.rays_intersect},{ost.rays_occluded})")
    return fb, ref, st, ost


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SMALL))
@pytest.mark.parametrize("mode", [0, 1])
def test_render_matches_oracle(gpu, name, mode):
    fb, ref, st, ost = _compare(gpu, SMALL[name](), mode)
    assert np.abs(fb - ref).max() <= TOL
    assert st.rays_intersect == ost.rays_intersect
    assert st.rays_occluded == ost.rays_occluded
    if mode == 1:
        assert np.array_equal(fb, ref), "paper mode must be bit-exact"


# Mid-resolution frames: more rays through the CSG fast paths and group culls
# (320x180 and up; the oracle runs them in ~1 s on the box's cores).
MID = {
    "cfg4_320": lambda: scenes.config_json(4, dpi=80)[0],
    "cfg3_320": lambda: scenes.config_json(3, dpi=80)[0],
    "snorlax_320": lambda: json.dumps(scenes.with_dpi(scenes.load_example("snorlax"), 80)),
    "csg_ops_240": lambda: json.dumps(scenes.torture_scenes(dpi=60)["csg_ops"]),
    "csg_groups_240": lambda: json.dumps(scenes.torture_scenes(dpi=60)["csg_groups"]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MID))
def test_midres_matches_oracle(gpu, name):
    fb, ref, st, ost = _compare(gpu, MID[name](), 0)
    assert np.abs(fb - ref).max() <= TOL
    assert st.rays_intersect == ost.rays_intersect
    assert st.rays_occluded == ost.rays_occluded


def _odd_size(text, w, h, dpi=16):
    """Same scene and screen centre, a W x H frame that leaves partial waves
    and blocks at the right and bottom edges (W, H exact multiples of 1/dpi)."""
    d = json.loads(text)
    scr = d["screen"]
    dims = scr.get("dimensions", [1, 1])
    cx, cy = scr["position"][0] + dims[0] / 2, scr["position"][1] + dims[1] / 2
    scr["dpi"] = dpi
    scr["dimensions"] = [w / dpi, h / dpi]
    scr["position"] = [cx - w / dpi / 2, cy - h / dpi / 2, scr["position"][2]]
    return json.dumps(d)


# Partial waves (frame edges) take the per-object fallback of the wave-culled
# kernels (WV): scenes with >= 4 bounded objects at sizes that are not
# multiples of the 8x4 / 16x16 pixel blocks.
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg4", "cfg5", "snorlax", "csg_groups"])
@pytest.mark.parametrize("mode", [0, 1])
def test_partial_waves_match_oracle(gpu, name, mode):
    fb, ref, st, ost = _compare(gpu, _odd_size(SMALL[name](), 55, 25), mode)
    assert fb.shape[:2] == (25, 55)
    assert np.abs(fb - ref).max() <= TOL
    assert st.rays_intersect == ost.rays_intersect
    assert st.rays_occluded == ost.rays_occluded
    if mode == 1:
        assert np.array_equal(fb, ref)


@pytest.mark.gpu
def test_no_cull_flag_same_image(gpu):
    text = SMALL["snorlax"]()
    sc = gpu.load_scene_from_json_text(text)
    a = gpu.Tracer(sc, sc.width, sc.height, 0).render()
    b = gpu.Tracer(sc, sc.width, sc.height, 0, flags=gpu.RT_FLAG_NO_CULL).render()
    assert np.array_equal(a, b)


# Counters of the FLOP model (bench.py model_flops).  With
# culling off, the standard-mode kernels execute the reference's primitive
# tests one for one; two counters legitimately differ: Pokeball regions are
# resolved only for the winning hit (lazy hit references) and eager
# (transform-inside-CSG) programs re-run once for the winner.
FLOP_COUNTERS = ["sphere_isect", "sphere_isect_hit", "sphere_ivl", "sphere_ivl_hit", "half_isect", "half_isect_hit",
                 "half_ivl", "xform", "shade_light", "shade_spec", "secondary", "light_eval", "shade_call"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg2", "cfg4", "cfg5", "penguin", "snorlax", "csg_ops", "reflect_refract",
                                  "rotation_scaling", "inside_camera", "halfspace_in_csg"])
def test_opcounts_match_reference_without_cull(gpu, name):
    """bench.py prices roofline.achieved with these counts: they must be the
    reference's own (the oracle counts every Primitive call it restates)."""
    rt = gpu
    sc = rt.load_scene_from_json_text(SMALL[name]())
    W, H = sc.width, sc.height
    st = rt.Stats()
    rt.Tracer(sc, W, H, 0, flags=rt.RT_FLAG_COUNT_OPS | rt.RT_FLAG_NO_CULL).render(st)
    _, ost = rt.oracle_render(sc, W, H, 0, threads=8)
    g = {n: int(st.ops[i]) for i, n in enumerate(rt.OP_NAMES)}
    o = {n: int(ost.ops[i]) for i, n in enumerate(rt.OP_NAMES)}
    assert {n: g[n] for n in FLOP_COUNTERS} == {n: o[n] for n in FLOP_COUNTERS}
    assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_dir_lights_match_oracle(gpu, mode):
    """Scenes with directional lights attached through the IR (the reference's
    loader never creates them) on the general kernels."""
    rt = gpu
    for name, (text, lights) in scenes.dir_light_cases().items():
        sc = rt.with_dir_lights(rt.load_scene_from_json_text(text), lights)
        W, H = sc.width, sc.height
        st = rt.Stats()
        fb = rt.Tracer(sc, W, H, mode).render(st)
        ref, ost = rt.oracle_render(sc, W, H, mode, threads=8)
        assert float(np.abs(fb - ref).max()) <= TOL, name
        if mode == 1:
            assert np.array_equal(fb, ref), name
        assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded), name


# The op-counting kernels (RT_FLAG_COUNT_OPS) take the timed kernels' control
# flow (every lane evaluates each candidate object; counting is gated to the
# reference's calls), so with culling ON they must render the same image and
# count the same rays as the plain render.  bench.py's executed_frac comes
# from exactly this pass.
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg4", "cfg5", "snorlax", "csg_groups", "reflect_refract", "csg_ops"])
@pytest.mark.parametrize("mode", [0, 1])
def test_counting_pass_with_cull_matches_plain(gpu, name, mode):
    sc = gpu.load_scene_from_json_text(SMALL[name]())
    W, H = sc.width, sc.height
    s0, s1 = gpu.Stats(), gpu.Stats()
    a = gpu.Tracer(sc, W, H, mode).render(s0)
    b = gpu.Tracer(sc, W, H, mode, flags=gpu.RT_FLAG_COUNT_OPS).render(s1)
    assert np.array_equal(a, b)
    assert (s0.rays_intersect, s0.rays_occluded) == (s1.rays_intersect, s1.rays_occluded)
    assert s1.ops[gpu.OP_NAMES.index("light_eval")] > 0


# Counters that do not depend on culling (shading calls, light evaluations,
# lit lights, specular terms, reflection / refraction rays) must agree between
# the culled counting kernel (for recursive scenes: trace_wave, where finished
# lanes ride along with valid = false and must count nothing) and the unculled
# one, whose counts equal the reference's (test_opcounts_match_reference_without_cull).
CULL_FREE_OPS = ("shade_call", "light_eval", "shade_light", "shade_spec", "secondary")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg5", "reflect_refract", "snorlax", "cfg4"])
def test_cull_independent_counts_match_unculled(gpu, name):
    sc = gpu.load_scene_from_json_text(SMALL[name]())
    W, H = sc.width, sc.height
    s0, s1 = gpu.Stats(), gpu.Stats()
    a = gpu.Tracer(sc, W, H, 0, flags=gpu.RT_FLAG_COUNT_OPS).render(s0)
    b = gpu.Tracer(sc, W, H, 0, flags=gpu.RT_FLAG_COUNT_OPS | gpu.RT_FLAG_NO_CULL).render(s1)
    assert np.array_equal(a, b)
    for op in CULL_FREE_OPS:
        k = gpu.OP_NAMES.index(op)
        assert s0.ops[k] == s1.ops[k], (op, s0.ops[k], s1.ops[k])
    assert (s0.rays_intersect, s0.rays_occluded) == (s1.rays_intersect, s1.rays_occluded)


@pytest.mark.gpu
def test_counting_pass_with_cull_matches_plain_midres(gpu):
    sc = gpu.load_scene_from_json_text(MID["cfg4_320"]())
    W, H = sc.width, sc.height
    s0, s1 = gpu.Stats(), gpu.Stats()
    a = gpu.Tracer(sc, W, H, 0).render(s0)
    b = gpu.Tracer(sc, W, H, 0, flags=gpu.RT_FLAG_COUNT_OPS).render(s1)
    assert np.array_equal(a, b)
    assert (s0.rays_intersect, s0.rays_occluded) == (s1.rays_intersect, s1.rays_occluded)


# Paper frames of one scene and row set: the first launches the timed primary
# (k_paper_primary_lean<C, WV, true>: wave ticks for the launch order), later
# ones the untimed kernel in costliest-first block order.  Every frame must be
# the oracle's, bit for bit, with the same ray counts.
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg5", "pokeballs", "csg_groups"])
def test_paper_timed_then_ordered_frames_identical(gpu, name):
    rt = gpu
    sc = rt.load_scene_from_json_text(SMALL[name]())
    W, H = sc.width, sc.height
    ref, ost = rt.oracle_render(sc, W, H, 1, threads=8)
    tr = rt.Tracer(sc, W, H, 1)
    for k in range(3):
        st = rt.Stats()
        fb = tr.render(st)
        assert np.array_equal(fb, ref), f"frame {k}"
        assert (st.rays_intersect, st.rays_occluded) == (ost.rays_intersect, ost.rays_occluded), f"frame {k}"
