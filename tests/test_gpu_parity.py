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


@pytest.mark.gpu
def test_no_cull_flag_same_image(gpu):
    text = SMALL["snorlax"]()
    sc = gpu.load_scene_from_json_text(text)
    a = gpu.Tracer(sc, sc.width, sc.height, 0).render()
    b = gpu.Tracer(sc, sc.width, sc.height, 0, flags=gpu.RT_FLAG_NO_CULL).render()
    assert np.array_equal(a, b)
