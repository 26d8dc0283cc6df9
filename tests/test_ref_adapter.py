"""The reference-side binding (integration/rt_ref_adapter.cpp):
the reference's own Scene / Camera objects (raytracer/src/scene.h:32-67,
camera.h:26-79), walked into the C-ABI IR by rtref::scene_from_reference.

Round trip: IR -> the reference's objects built through their public
constructors (oracle/ref_harness.cpp) -> the adapter -> IR'.  IR' must equal IR
(node kinds, parameters bit for bit, CSG operators, transform matrices, the
material identity partition and values, lights including directional ones,
camera, medium) and must render bit-identically on the CPU oracle.  Needs
oracle/_ref (built from /root/reference in this container only)."""
import json
import math
import os

import numpy as np
import pytest

import scenes
from conftest import REPO

REF_SO = os.path.join(REPO, "oracle", "_ref", "libref.so")
pytestmark = pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference)")


def _roundtrip(rt, sc):
    import ctypes as C

    lib = rt.ref_lib()
    out = C.c_void_p()
    rc = lib.ref_roundtrip(sc.desc_ptr, C.byref(out))
    assert rc == 0, rt.last_error()
    return rt.Scene(out.value)


def _canon(d):
    """Canonical form: objects walked in order; materials named by first use."""
    names = {}

    def mat(i):
        if i < 0:
            return None
        if i not in names:
            names[i] = len(names)
        m = d.materials[i]
        return (names[i], tuple(m.albedo), tuple(m.ambient), m.kd, m.ks, m.kr, m.kt, m.shininess, m.refractive_index)

    def node(i):
        n = d.nodes[i]
        k = n.kind
        if k in (0, 1):        # sphere / halfspace
            return (k, tuple(n.v[:6]), mat(n.mat))
        if k == 2:             # pokeball
            return (k, tuple(n.v[:10]), tuple(mat(n.mats[j]) for j in range(5)))
        if k in (3, 4, 5):     # transforms: forward + inverse matrices (what the device reads)
            return (k, tuple(n.v[:24]), n.op if k == 5 else 0, node(n.a))
        return (k, n.op, node(n.a), node(n.b))

    lights = tuple((tuple(l.pos), tuple(l.intensity)) for l in d.lights[:d.n_lights])
    dls = tuple((tuple(l.dir), tuple(l.radiance)) for l in d.dir_lights[:d.n_dir_lights])
    cam = (tuple(d.camera.eye), tuple(d.camera.P), d.camera.Lx, d.camera.Ly, d.camera.dpi)
    return (cam, tuple(d.background), tuple(d.ambient), d.medium_index, d.recursion_limit, lights, dls,
            tuple(node(d.objects[i]) for i in range(d.n_objects)))


def _rotation_angles(d):
    return [(n.op, n.aux[0]) for n in d.nodes[:d.n_nodes] if n.kind == 5]


CASES = {
    "penguin": lambda: json.dumps(scenes.with_dpi(scenes.load_example("penguin"), 12)),
    "pokeballs": lambda: json.dumps(scenes.with_dpi(scenes.load_example("pokeballs"), 12)),
    "snorlax": lambda: json.dumps(scenes.with_dpi(scenes.load_example("snorlax"), 12)),
    "cfg2": lambda: scenes.config_json(2, dpi=12)[0],
    "cfg5": lambda: scenes.config_json(5, dpi=12)[0],
}
CASES.update({k: (lambda v=v: json.dumps(v)) for k, v in scenes.torture_scenes(dpi=10).items()})


@pytest.mark.parametrize("name", sorted(CASES))
def test_adapter_roundtrip_is_identity(rt, name):
    sc = rt.load_scene_from_json_text(CASES[name]())
    back = _roundtrip(rt, sc)
    assert _canon(back.desc) == _canon(sc.desc)
    for (ax0, a0), (ax1, a1) in zip(_rotation_angles(sc.desc), _rotation_angles(back.desc)):
        assert ax0 == ax1 and math.isclose(a0, a1, rel_tol=0, abs_tol=1e-12)
    W, H = sc.width, sc.height
    for mode in (0, 1):
        a, sa = rt.oracle_render(sc, W, H, mode, threads=4)
        b, sb = rt.oracle_render(back, W, H, mode, threads=4)
        assert np.array_equal(a, b), mode
        assert (sa.rays_intersect, sa.rays_occluded) == (sb.rays_intersect, sb.rays_occluded)


def test_adapter_keeps_directional_lights(rt):
    """Scene::dir_lights exist only through the reference's API (the loader
    never fills them): the binding is how they reach the device."""
    for name, (text, lights) in scenes.dir_light_cases().items():
        sc = rt.with_dir_lights(rt.load_scene_from_json_text(text), lights)
        back = _roundtrip(rt, sc)
        assert back.desc.n_dir_lights == len(lights) > 0, name
        assert _canon(back.desc) == _canon(sc.desc), name
        a, _ = rt.oracle_render(sc, sc.width, sc.height, 0, threads=4)
        b, _ = rt.oracle_render(back, sc.width, sc.height, 0, threads=4)
        assert np.array_equal(a, b), name


def test_adapter_material_identity_by_pointer(rt):
    """Two colour blocks with equal values stay two materials (paper-mode edges
    compare Material pointers, tracer.cpp:170); one block shared by reference
    stays one."""
    scene = {"screen": {"dpi": 8, "dimensions": [2, 2], "position": [-1, -1, 0], "observer": [0, 0, 4]},
             "sources": [{"position": [0, 5, 5], "intensity": [10, 10, 10]}],
             "objects": [{"sphere": {"position": [-0.5, 0, -2], "radius": 0.4, "color": {"diffuse": [1, 0, 0]}}},
                         {"sphere": {"position": [0.5, 0, -2], "radius": 0.4, "color": {"diffuse": [1, 0, 0]}}}]}
    sc = rt.load_scene_from_json_text(json.dumps(scene))
    back = _roundtrip(rt, sc)
    assert back.desc.n_materials == 2
    assert _canon(back.desc) == _canon(sc.desc)
