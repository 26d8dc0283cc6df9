"""Scene inputs: the BASELINE.json configs and torture scenes.

Configs (BASELINE.json "configs"):
  1  examples/penguin.json unchanged, 1200x900 (CPU reference path)
  2  640x480 synthetic: 3 spheres + 1 halfSpace, 3 lights, recursion 1
  3  1920x1080 examples/pokeballs.json, 5 lights, recursion 3
  4  3840x2160 examples/snorlax.json (deep CSG), 5 lights, recursion 4
  5  7680x4320 synthetic 64 spheres + floor, 8 lights, recursion 6, --paper

Resize rule: dpi = W/4, dimensions = [4, H/dpi], screen
re-centred on the original screen centre.  Every function returns JSON text
in the reference schema (raytracer/src/json_loader.cpp).
"""
from __future__ import annotations

import copy
import json
import math
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
SCENE_DIR = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "tests", "golden", "scenes")

PENGUIN_LIGHTS = [
    {"position": [5, 6, 8], "intensity": [20, 20, 20]},
    {"position": [-5, 6, 8], "intensity": [15, 15, 15]},
    {"position": [0, 3, 7], "intensity": [12, 12, 12]},
]


def load_example(name: str) -> dict:
    with open(os.path.join(SCENE_DIR, f"{name}.json")) as f:
        return json.load(f)


def resize(scene: dict, width: int, height: int) -> dict:
    """Apply the resize rule: dpi = W/4, dims = [4, H/dpi], same screen centre."""
    s = copy.deepcopy(scene)
    scr = s["screen"]
    dims = scr.get("dimensions", [1, 1])
    P = scr["position"]
    cx, cy = P[0] + dims[0] / 2.0, P[1] + dims[1] / 2.0
    dpi = width // 4
    Ly = height / dpi
    scr["dpi"] = dpi
    scr["dimensions"] = [4, Ly]
    scr["position"] = [cx - 2.0, cy - Ly / 2.0, P[2]]
    return s


def with_dpi(scene: dict, dpi: int) -> dict:
    """Same screen, different dpi (used to make small parity cases)."""
    s = copy.deepcopy(scene)
    s["screen"]["dpi"] = dpi
    return s


def cfg2_scene() -> dict:
    return {
        "screen": {"dpi": 160, "dimensions": [4, 3], "position": [-2, -1.5, 0], "observer": [0, 0, 5]},
        "medium": {"ambient": [0.1, 0.1, 0.1], "index": 1.0, "recursion": 1},
        "background": [0.2, 0.3, 0.5],
        "sources": copy.deepcopy(PENGUIN_LIGHTS),
        "objects": [
            {"halfSpace": {"position": [0, -1, 0], "normal": [0, 1, 0],
                           "color": {"diffuse": [0.6, 0.6, 0.6], "specular": [0.1, 0.1, 0.1], "shininess": 8}}},
            {"sphere": {"position": [-1.2, 0, -2], "radius": 0.8,
                        "color": {"diffuse": [0.9, 0.1, 0.1], "specular": [0.5, 0.5, 0.5], "shininess": 32}}},
            {"sphere": {"position": [0, 0, -3], "radius": 1.0,
                        "color": {"diffuse": [0.1, 0.8, 0.2], "reflected": [0.5, 0.5, 0.5], "shininess": 64}}},
            {"sphere": {"position": [1.2, 0, -2], "radius": 0.8, "index": 1.5,
                        "color": {"diffuse": [0.1, 0.2, 0.9], "refracted": [0.5, 0.5, 0.5], "shininess": 16}}},
        ],
    }


def cfg3_scene() -> dict:
    s = resize(load_example("pokeballs"), 1920, 1080)
    s["medium"]["recursion"] = 3
    return s


def cfg4_scene() -> dict:
    s = resize(load_example("snorlax"), 3840, 2160)
    s["sources"] = s["sources"] + [
        {"position": [0, 8, 2], "intensity": [20, 20, 20]},
        {"position": [3, -1, 6], "intensity": [15, 15, 15]},
    ]
    s["medium"]["recursion"] = 4
    return s


def cfg5_scene() -> dict:
    objs = [{"halfSpace": {"position": [0, -1.6, 0], "normal": [0, 1, 0],
                           "color": {"diffuse": [0.6, 0.6, 0.6], "specular": [0.1, 0.1, 0.1], "shininess": 8}}}]
    for k in range(64):
        i, j = k % 8, k // 8
        col = {"diffuse": [(i + 1) / 9.0, (j + 1) / 9.0, 0.5], "specular": [0.3, 0.3, 0.3],
               "shininess": 16 + 8 * (k % 4)}
        sph = {"position": [-3.5 + i, -1.2 + 0.35 * j, -2.0 - j], "radius": 0.3 + 0.05 * ((i + j) % 3), "color": col}
        if k % 3 == 0:
            col["reflected"] = [0.3, 0.3, 0.3]
        if k % 5 == 0:
            col["refracted"] = [0.4, 0.4, 0.4]
            sph["index"] = 1.5
        objs.append({"sphere": sph})
    lights = [{"position": [6 * math.cos(2 * math.pi * l / 8), 6, 2 + 6 * math.sin(2 * math.pi * l / 8)],
               "intensity": [20, 20, 20]} for l in range(8)]
    return {
        "screen": {"dpi": 1920, "dimensions": [4, 2.25], "position": [-2, -1.125, 0], "observer": [0, 0, 5]},
        "medium": {"ambient": [0.1, 0.1, 0.1], "index": 1.0, "recursion": 6},
        "background": [0.2, 0.3, 0.5],
        "sources": lights,
        "objects": objs,
    }


def bvh_scenes(dpi: int = 16) -> dict[str, dict]:
    """Scenes of more than kWaveBvhMin = 256 objects (no eager programs), for the wave BVH
    (CompiledScene::wobjs; tests/test_gpu_bvh.py):
      grid  576 spheres on a 24 x 24 lattice over a floor (every 5th
            reflective, every 7th refractive), 4 lights;
      ties  exact closest-hit ties between objects of both acceptance rules:
            pairs of coincident spheres, some wrapped in a CSG union with a
            tiny far sphere (its first hit t is the same double as the bare
            sphere's, its bound centre lies far away, so Morton order and the
            reference's order disagree about which of a pair comes first):
            sphere vs union (the sphere wins), union vs union (the earlier
            wins), sphere vs sphere (the later wins), in both orders and
            different colours."""
    def mat(k):
        m = _mat([(k % 7) / 7.0, (k % 5) / 5.0, (k % 3) / 3.0], shininess=8 + 4 * (k % 5))
        if k % 5 == 0:
            m["reflected"] = [0.4, 0.4, 0.4]
        elif k % 7 == 0:
            m["refracted"] = [0.5, 0.5, 0.5]
        return m

    lights = [{"position": [4, 6, 3], "intensity": [30, 30, 30]}, {"position": [-5, 5, 2], "intensity": [20, 20, 20]},
              {"position": [0, 8, -4], "intensity": [15, 15, 15]}, {"position": [2, 1, 4], "intensity": [10, 10, 10]}]
    grid = [{"halfSpace": {"position": [0, -1.4, 0], "normal": [0, 1, 0], "color": _mat([0.6, 0.6, 0.6])}}]
    for k in range(576):
        i, j = k % 24, k // 24
        grid.append({"sphere": {"position": [-3.45 + 0.3 * i, -1.2 + 0.05 * (i % 3), -1.5 - 0.3 * j],
                                "radius": 0.1 + 0.03 * ((i + j) % 3), "color": mat(k), "index": 1.5}})
    ties = [{"halfSpace": {"position": [0, -1.4, 0], "normal": [0, 1, 0], "color": _mat([0.5, 0.5, 0.5])}}]
    for k in range(150):
        i, j = k % 15, k // 15
        c = [-3.5 + 0.5 * i, -1.0 + 0.3 * j, -2.5 - 0.5 * j]
        r = 0.18 + 0.04 * (k % 3)

        def bare(col):
            return {"sphere": {"position": list(c), "radius": r, "color": _mat(col)}}

        def wrapped(col, side):
            far = {"sphere": {"position": [c[0] + 40.0 * side, c[1] + 30.0, c[2] - 60.0], "radius": 0.01,
                              "color": _mat([0.5, 0.5, 0.5])}}
            return {"union": [{"sphere": {"position": list(c), "radius": r, "color": _mat(col)}}, far]}

        if k % 3 == 0:     # sphere vs union: the sphere wins either way
            pair = [bare([1.0, 0.1, 0.1]), wrapped([0.1, 1.0, 0.1], 1)]
        elif k % 3 == 1:   # union vs union: the earlier one wins
            pair = [wrapped([0.1, 1.0, 0.1], 1), wrapped([0.1, 0.1, 1.0], -1)]
        else:              # sphere vs sphere: the later one wins
            pair = [bare([1.0, 0.1, 0.1]), bare([1.0, 1.0, 0.1])]
        ties += pair if (k // 3) % 2 == 0 else pair[::-1]
    return {"grid": _base(grid, recursion=3, dpi=dpi, lights=lights),
            "ties": _base(ties, recursion=2, dpi=dpi, lights=lights[:2])}


def bvh_perf_scene(n: int = 4096, seed: int = 7, dpi: int = 480) -> dict:
    """n random spheres (seeded) over a floor, 4 lights, recursion 1, at
    dpi 480 (1920x1080): the wave BVH's perf case (tools/bvh_perf.py)."""
    import random
    rnd = random.Random(seed)
    objs = [{"halfSpace": {"position": [0, -1.4, 0], "normal": [0, 1, 0], "color": _mat([0.6, 0.6, 0.6])}}]
    for _ in range(n):
        objs.append({"sphere": {"position": [rnd.uniform(-6, 6), rnd.uniform(-1.3, 2.5), rnd.uniform(-14, -1.5)],
                                "radius": rnd.uniform(0.03, 0.12),
                                "color": _mat([rnd.random(), rnd.random(), rnd.random()], shininess=rnd.choice([8, 16, 32]))}})
    lights = [{"position": [4, 6, 3], "intensity": [30, 30, 30]}, {"position": [-5, 5, 2], "intensity": [20, 20, 20]},
              {"position": [0, 8, -4], "intensity": [15, 15, 15]}, {"position": [2, 1, 4], "intensity": [10, 10, 10]}]
    return _base(objs, recursion=1, dpi=dpi, lights=lights)


CONFIGS = {
    1: ("penguin 1200x900 (config 1)", lambda: load_example("penguin"), 0),
    2: ("synthetic 640x480 3 spheres + halfSpace, 3 lights, rec 1 (config 2)", cfg2_scene, 0),
    3: ("pokeballs 1920x1080, 5 lights, rec 3 (config 3)", cfg3_scene, 0),
    4: ("snorlax 3840x2160, 5 lights, rec 4 (config 4)", cfg4_scene, 0),
    5: ("synthetic 7680x4320 64 spheres, 8 lights, rec 6, paper (config 5)", cfg5_scene, 1),
    # not a BASELINE config: config 5's scene in STANDARD mode at 3840x2160, the
    # reflection / refraction recursion (tracer.cpp:22-73) at scale
    6: ("config-5 scene, standard mode 3840x2160, 8 lights, rec 6 (recursion row)",
        lambda: with_dpi(cfg5_scene(), 960), 0),
}


def config_json(n: int, dpi: int | None = None) -> tuple[str, int]:
    """(json_text, mode) for config n, optionally at a reduced dpi."""
    _, fn, mode = CONFIGS[n]
    s = fn()
    if dpi is not None:
        s = with_dpi(s, dpi)
    return json.dumps(s), mode


# ------------------------------------------------------------- torture scenes
def _mat(d, **kw):
    m = {"diffuse": list(d), "ambient": [0.05, 0.05, 0.05], "specular": [0.4, 0.4, 0.4], "shininess": 24}
    m.update(kw)
    return m


def _base(objects, recursion=3, dpi=24, lights=None):
    return {
        "screen": {"dpi": dpi, "dimensions": [4, 3], "position": [-2, -1.5, 0], "observer": [0, 0.3, 5]},
        "medium": {"ambient": [0.2, 0.2, 0.2], "index": 1.0, "recursion": recursion},
        "background": [0.3, 0.4, 0.6],
        "sources": lights or copy.deepcopy(PENGUIN_LIGHTS),
        "objects": objects,
    }


def torture_scenes(dpi: int = 24) -> dict[str, dict]:
    """Scenes covering every node kind, the CSG/transform quirks and recursion."""
    floor = {"halfSpace": {"position": [0, -1.2, 0], "normal": [0, 1, 0], "color": _mat([0.5, 0.6, 0.5])}}
    sc = {}
    sc["rotation_scaling"] = _base([
        floor,
        {"rotation": {"angle": 30, "direction": 1, "subject": {
            "scaling": {"factors": [1.5, 0.6, 1.0], "subject": {
                "sphere": {"position": [0, 0, 0], "radius": 0.8, "color": _mat([0.8, 0.3, 0.2])}}}}}},
        {"rotation": {"angle": -45, "direction": 2, "subject": {
            "translation": {"factors": [1.6, 0.2, -1.0], "subject": {
                "sphere": {"position": [0, 0, 0], "radius": 0.5, "color": _mat([0.2, 0.3, 0.9])}}}}}},
        {"rotation": {"angle": 60, "direction": 0, "subject": {
            "sphere": {"position": [-1.6, 0.3, -1.5], "radius": 0.6, "color": _mat([0.9, 0.9, 0.2])}}}},
    ], dpi=dpi)
    sc["csg_ops"] = _base([
        floor,
        {"intersection": [
            {"sphere": {"position": [-1.5, 0, -1], "radius": 0.9, "color": _mat([0.9, 0.2, 0.2])}},
            {"sphere": {"position": [-1.0, 0, -1], "radius": 0.9, "color": _mat([0.2, 0.9, 0.2])}}]},
        {"difference": [
            {"sphere": {"position": [0.3, 0.2, -1.5], "radius": 1.0, "color": _mat([0.9, 0.8, 0.2])}},
            {"sphere": {"position": [0.3, 0.2, -0.6], "radius": 0.6, "color": _mat([0.2, 0.2, 0.9])}},
            {"sphere": {"position": [0.9, 0.8, -1.0], "radius": 0.4, "color": _mat([0.7, 0.2, 0.7])}}]},
        {"csg": {"operator": "union",
                 "left": {"sphere": {"position": [1.8, -0.4, -1], "radius": 0.5, "color": _mat([0.3, 0.7, 0.9])}},
                 "right": {"union": [
                     {"sphere": {"position": [1.8, 0.3, -1], "radius": 0.35, "color": _mat([0.9, 0.5, 0.1])}},
                     {"sphere": {"position": [2.2, 0.0, -1], "radius": 0.3, "color": _mat([0.5, 0.9, 0.1])}}]}}},
    ], dpi=dpi)
    sc["halfspace_in_csg"] = _base([
        {"intersection": [
            {"sphere": {"position": [0, 0, -1.5], "radius": 1.2, "color": _mat([0.8, 0.4, 0.3])}},
            {"halfSpace": {"position": [0, 0.2, 0], "normal": [0.3, -1, 0.2], "color": _mat([0.3, 0.8, 0.4])}}]},
        {"difference": [
            {"sphere": {"position": [1.7, 0.3, -1.0], "radius": 0.7, "color": _mat([0.4, 0.4, 0.9])}},
            {"halfSpace": {"position": [1.7, 0.3, -1.0], "normal": [1, 1, 0], "color": _mat([0.9, 0.9, 0.9])}}]},
        {"union": [
            {"sphere": {"position": [-1.8, 0.0, -1.0], "radius": 0.5, "color": _mat([0.9, 0.9, 0.3])}},
            {"halfSpace": {"position": [0, -1.3, 0], "normal": [0, 1, 0], "color": _mat([0.4, 0.5, 0.4])}}]},
        {"translation": {"factors": [0.0, -0.2, 0.0], "subject": {
            "halfSpace": {"position": [0, -1.0, -6], "normal": [0, 0, 1], "color": _mat([0.5, 0.5, 0.7])}}}},
    ], dpi=dpi)
    sc["pokeball_csg"] = _base([
        floor,
        {"pokeball": {"position": [-1.2, 0, -1], "radius": 0.8, "button_dir": [0.2, 0.1, 1.0]}},
        {"difference": [
            {"pokeball": {"position": [1.2, 0, -1], "radius": 0.8, "button_dir": [-0.3, 0.2, 1.0],
                          "belt_half": 0.1, "button_outer": 0.35, "ring_width": 0.08}},
            {"sphere": {"position": [1.6, 0.5, -0.4], "radius": 0.4, "color": _mat([0.2, 0.2, 0.2])}}]},
        {"scaling": {"factors": [0.5, 0.5, 0.5], "subject": {
            "pokeball": {"position": [0, -1.6, -1], "radius": 0.8}}}},
    ], dpi=dpi)
    sc["reflect_refract"] = _base([
        floor,
        {"sphere": {"position": [-1.2, 0, -1.5], "radius": 0.7,
                    "color": _mat([0.2, 0.2, 0.2], reflected=[0.8, 0.8, 0.8])}},
        {"sphere": {"position": [0.3, -0.1, -0.8], "radius": 0.6, "index": 1.5,
                    "color": _mat([0.1, 0.1, 0.1], refracted=[0.9, 0.9, 0.9], reflected=[0.1, 0.1, 0.1])}},
        {"sphere": {"position": [1.6, 0.1, -1.2], "radius": 0.5, "index": 2.4,
                    "color": _mat([0.3, 0.1, 0.1], refracted=[0.7, 0.7, 0.7])}},
        {"difference": [
            {"sphere": {"position": [0.0, 1.0, -2.5], "radius": 0.6, "index": 1.3,
                        "color": _mat([0.5, 0.5, 0.8], refracted=[0.6, 0.6, 0.6], reflected=[0.3, 0.3, 0.3])}},
            {"sphere": {"position": [0.0, 1.0, -2.5], "radius": 0.3, "color": _mat([0.9, 0.2, 0.2])}}]},
    ], recursion=6, dpi=dpi)
    t_sph = {"translation": {"factors": [-1.2, 0.2, -1.0], "subject": {
        "sphere": {"position": [0, 0, 0], "radius": 0.6, "color": _mat([0.8, 0.3, 0.3])}}}}
    r_sph = {"rotation": {"angle": 35, "direction": 2, "subject": {"scaling": {"factors": [1.6, 0.5, 0.8], "subject": {
        "sphere": {"position": [-0.5, 0, -1.2], "radius": 0.5, "color": _mat([0.3, 0.8, 0.3])}}}}}}
    t_half = {"translation": {"factors": [0.0, 0.3, 0.0], "subject": {
        "halfSpace": {"position": [1.3, 0.0, -1.0], "normal": [0, 1, 0.2], "color": _mat([0.9, 0.9, 0.9])}}}}
    s_poke = {"scaling": {"factors": [1.0, 2.0, 1.0], "subject": {
        "pokeball": {"position": [0.0, 0.4, -2.5], "radius": 0.5, "button_dir": [0, 0, 1]}}}}
    sc["xform_in_csg"] = _base([
        floor,
        {"union": [t_sph, r_sph]},
        {"difference": [{"sphere": {"position": [1.3, 0.0, -1.0], "radius": 0.8, "color": _mat([0.3, 0.3, 0.9])}},
                        t_half]},
        {"intersection": [s_poke,
                          {"sphere": {"position": [0.0, 0.9, -2.5], "radius": 0.7, "color": _mat([0.9, 0.6, 0.2])}}]},
    ], dpi=dpi)
    def _cluster(cx, cy, cz, r, n, col, spread=0.18):
        out = []
        for i in range(n):
            a = 2.399963 * i
            out.append({"sphere": {"position": [cx + spread * math.cos(a), cy + spread * math.sin(a), cz + 0.05 * i],
                                   "radius": r * (1.0 - 0.08 * i), "color": _mat(col)}})
        return out
    # n-ary folds with runs of small spheres: OP_IVL_GROUP culling inside the
    # CSG program (scene_compile.cpp emit_compact_ivl) for all three operators
    sc["csg_groups"] = _base([
        floor,
        {"translation": {"factors": [-1.3, 0.1, -0.5], "subject": {"union": [
            {"sphere": {"position": [0, 0, -1], "radius": 0.7, "color": _mat([0.2, 0.5, 0.5])}},
            *_cluster(0.0, 0.75, -0.8, 0.12, 5, [0.9, 0.9, 0.9]),
            {"pokeball": {"position": [0.6, -0.5, -0.7], "radius": 0.2, "button_dir": [0, 0, 1]}},
            *_cluster(-0.6, -0.4, -0.6, 0.08, 4, [0.3, 0.2, 0.1], spread=0.1),
            {"halfSpace": {"position": [0, -0.55, 0], "normal": [0, -1, 0], "color": _mat([0.5, 0.5, 0.5])}},
            *_cluster(0.5, 0.4, -0.5, 0.1, 3, [0.8, 0.2, 0.2], spread=0.12)]}}},
        {"difference": [
            {"sphere": {"position": [1.2, 0.1, -1.2], "radius": 0.8, "color": _mat([0.8, 0.7, 0.3])}},
            *_cluster(1.2, 0.1, -0.45, 0.22, 6, [0.2, 0.2, 0.8], spread=0.35),
            *_cluster(1.7, 0.6, -1.0, 0.15, 3, [0.2, 0.8, 0.2], spread=0.1)]},
        {"intersection": [
            {"sphere": {"position": [0.0, -0.6, -0.4], "radius": 0.45, "color": _mat([0.7, 0.3, 0.7])}},
            {"sphere": {"position": [0.15, -0.5, -0.4], "radius": 0.45, "color": _mat([0.3, 0.7, 0.7])}},
            {"sphere": {"position": [-0.1, -0.45, -0.35], "radius": 0.4, "color": _mat([0.7, 0.7, 0.3])}},
            {"sphere": {"position": [0.05, -0.7, -0.45], "radius": 0.42, "color": _mat([0.5, 0.5, 0.5])}}]},
    ], dpi=dpi)
    sc["csg_groups_inside"] = {
        # eye inside an n-ary union whose later operands are grouped
        "screen": {"dpi": dpi, "dimensions": [4, 3], "position": [-2, -1.5, 0], "observer": [0, 0, 1]},
        "medium": {"ambient": [0.3, 0.3, 0.3], "index": 1.0, "recursion": 2},
        "background": [0.1, 0.1, 0.1],
        "sources": [{"position": [0, 0.5, 0.5], "intensity": [5, 5, 5]}],
        "objects": [
            {"union": [
                {"sphere": {"position": [0, 0, 1], "radius": 3.0, "color": _mat([0.6, 0.5, 0.4])}},
                *_cluster(0.3, 0.2, -1.5, 0.25, 5, [0.2, 0.5, 0.9], spread=0.4),
                *_cluster(-1.0, -0.6, -1.0, 0.2, 3, [0.9, 0.5, 0.2], spread=0.2)]},
            {"difference": [
                {"sphere": {"position": [0, 0, 1], "radius": 2.5, "color": _mat([0.4, 0.6, 0.4])}},
                *_cluster(0.0, 0.0, 1.0, 0.3, 4, [0.9, 0.9, 0.2], spread=0.2)]},
        ],
    }
    sc["recursion0"] = copy.deepcopy(sc["reflect_refract"])
    sc["recursion0"]["medium"]["recursion"] = 0
    sc["inside_camera"] = {
        # eye inside a CSG union and inside a sphere: origin-inside paths (csg.cpp:113-122)
        "screen": {"dpi": dpi, "dimensions": [4, 3], "position": [-2, -1.5, 0], "observer": [0, 0, 1]},
        "medium": {"ambient": [0.3, 0.3, 0.3], "index": 1.0, "recursion": 2},
        "background": [0.1, 0.1, 0.1],
        "sources": [{"position": [0, 0.5, 0.5], "intensity": [5, 5, 5]}],
        "objects": [
            {"union": [
                {"sphere": {"position": [0, 0, 1], "radius": 3.0, "color": _mat([0.6, 0.5, 0.4])}},
                {"sphere": {"position": [0, 0, -3], "radius": 1.0, "color": _mat([0.2, 0.5, 0.4])}}]},
            {"sphere": {"position": [0.5, 0, -1], "radius": 0.5, "color": _mat([0.9, 0.1, 0.1])}},
        ],
    }
    return sc


def deep_scenes(dpi: int = 12) -> dict[str, dict]:
    """Valid scenes beyond the common kernels' stacks (rt_launch.hpp): the
    reference recurses without a limit through trace_recursive
    (tracer.cpp:22-73), the transform wrappers (transform.cpp:18-255) and
    binary csg nodes (json_loader.cpp:354-366); the device runs these on its
    big-stack kernels.
      mirrors_rec24   reflective floor + ceiling, medium.recursion 24 (23 frames)
      xform_nest12    a sphere under 12 nested transforms inside a CSG operand
                      (eager program, ray stack 12) and as a bare chain
      csg_right12     a 12-leaf right-nested binary csg (interval stack 12)"""
    lights = [{"position": [0.0, 1.0, 2.0], "intensity": [6, 6, 6]},
              {"position": [-1.5, 0.5, -1.0], "intensity": [4, 3, 3]}]
    sc = {}
    sc["mirrors_rec24"] = _base([
        {"halfSpace": {"position": [0, -1.2, 0], "normal": [0, 1, 0],
                       "color": _mat([0.2, 0.3, 0.2], reflected=[0.85, 0.85, 0.85])}},
        {"halfSpace": {"position": [0, 1.6, 0], "normal": [0, -1, 0],
                       "color": _mat([0.3, 0.2, 0.2], reflected=[0.8, 0.8, 0.8])}},
        {"sphere": {"position": [-0.8, 0.0, -1.5], "radius": 0.6, "color": _mat([0.8, 0.5, 0.2])}},
        {"sphere": {"position": [0.9, 0.2, -2.0], "radius": 0.5, "index": 1.4,
                    "color": _mat([0.1, 0.1, 0.3], refracted=[0.8, 0.8, 0.8])}},
    ], recursion=24, dpi=dpi, lights=lights)

    def nest(leaf, n):
        node = leaf
        for k in range(n):
            if k % 3 == 0:
                node = {"translation": {"factors": [0.03 * (1 - 2 * (k % 2)), 0.02, 0.0], "subject": node}}
            elif k % 3 == 1:
                node = {"rotation": {"angle": 8 + k, "direction": k % 3, "subject": node}}
            else:
                node = {"scaling": {"factors": [1.03, 0.97, 1.01], "subject": node}}
        return node

    sc["xform_nest12"] = _base([
        {"halfSpace": {"position": [0, -1.2, 0], "normal": [0, 1, 0], "color": _mat([0.5, 0.6, 0.5])}},
        {"union": [nest({"sphere": {"position": [-0.9, 0.0, -1.0], "radius": 0.6, "color": _mat([0.8, 0.3, 0.3])}},
                        12),
                   {"sphere": {"position": [-0.2, 0.5, -1.4], "radius": 0.4, "color": _mat([0.3, 0.3, 0.8])}}]},
        nest({"sphere": {"position": [1.0, 0.0, -1.2], "radius": 0.5, "color": _mat([0.3, 0.8, 0.3])}}, 12),
    ], dpi=dpi)

    def right_nested(leaves, ops):
        node = leaves[-1]
        for leaf, op in zip(reversed(leaves[:-1]), reversed(ops)):
            node = {"csg": {"operator": op, "left": leaf, "right": node}}
        return node

    leaves = [{"sphere": {"position": [-1.6 + 0.3 * i, 0.25 * math.sin(i), -1.2 - 0.1 * i], "radius": 0.35 + 0.02 * i,
                          "color": _mat([0.2 + 0.06 * i, 0.8 - 0.05 * i, 0.4])}} for i in range(12)]
    ops = ["union"] * 5 + ["difference"] + ["union"] * 3 + ["intersection"] + ["union"]
    sc["csg_right12"] = _base([
        {"halfSpace": {"position": [0, -1.2, 0], "normal": [0, 1, 0], "color": _mat([0.5, 0.6, 0.5])}},
        right_nested(leaves, ops),
    ], dpi=dpi)
    return sc


def dir_light_cases(dpi: int = 16) -> dict[str, tuple[str, list]]:
    """Scenes with directional lights (the reference's Scene::dir_lights,
    scene.h:10-15; its loader never creates them, so they are attached to the
    IR: rtamd.with_dir_lights).  Cases: a sun and a back light beside point
    lights, a zero direction (Vec4::normalized's (0,1,0) fallback,
    core.h:58-64), the deep-CSG scene, and reflection/refraction recursion."""
    sun = ([-0.4, -1.0, -0.3], [0.9, 0.85, 0.8])
    back = ([0.0, 0.3, 1.0], [0.3, 0.3, 0.5])       # from behind the camera's view: mostly ndotl <= 0
    zero = ([0.0, 0.0, 0.0], [0.2, 0.2, 0.2])
    tort = torture_scenes(dpi=dpi)
    return {
        "cfg2_sun_back": (config_json(2, dpi=dpi)[0], [sun, back]),
        "cfg2_zero_dir": (config_json(2, dpi=dpi)[0], [zero]),
        "snorlax_sun": (json.dumps(with_dpi(load_example("snorlax"), dpi)), [sun]),
        "reflect_refract_sun": (json.dumps(tort["reflect_refract"]), [sun, back]),
        "pokeball_csg_sun": (json.dumps(tort["pokeball_csg"]), [sun]),
    }


def crowd_scene(seed: int, n_objects: int = 150, dpi: int = 16) -> dict:
    """A seeded random scene with more top-level objects than one wave's
    transposed cull test covers (64 per pass): spheres (some reflective or
    refractive), pokeballs, n-ary and binary CSG of spheres (with a half-space
    now and then), transforms over spheres and CSG, bare half-spaces; 4 point
    lights, recursion 3.  Exercises the multi-pass wave culling, groups and
    the fold / compact / eager CSG paths together (tests/test_gpu_crowd.py)."""
    import random
    rnd = random.Random(seed)

    def col():
        m = _mat([rnd.random(), rnd.random(), rnd.random()], shininess=rnd.choice([4, 8, 16, 32]))
        u = rnd.random()
        if u < 0.12:
            m["reflected"] = [0.5, 0.5, 0.5]
        elif u < 0.2:
            m["refracted"] = [0.6, 0.6, 0.6]
        return m

    def pos(spread=3.0):
        return [rnd.uniform(-spread, spread), rnd.uniform(-1.0, 1.8), rnd.uniform(-7.0, -0.5)]

    def sphere(p=None, r=None):
        return {"sphere": {"position": p or pos(), "radius": r or rnd.uniform(0.08, 0.45), "color": col(),
                           "index": rnd.choice([1.0, 1.33, 1.5])}}

    def csg():
        c = pos()
        leaves = [sphere([c[0] + rnd.uniform(-0.3, 0.3), c[1] + rnd.uniform(-0.3, 0.3), c[2] + rnd.uniform(-0.3, 0.3)],
                         rnd.uniform(0.1, 0.4)) for _ in range(rnd.randint(2, 6))]
        op = rnd.choice(["union", "union", "difference", "intersection"])
        if op != "union" and rnd.random() < 0.3:
            # (a half-space only where the CSG stays bounded: a union with one
            # would contain the camera and reduce every pixel to the
            # origin-inside entry)
            leaves.append({"halfSpace": {"position": c, "normal": [rnd.uniform(-1, 1), 1.0, rnd.uniform(-1, 1)],
                                         "color": col()}})
        if rnd.random() < 0.3 and len(leaves) >= 2:
            return {"csg": {"operator": op, "left": leaves[0], "right": {"union": leaves[1:]} if len(leaves) > 2
                            else leaves[1]}}
        return {op: leaves}

    def xform(sub):
        k = rnd.randint(0, 2)
        if k == 0:
            return {"translation": {"factors": [rnd.uniform(-0.5, 0.5) for _ in range(3)], "subject": sub}}
        if k == 1:
            return {"rotation": {"angle": rnd.uniform(-60, 60), "direction": rnd.randint(0, 2), "subject": sub}}
        return {"scaling": {"factors": [rnd.uniform(0.6, 1.4) for _ in range(3)], "subject": sub}}

    objs = [{"halfSpace": {"position": [0, -1.3, 0], "normal": [0, 1, 0], "color": col()}}]
    while len(objs) < n_objects:
        u = rnd.random()
        if u < 0.5:
            objs.append(sphere())
        elif u < 0.58:
            objs.append({"pokeball": {"position": pos(), "radius": rnd.uniform(0.15, 0.4),
                                      "button_dir": [rnd.uniform(-1, 1), rnd.uniform(-1, 1), 1.0]}})
        elif u < 0.8:
            objs.append(csg())
        elif u < 0.97:
            objs.append(xform(rnd.choice([sphere(), csg()])))
        else:
            objs.append({"halfSpace": {"position": [0, 0, -9], "normal": [rnd.uniform(-0.2, 0.2), 0, 1], "color": col()}})
    lights = [{"position": [rnd.uniform(-6, 6), rnd.uniform(3, 7), rnd.uniform(-2, 6)],
               "intensity": [rnd.uniform(8, 25)] * 3} for _ in range(4)]
    return _base(objs, recursion=3, dpi=dpi, lights=lights)
