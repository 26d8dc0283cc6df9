"""Host loader: the reference's JSON schema (raytracer/src/json_loader.cpp).

Restates raytracer/tests/test_json_loader.cpp and pins the semantics listed
in SURVEY.md §8b: defaults, colour-block rules, material identity, fold
order, error prefixes and nlohmann::json conversion rules."""
import json

import pytest

BASE_SCREEN = {"position": [0, 0, 0], "dimensions": [2, 2], "observer": [0, 0, 5]}


def _load(rt, obj):
    text = obj if isinstance(obj, str) else json.dumps(obj)
    return rt.load_scene_from_json_text(text)


_KEEP = []


def _desc(rt, obj):
    sc = _load(rt, obj)
    _KEEP.append(sc)   # the descriptor points into the scene's memory
    return sc.desc


def _err(rt, obj):
    with pytest.raises(rt.RTError) as e:
        _load(rt, obj)
    return e.value


def test_catch2_valid_scene(rt):   # test_json_loader.cpp:11-49
    sc = _load(rt, {"screen": dict(BASE_SCREEN, dpi=100), "objects": [{"sphere": {
        "position": [0, 0, 0], "radius": 1.0, "index": 1.0,
        "color": {"diffuse": [1.0, 0.0, 0.0], "ambient": [0.1, 0.0, 0.0], "specular": [0.5, 0.5, 0.5],
                  "reflected": [0.2, 0.2, 0.2], "refracted": [0.0, 0.0, 0.0], "shininess": 32}}}]})
    d = sc.desc
    assert d.n_objects == 1
    assert d.camera.Lx == 2.0 and d.camera.Ly == 2.0 and d.camera.dpi == 100
    m = d.materials[0]
    assert tuple(m.albedo) == (1.0, 0.0, 0.0) and tuple(m.ambient) == (0.1, 0.0, 0.0)
    assert m.ks == (0.5 + 0.5 + 0.5) / 3.0 and m.kr == (0.2 + 0.2 + 0.2) / 3.0 and m.kt == 0.0
    assert m.kd == 1.0 and m.shininess == 32.0 and m.refractive_index == 1.0


def test_catch2_default_dpi(rt):   # test_json_loader.cpp:52-66
    assert _desc(rt, {"screen": BASE_SCREEN, "objects": []}).camera.dpi == 72


def test_catch2_invalid_json(rt):   # test_json_loader.cpp:69-74
    e = _err(rt, "{ invalid json }")
    assert e.code == -2 and str(e).startswith("JSON parse error: ")


def test_catch2_color_must_be_object(rt):   # test_json_loader.cpp:77-98
    e = _err(rt, {"screen": BASE_SCREEN, "objects": [{"sphere": {"position": [0, 0, 0], "radius": 1.0,
                                                                   "color": [1.0, 0.0, 0.0]}}]})
    assert e.code == -3 and str(e) == "JSON processing error: color must be an object"


def test_catch2_halfspace(rt):   # test_json_loader.cpp:101-133
    sc = _load(rt, {"screen": BASE_SCREEN, "objects": [{"halfSpace": {
        "position": [0, 0, 0], "normal": [0, 1, 0], "color": {"diffuse": [0.0, 1.0, 0.0], "shininess": 1}}}]})
    assert sc.desc.n_objects == 1


def test_catch2_rotation(rt):   # test_json_loader.cpp:136-211
    sphere = {"sphere": {"position": [0, 0, 0], "radius": 1.0, "color": {"diffuse": [1, 0, 0]}}}
    sc = _load(rt, {"screen": BASE_SCREEN, "objects": [{"rotation": {"angle": 90, "direction": 2, "subject": sphere}}]})
    assert sc.desc.n_objects == 1
    e = _err(rt, {"screen": BASE_SCREEN, "objects": [{"rotation": {"angle": 90, "direction": 5, "subject": sphere}}]})
    assert "rotation direction must be 0 (X), 1 (Y), or 2 (Z)" in str(e)


def test_defaults(rt):   # scene.h:40-47, camera.h:26-35, json_loader.cpp:88-98
    d = _desc(rt, "{}")
    assert d.recursion_limit == 5 and d.medium_index == 1.0
    assert tuple(d.ambient) == (0, 0, 0) and tuple(d.background) == (0, 0, 0)
    assert tuple(d.camera.eye) == (0, 0, 1) and d.camera.Lx == 1.0 and d.camera.dpi == 72
    m = _desc(rt, {"objects": [{"sphere": {"position": [0, 0, 0], "radius": 1, "color": {}}}]}).materials[0]
    assert tuple(m.albedo) == (0, 0, 0) and m.shininess == 1.0 and m.kd == 1.0


def test_kd_ks_keys_ignored(rt):   # parse_color_block reads neither kd nor ks (README.md:144 is stale)
    m = _desc(rt, {"objects": [{"sphere": {"position": [0, 0, 0], "radius": 1,
                                           "color": {"kd": 0.3, "ks": 0.9}}}]}).materials[0]
    assert m.kd == 1.0 and m.ks == 0.0


def test_material_identity_not_deduplicated(rt):
    col = {"diffuse": [0.5, 0.5, 0.5]}
    d = _desc(rt, {"objects": [{"sphere": {"position": [0, 0, 0], "radius": 1, "color": col}},
                               {"sphere": {"position": [2, 0, 0], "radius": 1, "color": col}},
                               {"pokeball": {"position": [4, 0, 0], "radius": 1}}]})
    mats = [d.nodes[0].mat, d.nodes[1].mat] + list(d.nodes[2].mats)
    assert len(set(mats)) == 7 and d.n_materials == 7


def test_pokeball_defaults(rt):   # json_loader.cpp:264-274
    d = _desc(rt, {"objects": [{"pokeball": {"position": [0, 0, 0], "radius": 2, "button_dir": [0, 0, 3]}}]})
    n = d.nodes[0]
    assert tuple(n.v[4:7]) == (0.06, 0.28, 0.06)
    assert tuple(n.v[7:10]) == (0.0, 0.0, 1.0)
    top = d.materials[n.mats[0]]
    assert tuple(top.albedo) == (0.88, 0.12, 0.20) and top.ks == 0.15 and top.shininess == 64
    belt = d.materials[n.mats[2]]
    assert belt.ks == 0.0 and belt.shininess == 32.0   # Material{} default, not the colour-block default


def test_csg_folds_left(rt):   # json_loader.cpp:375-401
    s = {"sphere": {"position": [0, 0, 0], "radius": 1, "color": {}}}
    d = _desc(rt, {"objects": [{"union": [s, s, s]}]})
    root = d.nodes[d.objects[0]]
    assert root.kind == 6 and d.nodes[root.a].kind == 6 and d.nodes[root.b].kind == 0
    e = _err(rt, {"objects": [{"difference": [s]}]})
    assert "difference array must have at least 2 elements" in str(e)
    e = _err(rt, {"objects": [{"union": []}]})
    assert "CSG array must be a non-empty array" in str(e)
    e = _err(rt, {"objects": [{"csg": {"operator": "xor", "left": s, "right": s}}]})
    assert "csg.operator must be union/intersection/difference" in str(e)


def test_errors(rt):
    assert "unknown object kind: cube" in str(_err(rt, {"objects": [{"cube": {}}]}))
    assert "one-entry object" in str(_err(rt, {"objects": [{"sphere": {}, "halfSpace": {}}]}))
    assert "sphere requires" in str(_err(rt, {"objects": [{"sphere": {"position": [0, 0, 0]}}]}))
    assert "Expected array[3]" in str(_err(rt, {"objects": [{"sphere": {"position": [0, 0], "radius": 1,
                                                                        "color": {}}}]}))
    assert "screen.position is required" in str(_err(rt, {"screen": {"observer": [0, 0, 1]}}))
    assert "each source needs" in str(_err(rt, {"sources": [{"position": [0, 0, 0]}]}))
    assert "'objects' must be an array" in str(_err(rt, {"objects": {}}))
    assert "type must be number, but is string" in str(_err(rt, {"medium": {"index": "x"}}))


def test_nlohmann_conversions(rt):
    # get<int> truncates floats and accepts booleans; get<double> rejects booleans
    assert _desc(rt, {"screen": dict(BASE_SCREEN, dpi=100.9)}).camera.dpi == 100
    assert _desc(rt, {"screen": dict(BASE_SCREEN, dpi=True)}).camera.dpi == 1
    assert "type must be number, but is boolean" in str(_err(rt, {"medium": {"index": True}}))
    # an integer literal "-0" is integer zero -> +0.0; "-0.0" keeps its sign
    d = _desc(rt, '{"background": [-0, -0.0, 1]}')
    import math
    assert math.copysign(1, d.background[0]) == 1.0 and math.copysign(1, d.background[1]) == -1.0


def test_strict_json(rt):
    for bad in ('{"a": 1,}', '{"a": 1} x', '{/*c*/}', '{"a": NaN}', '[1, 2', '{"a": 01}', ''):
        assert _err(rt, bad).code == -2, bad
    assert _desc(rt, '﻿{}').n_objects == 0                       # BOM is skipped
    assert _desc(rt, '{"medium": {"recursion": 2, "recursion": 3}}').recursion_limit == 3   # last wins
    assert _desc(rt, '[1, 2]').n_objects == 0   # contains() on a non-object is false


def test_file_errors(rt, tmp_path):
    with pytest.raises(rt.RTError) as e:
        rt.load_scene_from_json(str(tmp_path / "missing.json"))
    assert e.value.code == -4 and str(e.value).startswith("Cannot open JSON file: ")
    p = tmp_path / "s.json"
    p.write_text(json.dumps({"objects": []}))
    assert rt.load_scene_from_json(str(p)).desc.n_objects == 0


def test_transform_matrices(rt):
    import math

    s = {"sphere": {"position": [0, 0, 0], "radius": 1, "color": {}}}
    d = _desc(rt, {"objects": [{"rotation": {"angle": 30, "direction": 1, "subject": s}},
                               {"scaling": {"factors": [2, 3, 4], "subject": s}},
                               {"translation": {"factors": [1, 2, 3], "subject": s}}]})
    rot = d.nodes[d.objects[0]]
    a = 30 * math.pi / 180.0
    assert rot.v[0] == math.cos(a) and rot.v[2] == math.sin(a) and rot.v[8] == -math.sin(a)
    assert rot.aux[0] == a
    sc = d.nodes[d.objects[1]]
    assert (sc.v[0], sc.v[5], sc.v[10]) == (2.0, 3.0, 4.0)
    tr = d.nodes[d.objects[2]]
    assert (tr.v[3], tr.v[7], tr.v[11]) == (1.0, 2.0, 3.0)


def test_desc_roundtrip(rt):
    import scenes

    sc = rt.load_scene_from_json_text(scenes.config_json(4, dpi=20)[0])
    sc2 = rt.scene_from_desc(sc.desc)
    a, b = sc.desc, sc2.desc
    assert (a.n_nodes, a.n_materials, a.n_lights, a.n_objects) == (b.n_nodes, b.n_materials, b.n_lights, b.n_objects)
    fa, _ = rt.oracle_render(sc, sc.width, sc.height, 1)
    fb, _ = rt.oracle_render(sc2, sc2.width, sc2.height, 1)
    assert (fa == fb).all()
