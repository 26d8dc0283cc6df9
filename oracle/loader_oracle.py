"""Loader oracle — TEST INFRASTRUCTURE ONLY (tests/ may import it; the product
never does).

A Python restatement of the reference's scene loader
(raytracer/src/json_loader.cpp of alp-aydin/Raytracing-Project) over
nlohmann::json semantics, used as the differential oracle of
tests/test_loader_fuzz.py for the C++ loader
(raytracing-project_amd/csrc/host/scene_loader.cpp).  The reference loader
itself cannot be built here (nlohmann/json is not installed), so parity is
anchored on its source text (cited per function) and on the Catch2 loader
tests restated in tests/test_loader.py.

load(text) returns either ("ok", scene) with scene a canonical dict
(camera, medium, lights, background, objects as trees with materials
inlined) or ("error", message) with the reference's message text, e.g.
"JSON processing error: sphere requires 'position', 'radius', 'color'".

Only the JSON value model matters here (inputs come from json.dumps): the
parser-level behaviours (BOM, duplicate keys, strictness, -0) are pinned by
tests/test_loader.py against the C++ parser directly.
"""
from __future__ import annotations

import json
import math

KEPS = 1e-6   # core.h:10


class Proc(Exception):
    """std::runtime_error / nlohmann::type_error caught as std::exception (json_loader.cpp:487)."""


# ------------------------------------------------------------ nlohmann model
def _tname(v) -> str:
    """basic_json::type_name()."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    return "object"


def _type_error(want: str, v):
    raise Proc(f"[json.exception.type_error.302] type must be {want}, but is {_tname(v)}")


def get_double(v) -> float:
    """get<double>(): numbers convert, booleans do not (from_json arithmetic)."""
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        _type_error("number", v)
    return float(v)


def get_int(v) -> int:
    """get<int>(): numbers (float truncates toward zero) and booleans."""
    if isinstance(v, bool):
        return int(v)
    if not isinstance(v, (int, float)):
        _type_error("number", v)
    return int(v) if isinstance(v, int) else int(math.trunc(v))


def get_string(v) -> str:
    if not isinstance(v, str):
        _type_error("string", v)
    return v


def contains(j, key) -> bool:
    """basic_json::contains(): false on anything but an object."""
    return isinstance(j, dict) and key in j


# ------------------------------------------------------------ json_loader.cpp
def as_vec3(a):   # json_loader.cpp:54-57
    if not isinstance(a, list) or len(a) != 3:
        raise Proc("Expected array[3]")
    return (get_double(a[0]), get_double(a[1]), get_double(a[2]))


def as_rgb(a):   # json_loader.cpp:64-67
    if not isinstance(a, list) or len(a) != 3:
        raise Proc("Expected color array[3]")
    return (get_double(a[0]), get_double(a[1]), get_double(a[2]))


def ensure_object_1key(j):   # json_loader.cpp:70-72
    if not isinstance(j, dict) or len(j) != 1:
        raise Proc("Each object node must be a one-entry object")


def material(albedo=(0.0, 0.0, 0.0), ambient=(0.0, 0.0, 0.0), kd=1.0, ks=0.0, kr=0.0, kt=0.0, shininess=1.0,
             refractive_index=1.0):
    return {"albedo": tuple(albedo), "ambient": tuple(ambient), "kd": kd, "ks": ks, "kr": kr, "kt": kt,
            "shininess": shininess, "refractive_index": refractive_index}


def parse_color_block(jc):   # json_loader.cpp:83-127
    if not isinstance(jc, dict):
        raise Proc("color must be an object")
    m = material()
    if "diffuse" in jc:
        m["albedo"] = as_rgb(jc["diffuse"])
    if "ambient" in jc:
        m["ambient"] = as_rgb(jc["ambient"])
    if "specular" in jc:
        s = as_rgb(jc["specular"])
        m["ks"] = (s[0] + s[1] + s[2]) / 3.0
    if "reflected" in jc:
        r = as_rgb(jc["reflected"])
        m["kr"] = (r[0] + r[1] + r[2]) / 3.0
    if "refracted" in jc:
        t = as_rgb(jc["refracted"])
        m["kt"] = (t[0] + t[1] + t[2]) / 3.0
    if "shininess" in jc:
        m["shininess"] = get_double(jc["shininess"])
    return m


def normalized(v):   # Dir3::normalized (core.h:95-101)
    L = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    if L > KEPS:
        return (v[0] / L, v[1] / L, v[2] / L)
    return (0.0, 1.0, 0.0)


def make_sphere(j):   # json_loader.cpp:204-221
    if not (contains(j, "position") and contains(j, "radius") and contains(j, "color")):
        raise Proc("sphere requires 'position', 'radius', 'color'")
    c = as_vec3(j["position"])
    r = get_double(j["radius"])
    m = parse_color_block(j["color"])
    if "index" in j:
        m["refractive_index"] = get_double(j["index"])
    return {"kind": "sphere", "c": c, "r": r, "mat": m}


def make_halfspace(j):   # json_loader.cpp:228-242
    if not (contains(j, "position") and contains(j, "normal") and contains(j, "color")):
        raise Proc("halfSpace requires 'position', 'normal', 'color'")
    p0 = as_vec3(j["position"])
    n = as_vec3(j["normal"])
    m = parse_color_block(j["color"])
    if "index" in j:
        m["refractive_index"] = get_double(j["index"])
    # HalfSpace constructor (geometry.h:124-134): scale by 1/sqrt(L2), +Y if L2 == 0
    L2 = n[0] * n[0] + n[1] * n[1] + n[2] * n[2]
    if L2 > 0.0:
        inv = 1.0 / math.sqrt(L2)
        nn = (n[0] * inv, n[1] * inv, n[2] * inv)
    else:
        nn = (0.0, 1.0, 0.0)
    return {"kind": "halfSpace", "p0": p0, "n_raw": n, "n": nn, "mat": m}


def make_pokeball(j):   # json_loader.cpp:250-295
    if not (contains(j, "position") and contains(j, "radius")):
        raise Proc("pokeball requires 'position' and 'radius'.")
    c = as_vec3(j["position"])
    r = get_double(j["radius"])
    # Material{} (geometry.h:5-22: shininess 32) with the fields :258-262 set
    mats = {
        "top": material(albedo=(0.88, 0.12, 0.20), ks=0.15, shininess=64.0),
        "bottom": material(albedo=(0.95, 0.95, 0.98), ks=0.08, shininess=32.0),
        "belt": material(albedo=(0.12, 0.12, 0.15), shininess=32.0),
        "ring": material(albedo=(0.35, 0.35, 0.40), shininess=32.0),
        "button": material(albedo=(0.96, 0.96, 0.99), ks=0.25, shininess=64.0),
    }
    belt_half, btn_outer, ring_width, btn_dir = 0.06, 0.28, 0.06, (1.0, 0.0, 0.0)
    if "colors" in j:
        jc = j["colors"]
        for k in ("top", "bottom", "belt", "ring", "button"):
            if contains(jc, k):
                mats[k] = parse_color_block(jc[k])
    if "belt_half" in j:
        belt_half = get_double(j["belt_half"])
    if "button_outer" in j:
        btn_outer = get_double(j["button_outer"])
    if "ring_width" in j:
        ring_width = get_double(j["ring_width"])
    if "button_dir" in j:
        btn_dir = as_vec3(j["button_dir"])
    return {"kind": "pokeball", "c": c, "r": r, "mats": mats, "belt_half": belt_half, "button_outer": btn_outer,
            "ring_width": ring_width, "button_dir_raw": btn_dir, "button_dir": normalized(btn_dir)}


def make_xform(kind, j):   # json_loader.cpp:302-320 (scaling, translation)
    if not (contains(j, "factors") and contains(j, "subject")):
        raise Proc(f"{kind} requires 'factors' and 'subject'")
    f = as_vec3(j["factors"])
    return {"kind": kind, "factors": f, "subject": parse_object_node(j["subject"])}


def make_rotation(j):   # json_loader.cpp:327-342
    if not (contains(j, "angle") and contains(j, "direction") and contains(j, "subject")):
        raise Proc("rotation requires 'angle', 'direction', and 'subject'")
    angle = get_double(j["angle"])
    axis = get_int(j["direction"])
    if axis not in (0, 1, 2):
        raise Proc("rotation direction must be 0 (X), 1 (Y), or 2 (Z)")
    sub = parse_object_node(j["subject"])
    return {"kind": "rotation", "axis": axis, "angle": angle * math.pi / 180.0, "subject": sub}


def make_csg_binary(j):   # json_loader.cpp:351-363
    if not (contains(j, "operator") and contains(j, "left") and contains(j, "right")):
        raise Proc("csg requires 'operator', 'left', 'right'")
    op = get_string(j["operator"])
    if op not in ("union", "intersection", "difference"):
        raise Proc("csg.operator must be union/intersection/difference")
    lhs = parse_object_node(j["left"])
    rhs = parse_object_node(j["right"])
    return {"kind": "csg", "op": op, "a": lhs, "b": rhs}


def fold(arr, op, min_len, msg):   # json_loader.cpp:372-401
    if not isinstance(arr, list) or len(arr) < min_len:
        raise Proc(msg)
    acc = parse_object_node(arr[0])
    for x in arr[1:]:
        acc = {"kind": "csg", "op": op, "a": acc, "b": parse_object_node(x)}
    return acc


def parse_object_node(j):   # json_loader.cpp:409-434
    ensure_object_1key(j)
    kind, val = next(iter(j.items()))
    if kind == "sphere":
        return make_sphere(val)
    if kind == "halfSpace":
        return make_halfspace(val)
    if kind == "pokeball":
        return make_pokeball(val)
    if kind in ("scaling", "translation"):
        return make_xform(kind, val)
    if kind == "rotation":
        return make_rotation(val)
    if kind == "csg":
        return make_csg_binary(val)
    if kind in ("union", "intersection"):
        return fold(val, kind, 1, "CSG array must be a non-empty array")
    if kind == "difference":
        return fold(val, "difference", 2, "difference array must have at least 2 elements")
    raise Proc("unknown object kind: " + kind)


def load(text: str):
    """jsonio::load_scene_from_json_text (json_loader.cpp:458-490)."""
    try:
        root = json.loads(text)
    except ValueError as e:
        return ("error", "JSON parse error: " + str(e))
    # Camera{} / ScreenSpec{} / Scene{} defaults (camera.h:9-16,33; scene.h:38-47)
    scene = {"camera": {"eye": (0.0, 0.0, 1.0), "P": (0.0, 0.0, 0.0), "Lx": 1.0, "Ly": 1.0, "dpi": 72},
             "ambient": (0.0, 0.0, 0.0), "index": 1.0, "recursion": 5, "lights": [],
             "background": (0.0, 0.0, 0.0), "objects": []}
    try:
        if contains(root, "screen"):   # parse_screen (json_loader.cpp:133-161)
            j = root["screen"]
            dpi = get_int(j["dpi"]) if contains(j, "dpi") else 72
            Lx = Ly = 1.0
            if contains(j, "dimensions"):
                d = j["dimensions"]
                if not isinstance(d, list) or len(d) != 2:
                    raise Proc("screen.dimensions must be [Lx, Ly]")
                Lx, Ly = get_double(d[0]), get_double(d[1])
            if not contains(j, "position"):
                raise Proc("screen.position is required")
            P = as_vec3(j["position"])
            if not contains(j, "observer"):
                raise Proc("screen.observer is required")
            eye = as_vec3(j["observer"])
            scene["camera"] = {"eye": eye, "P": P, "Lx": Lx, "Ly": Ly, "dpi": dpi}
        if contains(root, "medium"):   # parse_medium (json_loader.cpp:168-181)
            jm = root["medium"]
            if contains(jm, "ambient"):
                scene["ambient"] = as_rgb(jm["ambient"])
            if contains(jm, "index"):
                scene["index"] = get_double(jm["index"])
            if contains(jm, "recursion"):
                scene["recursion"] = get_int(jm["recursion"])
        if contains(root, "sources"):   # parse_sources (json_loader.cpp:188-202)
            arr = root["sources"]
            if not isinstance(arr, list):
                raise Proc("'sources' must be an array")
            for js in arr:
                if not (contains(js, "position") and contains(js, "intensity")):
                    raise Proc("each source needs 'position' and 'intensity'")
                p = as_vec3(js["position"])
                scene["lights"].append((p, as_rgb(js["intensity"])))
        if contains(root, "background"):
            scene["background"] = as_rgb(root["background"])
        if contains(root, "objects"):
            arr = root["objects"]
            if not isinstance(arr, list):
                raise Proc("'objects' must be an array")
            scene["objects"] = [parse_object_node(n) for n in arr]
    except Proc as e:
        return ("error", "JSON processing error: " + str(e))
    return ("ok", scene)
