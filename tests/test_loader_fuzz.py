"""Differential fuzz of the C++ scene loader against the loader oracle
(schema bug-parity).

oracle/loader_oracle.py restates raytracer/src/json_loader.cpp over the
nlohmann::json value model (the reference loader itself needs nlohmann/json,
which is absent, so it cannot be run here: parity for this layer is pinned by
the restatement plus the Catch2 cases in tests/test_loader.py).  A seeded
corpus of schema-valid scenes is mutated (keys dropped, values retyped,
arrays resized, node objects given a second key, kinds misspelt, ...) and
every case must give the same scene tree or the same error message from both.
"""
import copy
import json
import os
import random
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import loader_oracle  # noqa: E402

KINDS = ["union", "intersection", "difference"]
REGIONS = ["top", "bottom", "belt", "ring", "button"]


# ------------------------------------------------------- C++ IR -> canonical
def _mat(d, i):
    m = d.materials[i]
    return {"albedo": tuple(m.albedo), "ambient": tuple(m.ambient), "kd": m.kd, "ks": m.ks, "kr": m.kr, "kt": m.kt,
            "shininess": m.shininess, "refractive_index": m.refractive_index}


def _node(rt, d, i):
    n = d.nodes[i]
    v, aux = list(n.v), list(n.aux)
    if n.kind == rt.NODE_SPHERE:
        return {"kind": "sphere", "c": tuple(v[0:3]), "r": v[3], "mat": _mat(d, n.mat)}
    if n.kind == rt.NODE_HALFSPACE:
        return {"kind": "halfSpace", "p0": tuple(v[0:3]), "n_raw": tuple(aux[0:3]), "n": tuple(v[3:6]),
                "mat": _mat(d, n.mat)}
    if n.kind == rt.NODE_POKEBALL:
        return {"kind": "pokeball", "c": tuple(v[0:3]), "r": v[3],
                "mats": {REGIONS[k]: _mat(d, n.mats[k]) for k in range(5)},
                "belt_half": v[4], "button_outer": v[5], "ring_width": v[6],
                "button_dir_raw": tuple(aux[0:3]), "button_dir": tuple(v[7:10])}
    if n.kind in (rt.NODE_TRANSLATION, rt.NODE_SCALING):
        kind = "translation" if n.kind == rt.NODE_TRANSLATION else "scaling"
        return {"kind": kind, "factors": tuple(aux[0:3]), "subject": _node(rt, d, n.a)}
    if n.kind == rt.NODE_ROTATION:
        return {"kind": "rotation", "axis": n.op, "angle": aux[0], "subject": _node(rt, d, n.a)}
    return {"kind": "csg", "op": KINDS[n.op], "a": _node(rt, d, n.a), "b": _node(rt, d, n.b)}


def ours(rt, text):
    try:
        sc = rt.load_scene_from_json_text(text)
    except rt.RTError as e:
        return ("error", str(e))
    d = sc.desc
    c = d.camera
    return ("ok", {
        "camera": {"eye": tuple(c.eye), "P": tuple(c.P), "Lx": c.Lx, "Ly": c.Ly, "dpi": c.dpi},
        "ambient": tuple(d.ambient), "index": d.medium_index, "recursion": d.recursion_limit,
        "lights": [(tuple(d.lights[i].pos), tuple(d.lights[i].intensity)) for i in range(d.n_lights)],
        "background": tuple(d.background),
        "objects": [_node(rt, d, d.objects[i]) for i in range(d.n_objects)],
    })


# ------------------------------------------------------------- generator
class Gen:
    def __init__(self, seed):
        self.r = random.Random(seed)

    def num(self):
        r = self.r
        k = r.random()
        if k < 0.4:
            return r.randint(-4, 6)
        if k < 0.9:
            return round(r.uniform(-8.0, 8.0), r.choice([1, 3, 17]))
        return r.choice([0.0, -0.0, 1e-7, 2.5e-300, 123456.789])

    def vec(self, n=3):
        return [self.num() for _ in range(n)]

    def color(self):
        r = self.r
        c = {}
        for k in ("diffuse", "ambient", "specular", "reflected", "refracted"):
            if r.random() < 0.5:
                c[k] = [abs(self.num()) for _ in range(3)]
        if r.random() < 0.5:
            c["shininess"] = r.choice([1, 8, 32.5, 0])
        if r.random() < 0.2:
            c[r.choice(["kd", "ks", "note"])] = self.num()   # ignored keys
        return c

    def node(self, depth=0):
        r = self.r
        kinds = ["sphere", "halfSpace", "pokeball"]
        if depth < 3:
            kinds += ["translation", "scaling", "rotation", "csg", "union", "intersection", "difference"]
        k = r.choice(kinds)
        if k == "sphere":
            v = {"position": self.vec(), "radius": abs(self.num()) + 0.1, "color": self.color()}
            if r.random() < 0.3:
                v["index"] = 1.0 + abs(self.num()) / 4
        elif k == "halfSpace":
            v = {"position": self.vec(), "normal": self.vec(), "color": self.color()}
            if r.random() < 0.3:
                v["index"] = 1.5
        elif k == "pokeball":
            v = {"position": self.vec(), "radius": abs(self.num()) + 0.1}
            if r.random() < 0.5:
                v["colors"] = {reg: self.color() for reg in REGIONS if r.random() < 0.5}
            for key in ("belt_half", "button_outer", "ring_width"):
                if r.random() < 0.3:
                    v[key] = abs(self.num()) / 10
            if r.random() < 0.4:
                v["button_dir"] = self.vec()
        elif k in ("translation", "scaling"):
            v = {"factors": self.vec(), "subject": self.node(depth + 1)}
        elif k == "rotation":
            v = {"angle": self.num() * 15, "direction": r.choice([0, 1, 2, 2.0, 1.9, True]),
                 "subject": self.node(depth + 1)}
        elif k == "csg":
            v = {"operator": r.choice(KINDS), "left": self.node(depth + 1), "right": self.node(depth + 1)}
        else:
            lo = 2 if k == "difference" else 1
            v = [self.node(depth + 1) for _ in range(r.randint(lo, 3))]
        return {k: v}

    def scene(self):
        r = self.r
        s = {}
        if r.random() < 0.9:
            sc = {"position": self.vec(), "observer": self.vec()}
            if r.random() < 0.7:
                sc["dimensions"] = [abs(self.num()) + 1, abs(self.num()) + 1]
            if r.random() < 0.7:
                sc["dpi"] = r.choice([4, 8, 12.7, 16, True])
            s["screen"] = sc
        if r.random() < 0.7:
            m = {}
            if r.random() < 0.6:
                m["ambient"] = [abs(self.num()) / 10 for _ in range(3)]
            if r.random() < 0.6:
                m["index"] = r.choice([1, 1.0, 1.33])
            if r.random() < 0.6:
                m["recursion"] = r.choice([0, 1, 3, 4.9, -1])
            s["medium"] = m
        if r.random() < 0.8:
            s["sources"] = [{"position": self.vec(), "intensity": [abs(self.num()) for _ in range(3)]}
                            for _ in range(r.randint(0, 3))]
        if r.random() < 0.6:
            s["background"] = [abs(self.num()) / 8 for _ in range(3)]
        s["objects"] = [self.node() for _ in range(r.randint(0, 4))]
        return s

    # ------------------------------------------------------------ mutations
    def _paths(self, x, path=()):
        yield path
        if isinstance(x, dict):
            for k, v in x.items():
                yield from self._paths(v, path + (k,))
        elif isinstance(x, list):
            for i, v in enumerate(x):
                yield from self._paths(v, path + (i,))

    def mutate(self, s):
        r = self.r
        s = copy.deepcopy(s)
        paths = list(self._paths(s))[1:]
        if not paths:
            return s
        path = r.choice(paths)
        parent = s
        for p in path[:-1]:
            parent = parent[p]
        key = path[-1]
        m = r.randint(0, 6)
        if m == 0 and isinstance(parent, dict):
            del parent[key]
        elif m == 1:
            parent[key] = r.choice([None, True, False, "str", [], {}, 3, 2.5, [1, 2], [1, 2, 3, 4], {"a": 1}])
        elif m == 2 and isinstance(parent[key], list) and parent[key]:
            parent[key] = parent[key][:-1]
        elif m == 3 and isinstance(parent[key], dict):
            parent[key]["extra"] = 1   # node objects become two-key objects
        elif m == 4 and isinstance(parent[key], dict) and len(parent[key]) == 1:
            (k, v), = parent[key].items()
            parent[key] = {r.choice(["cube", "Sphere", "halfspace", "Union"]): v}
        elif m == 5 and isinstance(parent[key], list):
            parent[key] = parent[key] + [r.choice([1, "x", None, {"sphere": {}}])]
        else:
            parent[key] = r.choice([-1, 0, 7.5, "union", [0, 0, 0]])
        return s


@pytest.mark.parametrize("block", range(6))
def test_loader_matches_oracle_on_fuzz_corpus(rt, block):
    g = Gen(1000 + block)
    n_ok = n_err = 0
    for case in range(400):
        s = g.scene()
        for _ in range(g.r.choice([0, 0, 1, 1, 2, 3])):
            s = g.mutate(s)
        text = json.dumps(s)
        got, want = ours(rt, text), loader_oracle.load(text)
        assert got == want, (block, case, text)
        n_ok += got[0] == "ok"
        n_err += got[0] == "error"
    assert n_ok > 50 and n_err > 50   # the corpus exercises both sides


def test_oracle_agrees_with_catch2_cases():
    """The oracle itself on the reference's own loader tests (test_json_loader.cpp)."""
    ok, sc = loader_oracle.load(json.dumps({"screen": {"position": [0, 0, 0], "dimensions": [2, 2],
                                                       "observer": [0, 0, 5], "dpi": 100},
                                            "objects": [{"sphere": {"position": [0, 0, 0], "radius": 1.0,
                                                                    "index": 1.0, "color": {
                                                                        "diffuse": [1.0, 0.0, 0.0],
                                                                        "specular": [0.5, 0.5, 0.5],
                                                                        "shininess": 32}}}]}))
    assert ok == "ok" and sc["camera"]["dpi"] == 100 and sc["objects"][0]["mat"]["ks"] == 0.5
    assert loader_oracle.load(json.dumps({"objects": [{"sphere": {"position": [0, 0, 0], "radius": 1,
                                                                  "color": [1, 0, 0]}}]})) == \
        ("error", "JSON processing error: color must be an object")
    assert loader_oracle.load("{}")[1]["camera"]["dpi"] == 72
