#!/usr/bin/env python3
"""Base cost of the recursion kernel (k_std_secw) against the lean kernel on
the same frame (GPU box; diagnostic): config 6's scene without reflective /
refractive materials (lean kernel), then the same scene plus one off-screen
sphere with a tiny reflectance (k_std_secw, almost no bounces).

Usage: python tools/secw_base.py"""
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import ablate  # noqa: E402
import scenes  # noqa: E402


def main():
    base = json.loads(scenes.config_json(6)[0])
    flat = copy.deepcopy(base)
    for o in flat["objects"]:
        col = next(iter(o.values())).get("color", {})
        col.pop("reflected", None)
        col.pop("refracted", None)
    ablate.run("no reflective materials (lean)", flat)
    plus = copy.deepcopy(flat)
    plus["objects"].append({"sphere": {"position": [0, 0, 50], "radius": 0.1,
                                       "color": {"diffuse": [0.5, 0.5, 0.5], "reflected": [1e-9, 1e-9, 1e-9]}}})
    ablate.run("+ off-screen mirror (secw, no bounces)", plus)
    ablate.run("config 6 (secw, bounces)", base)


if __name__ == "__main__":
    main()
