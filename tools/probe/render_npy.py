"""Diagnostic: render a scene with the library in RTAMD_LIB and save the framebuffer (GPU box)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
import torch  # noqa: E402,F401
import numpy as np  # noqa: E402

import rtamd  # noqa: E402
import scenes  # noqa: E402

name, mode, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
flags = int(sys.argv[4]) if len(sys.argv) > 4 else 0
sc = rtamd.load_scene_from_json_text(json.dumps(scenes.load_example(name)))
st = rtamd.Stats()
fb = rtamd.Tracer(sc, sc.width, sc.height, mode, flags).render(st)
np.save(out, fb)
print(name, sc.width, sc.height, st.rays_intersect, st.rays_occluded)
