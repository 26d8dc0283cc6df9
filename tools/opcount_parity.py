#!/usr/bin/env python3
"""Diagnostic (GPU box): executed-op counters of the GPU with culling OFF vs the
CPU oracle (reference-equivalent counts) on the small parity scenes."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import rtamd  # noqa: E402
from test_gpu_parity import SMALL  # noqa: E402

for name in sorted(SMALL):
    for mode in (0, 1):
        sc = rtamd.load_scene_from_json_text(SMALL[name]())
        W, H = sc.width, sc.height
        st = rtamd.Stats()
        rtamd.Tracer(sc, W, H, mode, flags=rtamd.RT_FLAG_COUNT_OPS | rtamd.RT_FLAG_NO_CULL).render(st)
        _, ost = rtamd.oracle_render(sc, W, H, mode, threads=8)
        g = {n: int(st.ops[i]) for i, n in enumerate(rtamd.OP_NAMES)}
        o = {n: int(ost.ops[i]) for i, n in enumerate(rtamd.OP_NAMES)}
        diff = {n: (g[n], o[n]) for n in g if g[n] != o[n]}
        print(json.dumps({"scene": name, "mode": mode, "diff": diff}), flush=True)
