#!/usr/bin/env python3
"""Print the executed-operation counters (lane level) of one frame (GPU box; diagnostic).

Usage: python tools/opcounts.py [config] [dpi_scale]"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))


import rtamd  # noqa: E402
import scenes  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    text, mode = scenes.config_json(cfg)[0], scenes.config_json(cfg)[1]
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    st = rtamd.Stats()
    lib = rtamd.amd_lib()
    rc = lib.rt_render_rows_device(sc.handle, W, H, mode, rtamd.RT_FLAG_COUNT_OPS, (C.c_int32 * H)(*range(H)), H,
                                   buf.ptr, None, C.byref(st))
    assert rc == 0, rtamd.last_error()
    d = st.as_dict() if hasattr(st, "as_dict") else None
    rays = st.rays_intersect + st.rays_occluded
    print(f"config {cfg}: {W}x{H} mode {mode}: intersect {st.rays_intersect}  occluded {st.rays_occluded}")
    for i, name in enumerate(rtamd.OP_NAMES):
        v = int(st.ops[i])
        print(f"  {name:18s} {v:14d}   per ray {v / max(rays, 1):8.3f}")
    json.dump({"config": cfg, "isect": st.rays_intersect, "occl": st.rays_occluded,
               "ops": {n: int(st.ops[i]) for i, n in enumerate(rtamd.OP_NAMES)}}, sys.stderr)


if __name__ == "__main__":
    main()
