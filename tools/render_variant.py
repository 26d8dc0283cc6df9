#!/usr/bin/env python3
"""Render one variant of the config-4 scene twice (GPU box; diagnostic, for
rocprofv3 --pmc passes on a sub-scene).  Variants: full, nolights, nounion,
nolights_nounion, half, nolights_half.

Usage: python tools/render_variant.py VARIANT"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))


import rtamd  # noqa: E402
import scenes  # noqa: E402


def variant(name):
    base = json.loads(scenes.config_json(4)[0])
    objs = base["objects"]
    if "nolights" in name:
        base = dict(base, sources=[])
    if "nounion" in name:
        base = dict(base, objects=[o for o in objs if "translation" not in o])
    if name.endswith("half"):
        base = dict(base, objects=[o for o in objs if "halfSpace" in o])
    return base


def main():
    sc = rtamd.load_scene_from_json_text(json.dumps(variant(sys.argv[1])))
    W, H = sc.width, sc.height
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    st = rtamd.Stats()
    for _ in range(2):
        rc = rtamd.amd_lib().rt_render_rows_device(sc.handle, W, H, 0, 0, (C.c_int32 * H)(*range(H)), H,
                                                   buf.ptr, None, C.byref(st))
        assert rc == 0, rtamd.last_error()
    print(sys.argv[1], "kernel ms", st.ms_kernel)


if __name__ == "__main__":
    main()
