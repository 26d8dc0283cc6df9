#!/usr/bin/env python3
"""Wave-level event counts of the standard-mode trace kernel (diagnostic).

Needs a library built with -DRT_EVENT_PROF (tools/build_exp.sh ev
"-DRT_EVENT_PROF"), loaded with RTAMD_LIB=...; rt_stats.ops[k] then counts
how many times a wave executed event k (EV_* in rt_device.hpp).  Prints the
counts per wave.  Usage (GPU box): RTAMD_LIB=... python tools/event_prof.py [config]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))


import rtamd  # noqa: E402
import scenes  # noqa: E402

EVENTS = ["shadow_queries", "shadow_candidates", "shadow_object_hits", "shadow_csg_hits", "primary_candidates",
          "primary_object_hits", "fold_leaves", "csg_combines", "comb_single", "comb_union_easy", "comb_general",
          "light_pass1", "light_pass2", "bounce_steps", "compact_leaves|bounce_lanes", "waves"]


def main():
    arg = sys.argv[1] if len(sys.argv) > 1 else "4"
    if arg.startswith("bvh"):   # e.g. bvh4096: tools/bvh_perf.py's random-sphere scene
        import json
        cfg, text, mode = arg, json.dumps(scenes.bvh_perf_scene(int(arg[3:]), dpi=480)), 0
    else:
        cfg = int(arg)
        text, mode = scenes.config_json(cfg)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    lib = rtamd.amd_lib()
    rows = (C.c_int32 * H)(*range(H))
    st = rtamd.Stats()
    rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, rows, H, buf.ptr, None, C.byref(st))
    assert rc == 0, rtamd.last_error()
    ev = [int(st.ops[k]) for k in range(len(EVENTS))]
    waves = max(1, ev[-1])
    print(f"config {cfg}: kernel {st.ms_kernel:.3f} ms, waves {waves}")
    for k, n in enumerate(EVENTS):
        print(f"  {n:20s} {ev[k]:14d}  {ev[k] / waves:9.3f} per wave")


if __name__ == "__main__":
    main()
