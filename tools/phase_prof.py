#!/usr/bin/env python3
"""Phase breakdown of the standard-mode trace kernel (diagnostic).

Needs a library built with -DRT_PHASE_PROF (tools/build_exp.sh prof
"-DRT_PHASE_PROF"), loaded with RTAMD_LIB=...; rt_stats.ops[k] then holds the
shader-clock cycles lane 0 of every full wave spent in phase k (PH_* in
rt_device.hpp).  Prints each phase's share of the summed wave time.
Usage (GPU box): RTAMD_LIB=.../librtamd_prof.so python tools/phase_prof.py [config]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))


import rtamd  # noqa: E402
import scenes  # noqa: E402

PHASES = ["setup", "primary", "shade1(+shadow)", "shadow", "shadow_csg", "shade2", "primary_csg", "tail",
          "csg_leaf", "csg_combine", "chain_xform", "obj_prefilter", "obj_hit", "wave_setup"]


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    text, mode = scenes.config_json(cfg)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    lib = rtamd.amd_lib()
    rows = (C.c_int32 * H)(*range(H))
    st = rtamd.Stats()
    for _ in range(3):
        rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, rows, H, buf.ptr, None,
                                       C.byref(st))
        assert rc == 0, rtamd.last_error()
    ph = [int(st.ops[k]) for k in range(len(PHASES))]
    tot = ph[0] + ph[1] + ph[2] + ph[5] + ph[7]
    print(f"config {cfg}: kernel {st.ms_kernel:.3f} ms, summed wave cycles {tot:.4g}")
    for k, n in enumerate(PHASES):
        print(f"  {n:18s} {ph[k]:14d}  {100.0 * ph[k] / max(1, tot):6.2f} %")
    print(f"  shade1 net         {100.0 * (ph[2] - ph[3]) / max(1, tot):6.2f} %")


if __name__ == "__main__":
    main()
