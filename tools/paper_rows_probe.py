#!/usr/bin/env python3
"""Diagnostic (GPU box): paper-mode kernel time of config 5 for different row
sets through rt_render_rows_device (one call, one chunk): all rows, rank 0
of the 2- and 8-way strip partitions, and contiguous bands of the same size."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
import rtamd  # noqa: E402
import scenes  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    text, mode = scenes.config_json(cfg)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    lib = rtamd.amd_lib()
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    st = rtamd.Stats()

    def t(rows, name, flags=0):
        best = 1e9
        for _ in range(3):
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, flags, (C.c_int32 * len(rows))(*rows), len(rows),
                                           buf.ptr, None, C.byref(st))
            assert rc == 0, rtamd.last_error()
            best = min(best, st.ms_kernel)
        print(f"{name:40s} rows {len(rows):5d}  kernel {best:8.3f} ms  per 1000 rows {best / len(rows) * 1000:7.3f} ms "
              f"rays {st.rays_intersect + st.rays_occluded}", flush=True)

    t(list(range(H)), "all rows")
    for N in (2, 8):
        r0 = rtamd.dist_rows(H, N, 0, mode)
        t(r0, f"rank 0 of {N} (strips)")
        t(list(range(len(r0))), f"contiguous band of {N}")
        t(list(range(H // 2 - len(r0) // 2, H // 2 - len(r0) // 2 + len(r0))), f"middle band of {N}")
    t(list(range(0, H, 2)), "every other row")


if __name__ == "__main__":
    main()
