#!/usr/bin/env python3
"""Trace-kernel time of scenes with many objects, with and without the wave
BVH (RT_FLAG_NO_BVH) (GPU box; diagnostic / DESIGN.md §Wave BVH).

Usage: python tools/bvh_perf.py"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))

import rtamd  # noqa: E402
import scenes  # noqa: E402


def run(name, scene, mode=0, reps=3):
    sc = rtamd.load_scene_from_json_text(json.dumps(scene))
    W, H = sc.width, sc.height
    rows = (C.c_int32 * H)(*range(H))
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    lib = rtamd.amd_lib()
    out = []
    for flags, tag in ((rtamd.RT_FLAG_FORCE_BVH, "bvh"), (rtamd.RT_FLAG_NO_BVH, "no-bvh")):
        st = rtamd.Stats()
        best = None
        for _ in range(reps):
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, flags, rows, H, buf.ptr, None, C.byref(st))
            assert rc == 0, rtamd.last_error()
            best = st.ms_kernel if best is None else min(best, st.ms_kernel)
        rays = st.rays_intersect + st.rays_occluded
        out.append((tag, best, rays))
    (_, tb, rays), (_, tn, rays_n) = out
    assert rays == rays_n
    # the product's default: the first two frames of a shape try the BVH and
    # the flat list, later frames take the faster (rt_render.hip SceneCache);
    # a fresh scene handle starts the trial over
    sc2 = rtamd.load_scene_from_json_text(json.dumps(scene))
    st = rtamd.Stats()
    times = []
    for _ in range(2 + reps):
        rc = lib.rt_render_rows_device(sc2.handle, W, H, mode, 0, rows, H, buf.ptr, None, C.byref(st))
        assert rc == 0, rtamd.last_error()
        times.append(st.ms_kernel)
    ta = min(times[2:])
    print(f"{name:34s} {W}x{H} mode {mode}  objects {len(scene['objects']):5d}  rays {rays:>11d}  "
          f"bvh {tb:8.3f} ms ({rays / tb / 1e3:8.1f} Mrays/s)  no-bvh {tn:8.3f} ms  speed-up {tn / tb:5.2f}x  "
          f"auto {ta:8.3f} ms ({tn / ta:5.2f}x)", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "split":   # where the time goes: primary rays vs each light
        s = scenes.bvh_perf_scene(4096, dpi=480)
        for nl in (0, 1, 4):
            run(f"random spheres 4096, {nl} lights", dict(s, sources=s["sources"][:nl]))
        return
    run("random spheres 4096", scenes.bvh_perf_scene(4096, dpi=480))
    run("random spheres 1024", scenes.bvh_perf_scene(1024, dpi=480))
    run("random spheres 4096, paper", scenes.bvh_perf_scene(4096, dpi=480), mode=1)
    g = scenes.bvh_scenes(480)["grid"]
    run("lattice 576 (rec 3)", g)
    run("ties 300 (rec 2)", scenes.bvh_scenes(480)["ties"])


if __name__ == "__main__":
    main()
