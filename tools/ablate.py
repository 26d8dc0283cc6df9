#!/usr/bin/env python3
"""Time the trace kernel on variants of a bench scene (GPU box; diagnostic).

Usage: python tools/ablate.py [config]
Prints one line per variant: kernel ms, rays, Mrays/s."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))


import rtamd  # noqa: E402
import scenes  # noqa: E402


def run(name, scene, mode=0, flags=0, reps=2):
    sc = rtamd.load_scene_from_json_text(json.dumps(scene))
    W, H = sc.width, sc.height
    rows = list(range(H))
    buf = rtamd.DeviceBuffer(H * W * 3 * 8)
    lib = rtamd.amd_lib()
    st = rtamd.Stats()
    best = None
    for _ in range(reps):
        rc = lib.rt_render_rows_device(sc.handle, W, H, mode, flags, (C.c_int32 * H)(*rows), H,
                                       buf.ptr, None, C.byref(st))
        assert rc == 0, rtamd.last_error()
        best = st.ms_kernel if best is None else min(best, st.ms_kernel)
    rays = st.rays_intersect + st.rays_occluded
    print(f"{name:40s} kernel {best:8.3f} ms  rng {st.ms_rng:6.3f} ms  rays {rays:>11d}  "
          f"{rays / best / 1e3:9.1f} Mrays/s", flush=True)


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    base = json.loads(scenes.config_json(cfg)[0])
    mode = scenes.config_json(cfg)[1]
    run("full" + (" (paper)" if mode else ""), base, mode=mode, reps=3)
    if os.environ.get("ABLATE_QUICK"):
        return
    run("full no-cull", base, flags=rtamd.RT_FLAG_NO_CULL)
    objs = base["objects"]
    s = dict(base, objects=[o for o in objs if "translation" not in o])
    run("without the CSG union", s)
    s = dict(base, objects=[o for o in objs if "translation" in o or "halfSpace" in o])
    run("only halfSpace + CSG union", s)
    s = dict(base, sources=base["sources"][:1])
    run("1 light", s)
    s = dict(base, sources=[])
    run("0 lights (primary rays only)", s)
    s = dict(base, objects=[o for o in objs if "halfSpace" in o])
    run("only halfSpace", s)
    s = dict(base, objects=[])
    run("empty scene", s)


if __name__ == "__main__":
    main()
