"""Per-strip trace cost of a BASELINE config on one GPU, and what it implies
for the multi-GPU row partition (rt_dist.hip strip_owners / partition_rows).

Each strip of `--strip` rows (default: the product's for the mode) is traced
alone through rt_render_rows_device, `--reps` times, min kernel ms kept (a
lone strip does not fill the GPU, so this is a relative cost, summed per
rank).  Prints one JSON line per config: the strip costs, and for worlds
2/4/8 every rank's summed cost under the product's partition plus the
max/mean imbalance.  Needs a GPU.
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raytracing-project_amd", "python"))

import frame_dist  # noqa: E402
import rtamd  # noqa: E402
import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--strip", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    S = args.strip or frame_dist.strip_for(mode)
    lib = rtamd.amd_lib()
    buf = rtamd.DeviceBuffer(H * W * 24)
    stream = rtamd.Stream()
    st = rtamd.Stats()
    costs, rays = [], []
    for s0 in range(0, H, S):
        rows = list(range(s0, min(H, s0 + S)))
        arr = (C.c_int32 * len(rows))(*rows)
        best = None
        for _ in range(args.reps + 1):
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, arr, len(rows), buf.ptr, stream.handle,
                                           C.byref(st))
            assert rc == 0, rtamd.last_error()
            best = st.ms_kernel if best is None else min(best, st.ms_kernel)
        costs.append(round(best, 4))
        rays.append(st.rays_intersect + st.rays_occluded)
    out = {"config": args.config, "strip": S, "W": W, "H": H, "strip_kernel_ms": costs, "strip_rays": rays,
           "sum_ms": round(sum(costs), 3), "worlds": {}}
    for N in (2, 4, 8):
        own = frame_dist.strip_owners(len(costs), N, mode)
        per = [0.0] * N
        per_rays = [0] * N
        for s, r in enumerate(own):
            per[r] += costs[s]
            per_rays[r] += rays[s]
        mean = sum(per[1:]) / (N - 1)
        out["worlds"][N] = {"rank_ms": [round(v, 3) for v in per], "rank_rays": per_rays,
                            "max_over_mean_nonroot": round(max(per[1:]) / mean, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
