"""Does the order of a rank's strips change its trace time?  (the launch tail)

For each rank of a `--world`-way split of a BASELINE config, the rank's rows
are traced in one rt_render_rows_device launch (i) in ascending row order (the
product's), (ii) strip by strip in decreasing measured cost, (iii) increasing
cost.  Strip costs come from tracing every strip alone first (as
tools/strip_costs.py).  Prints one JSON line per order with every rank's
kernel ms (min over --reps).  Needs a GPU.
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
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    S = frame_dist.strip_for(mode)
    lib = rtamd.amd_lib()
    buf = rtamd.DeviceBuffer(H * W * 24)
    stream = rtamd.Stream()
    st = rtamd.Stats()

    def kernel_ms(rows):
        arr = (C.c_int32 * len(rows))(*rows)
        best = None
        for _ in range(args.reps + 1):
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, arr, len(rows), buf.ptr, stream.handle,
                                           C.byref(st))
            assert rc == 0, rtamd.last_error()
            best = st.ms_kernel if best is None else min(best, st.ms_kernel)
        return best

    cost = {s0: kernel_ms(list(range(s0, min(H, s0 + S)))) for s0 in range(0, H, S)}
    full = kernel_ms(list(range(H)))
    for name in ("ascending", "costly_first", "cheap_first"):
        per = []
        for r in range(args.world):
            rows = rtamd.dist_rows(H, args.world, r, mode)
            strips = sorted({(y // S) * S for y in rows})
            if name != "ascending":
                strips.sort(key=lambda s0: cost[s0], reverse=(name == "costly_first"))
            order = [y for s0 in strips for y in range(s0, min(H, s0 + S)) if y in set(rows)]
            per.append(round(kernel_ms(order), 4))
        print(json.dumps({"config": args.config, "world": args.world, "order": name, "full_frame_ms": round(full, 4),
                          "ideal_share_ms": round(full / args.world, 4), "rank_kernel_ms": per,
                          "max": max(per), "sum": round(sum(per), 4)}), flush=True)


if __name__ == "__main__":
    main()
