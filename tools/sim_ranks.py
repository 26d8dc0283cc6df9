#!/usr/bin/env python3
"""Per-rank cost of the multi-GPU row split, measured on ONE GPU (GPU box).

For each world size N, every rank's share of the frame (frame_dist.strip_rows)
is rendered in turn on cuda:0 and timed (host wall clock around the blocking
rt_render_rows_device call, plus the library's own HIP-event split into
jitter stream and trace kernel).  The slowest rank bounds the N-GPU step
before the gather; the gather itself is not simulated here.

Usage: python tools/sim_ranks.py [--config 4] [--worlds 1,2,4,8] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))

import torch  # noqa: E402

import frame_dist  # noqa: E402
import rtamd  # noqa: E402
import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--strip", type=int, default=frame_dist.STRIP)
    ap.add_argument("--chunks", type=int, default=1, help="trace through rt_frame_* in this many chunks")
    ap.add_argument("--two-streams", action="store_true", help="alternate chunks between two streams")
    args = ap.parse_args()
    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    lib = rtamd.amd_lib()
    buf = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    streams = [stream, torch.cuda.Stream()] if args.two_streams else [stream]
    st = rtamd.Stats()

    def run(rows):
        if args.chunks <= 1:
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                           C.c_void_p(buf.data_ptr()), C.c_void_p(stream.cuda_stream), C.byref(st))
            assert rc == 0, rtamd.last_error()
            return
        fr = C.c_void_p()
        rc = lib.rt_frame_begin(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                C.c_void_p(stream.cuda_stream), C.byref(fr))
        assert rc == 0, rtamd.last_error()
        for k, (a, b) in enumerate(frame_dist.chunk_bounds(len(rows), args.chunks)):
            s = streams[k % len(streams)]
            rc = lib.rt_frame_trace(fr, a, b, C.c_void_p(buf[a].data_ptr()), C.c_void_p(s.cuda_stream))
            assert rc == 0, rtamd.last_error()
        rc = lib.rt_frame_end(fr, C.byref(st))
        assert rc == 0, rtamd.last_error()

    base = None
    for N in [int(v) for v in args.worlds.split(",")]:
        per = []
        for r in range(N):
            rows = frame_dist.strip_rows(H, r, N, args.strip)
            run(rows)
            wall, rng, ker = [], [], []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(rows)
                torch.cuda.synchronize()
                wall.append((time.perf_counter() - t0) * 1e3)
                rng.append(st.ms_rng)
                ker.append(st.ms_kernel)
            per.append({"rank": r, "rows": len(rows), "wall_ms": min(wall), "rng_ms": min(rng),
                        "kernel_ms": min(ker), "rays": st.rays_intersect + st.rays_occluded})
        worst = max(p["wall_ms"] for p in per)
        if base is None and N == 1:
            base = worst
        out = {"config": args.config, "world": N, "strip": args.strip, "chunks": args.chunks, "two_streams": args.two_streams, "max_rank_wall_ms": round(worst, 3),
               "max_rank_rng_ms": round(max(p["rng_ms"] for p in per), 3),
               "max_rank_kernel_ms": round(max(p["kernel_ms"] for p in per), 3),
               "min_rank_kernel_ms": round(min(p["kernel_ms"] for p in per), 3),
               "speedup_before_gather": round(base / worst, 3) if base else None}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
