#!/usr/bin/env python3
"""Per-rank cost of the multi-GPU row split, measured on ONE GPU (GPU box).

For each world size N, every rank's share of the frame (rt_dist_rows: the
partition rt_render_dist uses) is rendered in turn on cuda:0 through
rt_frame_* in the product's 4 row chunks and timed (host wall clock around
the blocking call, plus the library's HIP-event split into jitter stream and
trace kernel).  The slowest rank bounds the N-GPU step before the gather.

The gather is added as a model: chunks 1..3 of a rank (40/30/20/10 % of its
rows) are gathered while the next chunk traces, so the exposed part is the
LAST (smallest) chunk's ncclGather into
rank 0 (N-1 peers, each on its own xGMI link, in parallel) plus its
placement on the root; a link is priced at 64 GB/s (conservative) and 153
GB/s (the per-link figure of the MI355X spec sheet), the placement at the
measured device copy rate of the same bytes.

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

import numpy as np  # noqa: E402

import frame_dist  # noqa: E402
import rtamd  # noqa: E402
import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--strip", type=int, default=None, help="strip height (default: the product's for the mode)")
    ap.add_argument("--chunks", type=int, default=4, help="trace through rt_frame_* in this many chunks")
    ap.add_argument("--rgb8", action="store_true", help="gather 3 B/px (the CLI path) instead of FP64")
    ap.add_argument("--one-stream", dest="two_streams", action="store_false",
                    help="all chunks on one stream (the product alternates two, rt_dist.hip)")
    ap.add_argument("--legacy", action="store_true",
                    help="time rt_frame_* chunks directly (FP64 rows) instead of the product's rank path "
                         "(rt_test_dist_sim_rank: paper codes, placement on rank 0)")
    ap.set_defaults(two_streams=True)
    args = ap.parse_args()
    if not args.legacy:
        return product_ranks(args)
    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    strip = args.strip or frame_dist.strip_for(mode)
    lib = rtamd.amd_lib()
    row_bytes = W * 3 * 8
    buf = rtamd.DeviceBuffer(H * row_bytes)
    stream = rtamd.Stream()
    streams = [stream, rtamd.Stream()] if args.two_streams else [stream]
    st = rtamd.Stats()

    def run(rows):
        if args.chunks <= 1:
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                           buf.ptr, stream.handle, C.byref(st))
            assert rc == 0, rtamd.last_error()
            return
        fr = C.c_void_p()
        rc = lib.rt_frame_begin(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                stream.handle, C.byref(fr))
        assert rc == 0, rtamd.last_error()
        for k, (a, b) in enumerate(frame_dist.chunk_bounds(len(rows), args.chunks, strip)):
            s = streams[k % len(streams)]
            rc = lib.rt_frame_trace(fr, a, b, C.c_void_p(buf.ptr.value + a * row_bytes), s.handle)
            assert rc == 0, rtamd.last_error()
        rc = lib.rt_frame_end(fr, C.byref(st))
        assert rc == 0, rtamd.last_error()

    base = None
    for N in [int(v) for v in args.worlds.split(",")]:
        per = []
        for r in range(N):
            rows = rtamd.dist_rows(H, N, r, mode) if args.strip is None else frame_dist.strip_rows(H, r, N, args.strip)
            run(rows)
            wall, rng, ker = [], [], []
            for _ in range(args.reps):
                rtamd.device_synchronize()
                t0 = time.perf_counter()
                run(rows)
                rtamd.device_synchronize()
                wall.append((time.perf_counter() - t0) * 1e3)
                rng.append(st.ms_rng)
                ker.append(st.ms_kernel)
            per.append({"rank": r, "rows": len(rows), "wall_ms": min(wall), "rng_ms": min(rng),
                        "kernel_ms": min(ker), "rays": st.rays_intersect + st.rays_occluded})
        worst = max(p["wall_ms"] for p in per)
        if base is None and N == 1:
            base = worst
        # exposed gather of the last chunk (model) + its placement on the root (measured copy rate)
        m = max(p["rows"] for p in per)
        bpp = 3 if args.rgb8 else 24
        a_last, b_last = frame_dist.chunk_bounds(m, args.chunks, strip)[-1]   # the product's (decreasing) chunks
        last_chunk = (b_last - a_last) * W * bpp
        # placement of the gathered slots on the root: the same row-scatter the
        # product runs (k_scatter_rows / k_place_rows), timed on N * last-chunk rows
        n_slots = max(1, (last_chunk // row_bytes) * N) if not args.rgb8 else max(1, (last_chunk * 8 // row_bytes) * N)
        src = rtamd.DeviceBuffer(n_slots * row_bytes)
        rows_d = rtamd.DeviceBuffer(n_slots * 4)
        rows_d.from_host(np.arange(n_slots, dtype=np.int32) % H)
        dst = rtamd.DeviceBuffer(H * row_bytes)
        lib.rt_scatter_rows_device(src.ptr, rows_d.ptr, n_slots, W, dst.ptr, None)
        rtamd.device_synchronize()
        tc = time.perf_counter()
        for _ in range(5):
            lib.rt_scatter_rows_device(src.ptr, rows_d.ptr, n_slots, W, dst.ptr, None)
        rtamd.device_synchronize()
        place_ms = (time.perf_counter() - tc) / 5 * 1e3 if N > 1 else 0.0
        if args.rgb8:
            place_ms /= 8.0   # (3 B/px placed, the scatter above moved 24 B/px)
        g64 = (last_chunk / 64e9 * 1e3 + place_ms) if N > 1 else 0.0
        g153 = (last_chunk / 153e9 * 1e3 + place_ms) if N > 1 else 0.0
        out = {"config": args.config, "world": N, "strip": strip, "chunks": args.chunks, "two_streams": args.two_streams, "max_rank_wall_ms": round(worst, 3),
               "max_rank_rng_ms": round(max(p["rng_ms"] for p in per), 3),
               "max_rank_kernel_ms": round(max(p["kernel_ms"] for p in per), 3),
               "min_rank_kernel_ms": round(min(p["kernel_ms"] for p in per), 3),
               "speedup_before_gather": round(base / worst, 3) if base else None,
               "gather_bytes_per_rank": m * W * bpp, "exposed_gather_ms_64GBs": round(g64, 3),
               "exposed_gather_ms_153GBs": round(g153, 3),
               "projected_speedup_64GBs": round(base / (worst + g64), 3) if base else None,
               "projected_speedup_153GBs": round(base / (worst + g153), 3) if base else None}
        print(json.dumps(out), flush=True)


def product_ranks(args):
    """Every rank's share through the product's rank path on this GPU
    (rt_test_dist_sim_rank: rt_render_dist's dist_frame with the RCCL gather
    replaced by a device copy; rank 0 also places/decodes every slot).  The
    frame ends at the later of rank 0's own timeline and the slowest other
    rank + its last chunk's bytes over one xGMI link + that chunk's placement
    on rank 0 (timed)."""
    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    lib = rtamd.amd_lib()
    lib.rt_test_dist_sim_rank.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(rtamd.Stats)]
    st = rtamd.Stats()
    rgb8 = 1 if args.rgb8 else 0
    base = None
    for N in [int(v) for v in args.worlds.split(",")]:
        per = []
        for r in range(N):
            def run():
                rc = lib.rt_test_dist_sim_rank(sc.handle, W, H, mode, 0, N, r, rgb8, C.byref(st))
                assert rc == 0, rtamd.last_error()
            run()
            wall, ker = [], []
            for _ in range(args.reps):
                rtamd.device_synchronize()
                t0 = time.perf_counter()
                run()
                wall.append((time.perf_counter() - t0) * 1e3)
                ker.append(st.ms_kernel)
            per.append({"rank": r, "wall_ms": min(wall), "kernel_ms": min(ker),
                        "rays": st.rays_intersect + st.rays_occluded})
        worst = max(p["wall_ms"] for p in per)
        if base is None and N == 1:
            base = worst
        m = max(len(rtamd.dist_rows(H, N, r, mode)) for r in range(N))   # rows per rank slot (dist_frame's m)
        strip = frame_dist.strip_for(mode)
        nch = int(os.environ.get("RT_DIST_CHUNKS_PAPER", "2") if mode == 1 else os.environ.get("RT_DIST_CHUNKS", "4"))
        a_last, b_last = frame_dist.chunk_bounds(m, max(1, min(4, nch)), strip)[-1]
        bpp = 1 if mode == 1 else (3 if args.rgb8 else 24)   # paper: one code byte per pixel
        last_chunk = (b_last - a_last) * W * bpp
        # the last chunk's placement on rank 0 can only start once the slowest
        # rank's gather has landed: timed as the same row scatter over N * the
        # last chunk's rows (24 B/px read + written), scaled to what the product
        # moves (FP64: 24 + 24 B/px; paper codes: 1 + 24; RGB8: 3 + 3)
        place_ms = 0.0
        if N > 1:
            row_bytes = W * 24
            n_slots = max(1, (b_last - a_last) * N)
            src = rtamd.DeviceBuffer(n_slots * row_bytes)
            rows_d = rtamd.DeviceBuffer(n_slots * 4)
            rows_d.from_host(np.arange(n_slots, dtype=np.int32) % H)
            dst = rtamd.DeviceBuffer(H * row_bytes)
            lib.rt_scatter_rows_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
            lib.rt_scatter_rows_device(src.ptr, rows_d.ptr, n_slots, W, dst.ptr, None)
            rtamd.device_synchronize()
            tc = time.perf_counter()
            for _ in range(5):
                lib.rt_scatter_rows_device(src.ptr, rows_d.ptr, n_slots, W, dst.ptr, None)
            rtamd.device_synchronize()
            place_ms = (time.perf_counter() - tc) / 5 * 1e3 * (bpp + (3 if args.rgb8 else 24)) / 48.0
        others = max((p["wall_ms"] for p in per[1:]), default=0.0)

        def frame_ms(rate):   # rank 0's own timeline vs. the slowest peer + its last gather + placement
            if N == 1:
                return worst
            return max(per[0]["wall_ms"], others + last_chunk / rate * 1e3 + place_ms)
        t64, t153 = frame_ms(64e9), frame_ms(153e9)
        out = {"config": args.config, "world": N, "path": "product rank (rt_test_dist_sim_rank)", "chunks": nch,
               "max_rank_wall_ms": round(worst, 3), "rank0_wall_ms": round(per[0]["wall_ms"], 3),
               "min_rank_wall_ms": round(min(p["wall_ms"] for p in per), 3),
               "max_rank_kernel_ms": round(max(p["kernel_ms"] for p in per), 3),
               "rank_wall_ms": [round(p["wall_ms"], 3) for p in per],
               "gather_bytes_per_rank": m * W * bpp,
               "speedup_before_gather": round(base / worst, 3) if base else None,
               "last_chunk_place_ms": round(place_ms, 4),
               "frame_ms_64GBs": round(t64, 4), "frame_ms_153GBs": round(t153, 4),
               "projected_speedup_64GBs": round(base / t64, 3) if base else None,
               "projected_speedup_153GBs": round(base / t153, 3) if base else None}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
