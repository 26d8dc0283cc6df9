#!/usr/bin/env python3
"""bench.py — BASELINE.json headline metric on MI355X.

Metric: Mrays/s (primary + secondary) and wall-clock per frame on config 4:
examples/snorlax.json at 3840x2160, 5 lights, recursion 4.
A "ray" is one Scene::intersect or Scene::occluded query of the reference
(raytracer/src/scene.cpp:10,33).  A "step" renders one whole frame: jitter
stream generation (mt19937 jump-ahead) + trace kernels, with the scene and
all buffers resident on the device; for N > 1 each rank renders interleaved
8-row strips of the SAME frame (strong scaling) and rank 0 receives all rows
with one RCCL all_gather over xGMI and scatters them into the frame.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4]
For N > 1 the driver launches one process per GPU with torch.distributed.run.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))

FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector: 256 CU x 64 lanes x 2 x 2.4 GHz
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table


def model_flops(ops: dict, primary: int, paper: bool) -> tuple[float, dict]:
    """Algorithmic FP64 FLOPs from executed-op counters, per SURVEY.md §8d's
    table (+,-,*,/,sqrt = 1; pow/acos counted separately)."""
    si, sih = ops["sphere_isect"], ops["sphere_isect_hit"]
    sv, svh = ops["sphere_ivl"], ops["sphere_ivl_hit"]
    hi, hih, hv = ops["half_isect"], ops["half_isect_hit"], ops["half_ivl"]
    f = 17 * (si - sih) + 36 * sih + 17 * (sv - svh) + 54 * svh
    f += 14 * (hi - hih) + 25 * hih + 30 * hv
    f += 12 * ops["poke_region"] + 34 * ops["xform"]
    f += (39 if paper else 51) * primary
    f += 4 * ops["shade_call"]
    occl = ops.get("_occluded", 0)
    f += 17 * max(0, ops["light_eval"] - occl) + 33 * occl
    f += 38 * (ops["shade_light"] - ops["shade_spec"]) + 80 * ops["shade_spec"]
    f += 70 * ops["secondary"]
    return float(f), {"pow": ops["shade_spec"], "acos": ops["poke_region"]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--cpu-rows", type=int, default=64, help="rows in the CPU-oracle baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-cull", action="store_true", help="disable wave-uniform bound culling")
    ap.add_argument("--fp32", action="store_true",
                    help="time the NON-PARITY FP32 fast path as the headline (RT_FLAG_FP32); default is FP64")
    ap.add_argument("--fp32-steps", type=int, default=3, help="frames of the FP32 side leg (0 = skip)")
    ap.add_argument("--chunks", type=int, default=4, help="row chunks per rank pipelined with the gather (N > 1)")
    args = ap.parse_args()

    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import frame_dist
    import rtamd
    import scenes
    from frame_dist import STRIP

    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    lib = rtamd.amd_lib()
    flags = rtamd.RT_FLAG_NO_CULL if args.no_cull else rtamd.RT_FLAG_NONE
    if args.fp32:
        flags |= rtamd.RT_FLAG_FP32
    dev = torch.device("cuda", local)

    df = frame_dist.DistFrame(W, H, rank, world, dev, chunks=args.chunks)
    rows = df.rows
    n_rows = len(rows)
    rows_c = (C.c_int32 * max(1, n_rows))(*rows)
    stream = torch.cuda.current_stream(dev)
    # chunks alternate between two streams so one chunk's launch tail overlaps the next chunk
    streams = [stream, torch.cuda.Stream(dev)]
    st = rtamd.Stats()

    def scatter(src, slot_rows, full):
        rc = lib.rt_scatter_rows_device(C.c_void_p(src.data_ptr()), C.c_void_p(slot_rows.data_ptr()),
                                        slot_rows.numel(), W, C.c_void_p(full.data_ptr()),
                                        C.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"rt_scatter_rows_device failed ({rc}): {rtamd.last_error()}")

    def step(f=flags, stats=st):
        # one frame: jitter stream of this rank's rows (rt_frame_begin), the
        # trace chunk by chunk, each chunk gathered to rank 0 over RCCL while
        # the next one is traced (frame_dist.DistFrame), scatter on rank 0
        fr = C.c_void_p()
        rc = lib.rt_frame_begin(sc.handle, W, H, mode, f, rows_c, n_rows, C.c_void_p(stream.cuda_stream),
                                C.byref(fr))
        if rc != 0:
            raise RuntimeError(f"rt_frame_begin failed ({rc}): {rtamd.last_error()}")
        err = []

        def trace_chunk(a, b, out, s):
            r = lib.rt_frame_trace(fr, a, b, C.c_void_p(out.data_ptr()), C.c_void_p(s.cuda_stream))
            if r != 0:
                err.append((r, rtamd.last_error()))

        try:
            df.run(trace_chunk, dist, scatter, streams)
        finally:
            rc = lib.rt_frame_end(fr, C.byref(stats))
        if err or rc != 0:
            raise RuntimeError(f"frame failed: {err or rc} {rtamd.last_error()}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms, rng_ms, rays_local = [], [], 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kernel_ms.append(st.ms_kernel)
        rng_ms.append(st.ms_rng)
        rays_local += st.rays_intersect + st.rays_occluded
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays_local], dtype=torch.float64, device=dev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays_total = float(r.item())
    else:
        rays_total = float(rays_local)

    # Instrumented passes (outside the timed region) for the FLOP model:
    # culling off = the reference's own primitive calls one for one
    # (tests/test_gpu_parity.py::test_opcounts_match_reference_without_cull),
    # culling on = what this kernel actually executed.
    st_ops = rtamd.Stats()
    step(flags | rtamd.RT_FLAG_COUNT_OPS | rtamd.RT_FLAG_NO_CULL, st_ops)
    st_exe = rtamd.Stats()
    step(flags | rtamd.RT_FLAG_COUNT_OPS, st_exe)
    torch.cuda.synchronize()

    # Side leg (outside the timed region, not the headline): the NON-PARITY
    # FP32 fast path (RT_FLAG_FP32) on the same frame.
    fp32 = None
    if args.fp32_steps > 0 and not args.fp32:
        st32 = rtamd.Stats()
        f32 = flags | rtamd.RT_FLAG_FP32
        step(f32, st32)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t32 = time.perf_counter()
        rays32, k32 = 0, []
        for _ in range(args.fp32_steps):
            step(f32, st32)
            rays32 += st32.rays_intersect + st32.rays_occluded
            k32.append(st32.ms_kernel)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        e32 = time.perf_counter() - t32
        if dist:
            t = torch.tensor([e32, rays32], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e32 = float(t[0].item())
            r = torch.tensor([rays32], dtype=torch.float64, device=dev)
            dist.all_reduce(r, op=dist.ReduceOp.SUM)
            rays32 = float(r.item())
        fp32 = {"value": round(rays32 / e32 / 1e6, 3), "unit": "Mrays/s",
                "ms_per_step": round(e32 / args.fp32_steps * 1e3, 3),
                "kernel_ms": round(sum(k32) / len(k32), 3), "steps": args.fp32_steps,
                "note": "RT_FLAG_FP32: non-parity fast path, not within the 1e-5 tolerance (tests/test_gpu_fp32.py)"}

    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return 0

    def counted(s):
        d = {rtamd.OP_NAMES[i]: int(s.ops[i]) for i in range(16)}
        d["_occluded"] = int(s.rays_occluded)
        return d

    primary = n_rows * W * (1 if mode == 1 else 8)
    flops, transc = model_flops(counted(st_ops), primary, mode == 1)
    flops_exe, _ = model_flops(counted(st_exe), primary, mode == 1)
    k_ms = sum(kernel_ms) / len(kernel_ms)
    achieved = flops / (k_ms * 1e-3) / 1e12
    value = rays_total / elapsed / 1e6
    rays_per_frame = rays_total / args.steps

    prof_traffic = None
    tpath = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(tpath):
        try:
            with open(tpath) as f:
                tj = json.load(f)
            if tj.get("config") == args.config and world == 1:
                prof_traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            prof_traffic = None

    cpu = None
    if not args.no_cpu and world == 1:
        # bounded sample: a band of rows from the middle of the same frame,
        # single-threaded CPU oracle (C port of the reference path)
        r0 = max(0, H // 2 - args.cpu_rows // 2)
        r1 = min(H, r0 + args.cpu_rows)
        tc = time.perf_counter()
        _, ost = rtamd.oracle_render(sc, W, H, mode, r0, r1, threads=1)
        dt = time.perf_counter() - tc
        cpu_rays = ost.rays_intersect + ost.rays_occluded
        cpu = {"value": round(cpu_rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "port",
               "sample": f"config {args.config} output rows [{r0},{r1}) x {W} px, {cpu_rays} rays in {dt:.1f} s "
                         f"on {platform.processor() or platform.machine()} (oracle/oracle.c, 1 thread)"}
        # the same port over all the cores this job may use
        # (rows split across pthreads; the box grants 16), a 4x larger band
        nt = max(1, min(16, os.cpu_count() or 1))
        r0m = max(0, H // 2 - 2 * args.cpu_rows)
        r1m = min(H, r0m + 4 * args.cpu_rows)
        tc = time.perf_counter()
        _, ostm = rtamd.oracle_render(sc, W, H, mode, r0m, r1m, threads=nt)
        dtm = time.perf_counter() - tc
        raysm = ostm.rays_intersect + ostm.rays_occluded
        cpu["all_cores"] = {"value": round(raysm / dtm / 1e6, 4), "cores": nt,
                            "sample": f"output rows [{r0m},{r1m}) x {W} px, {raysm} rays in {dtm:.1f} s"}

    name = scenes.CONFIGS[args.config][0]
    out = {
        "metric": "Mrays/s (primary+secondary) + wall-clock per frame, 4K scene @1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32" if args.fp32 else "f64",
        "data": "synthetic: reference example scene JSON + mt19937(12345) jitter, rendered on device",
        "config": {"workload": name, "width": W, "height": H, "mode": "paper" if mode else "standard",
                   "rays_per_frame": int(rays_per_frame), "parallelism": f"row-strips{STRIP}x{world}" + (f", gather-to-rank0 in {len(df.bounds)} chunks" if world > 1 else ""),
                   "cull": not args.no_cull},
        "roofline": {"bound": "fp64-valu", "achieved": round(achieved, 3), "peak": FP64_VALU_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / FP64_VALU_PEAK_TFLOPS, 4),
                     "traffic": prof_traffic, "kernel": "k_std" if mode == 0 else "k_paper_primary",
                     "kernel_ms": round(k_ms, 3), "flops_per_launch": flops, "transcendentals": transc,
                     "flops_model": "SURVEY.md 8d table x the reference's own primitive calls (GPU counters, "
                                    "culling off; equal to the CPU oracle's by test)",
                     "executed_flops_per_launch": flops_exe,
                     "executed_frac": round(flops_exe / (k_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS, 4),
                     "hbm_frac": None if prof_traffic is None else
                     round(prof_traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)},
        "rng_ms": round(sum(rng_ms) / len(rng_ms), 3),
        "cpu_baseline": cpu,
        "fp32_fast_path": fp32,
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
