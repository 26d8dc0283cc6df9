#!/usr/bin/env python3
"""bench.py — BASELINE.json headline metric on MI355X.

Metric: Mrays/s (primary + secondary) and wall-clock per frame on config 4:
examples/snorlax.json at 3840x2160, 5 lights, recursion 4.
A "ray" is one Scene::intersect or Scene::occluded query of the reference
(raytracer/src/scene.cpp:10,33).  A "step" renders one whole frame through the
product path rt_render_dist (include/rt.h): jitter stream (mt19937 jump-ahead)
+ trace kernels, with the scene resident on the device and the frame left in
HBM on rank 0.  For N > 1 (one process per GPU, launched by
torch.distributed.run) every rank renders interleaved 8-row strips of the SAME
frame (strong scaling) and rank 0 receives them through RCCL ncclGather over
xGMI inside librtamd.  The process never imports torch: device buffers,
streams, the max-over-ranks timing and the barriers come from librtamd.so
(rt_device_alloc, rt_stream_create, rt_dist_reduce_max / rt_dist_barrier over
RCCL), so the bench runs on /opt/rocm's HIP runtime like the `ray` CLI; the
RCCL id reaches the other ranks through rendezvous.py.

After the timed region (never inside it): op-counted passes for the FLOP
model, the wall-clock split of the CLI's end-to-end path (render + device
toByte + D2H + parallel PNG, and the `ray` binary itself), kernel resources
and occupancy, the trace kernel's HBM traffic from rocprofv3 PMC passes over
the same frame, and the CPU baseline (the C port of the reference path,
oracle/oracle.c, on a whole frame over the host cores plus a 1-thread band).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4]
"""
from __future__ import annotations

import argparse
import csv
import ctypes as C
import glob
import json
import os
import platform
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))

FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector: 256 CU x 64 lanes x 2 x 2.4 GHz
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table
JITTER_BYTES_PER_PX = 128      # 8 samples x (dx, dy) doubles, read once by the trace kernel
FB_BYTES_PER_PX = 24           # RGB doubles written once


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


def pmc_traffic(config: int, timeout: int = 120) -> dict | None:
    """HBM bytes per launch of the trace kernel, measured by rocprofv3 PMC
    passes (one counter per pass, no tracing domains) over tools/one_frame.py
    renders of the same frame.  FETCH_SIZE is doubled per the gfx950
    calibration and both counters are KiB (MI355X_MICROARCH.md §HBM)."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    vals = {}
    tmp = tempfile.mkdtemp(prefix="rt_pmc_")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", ctr, "--output-format", "csv", "-d", out,
                   "-o", "pmc", "--", sys.executable, os.path.join(REPO, "tools", "one_frame.py"), "--config",
                   str(config), "--frames", "2"]
            r = subprocess.run(cmd, capture_output=True, text=True, cwd=REPO)
            if r.returncode != 0:
                return {"error": f"{ctr} pass rc={r.returncode}"}
            per = []
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    n = row.get("Kernel_Name", "")
                    if ("k_std" in n or "k_paper_primary" in n) and row.get("Counter_Name") == ctr:
                        per.append(float(row["Counter_Value"]))
            if not per:
                return {"error": f"{ctr}: no trace-kernel rows"}
            vals[ctr] = sum(per) / len(per)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write = vals["WRITE_SIZE"] * 1024.0
    return {"fetch_bytes": fetch, "write_bytes": write, "bytes": fetch + write}


SPLIT_NAMES = ["call_ms", "agreement_reduce_ms", "agreement_wait_ms", "gather_ms", "placement_ms",
               "last_gather_ms", "last_placement_ms", "tail_ms", "rccl_world", "rows"]


def ranks_block(kernel_ms: list, rng_ms: list, splits: list) -> dict:
    """N > 1: every rank's view of its frame, so that an imbalance or a slow
    collective shows in the driver's own line.  kernel_ms / rng_ms: each
    rank's mean trace-kernel / jitter time over the timed steps; splits: each
    rank's rt_dist_frame_split of its last timed frame (include/rt.h)."""
    world = len(kernel_ms)
    assert len(splits) == world and len(rng_ms) == world
    col = {name: [round(float(sp[i]), 4) for sp in splits] for i, name in enumerate(SPLIT_NAMES)}
    k = [round(float(x), 4) for x in kernel_ms]
    out = {
        "kernel_ms": {"min": min(k), "max": max(k), "per_rank": k,
                      "imbalance": round(max(k) / (sum(k) / world), 4) if sum(k) > 0 else None},
        "rng_ms": [round(float(x), 4) for x in rng_ms],
        "rows": [int(x) for x in col["rows"]],
        "rccl_world": sorted(set(int(x) for x in col["rccl_world"])),
        "agreement_ms": {"reduce_device": col["agreement_reduce_ms"], "verdict_wait_host": col["agreement_wait_ms"]},
        "gather_ms": {"per_rank": col["gather_ms"], "last_chunk_per_rank": col["last_gather_ms"]},
        "placement_ms": {"root_total": col["placement_ms"][0], "root_last_chunk": col["last_placement_ms"][0]},
        "call_ms": col["call_ms"],
        "tail_ms": col["tail_ms"],
        "note": "rt_dist_frame_split of each rank's last timed frame; kernel/rng = means over the timed steps",
    }
    return out


def host_cpu() -> dict:
    """The CPU the baseline ran on (report nproc and the model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"model": model or platform.processor() or platform.machine(), "nproc": os.cpu_count(),
            "usable_cpus": usable,
            "note": "nproc counts the whole machine; the GPU box grants this job 16 of them (OMP_NUM_THREADS)"}


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (one per GPU, LOCAL_RANK = GPU index) with the environment
    torch.distributed.run would give them, BEFORE this process makes any HIP
    call (it never makes one), and exit with their status.  Rank 0 prints the
    JSON line; the others print nothing on stdout.  If a rank fails, the
    others are stopped (they would wait in a collective for it)."""
    import uuid

    port = str(_free_port())
    run_id = uuid.uuid4().hex[:12]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RTAMD_RUN_ID=run_id,
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      start_new_session=True))
    # the ranks run in their own sessions (a terminal's job-control signals do
    # not reach them), so a SIGTERM / SIGINT to this process stops them first
    import signal

    def _stop(signum, frame):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        signal.signal(signum, signal.SIG_DFL)
        os.kill(os.getpid(), signum)

    old_handlers = {sig: signal.signal(sig, _stop) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        live = list(range(n))
        while live:
            time.sleep(0.05)
            for r in list(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.remove(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench.py: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    for q in live:
                        procs[q].terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for sig, h in old_handlers.items():
            signal.signal(sig, h)
        try:   # the id file (rendezvous._path: port + run id)
            os.unlink(os.path.join(tempfile.gettempdir(), f"rtamd_uid_{port}_{run_id}"))
        except FileNotFoundError:
            pass
    return rc


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Without a launcher's RANK/WORLD_SIZE, bench.py starts them itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up ranks and the id exchange, print each rank's view, stop before any GPU call")
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--cpu-rows", type=int, default=64, help="rows of the 1-thread CPU-oracle band")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 traffic passes")
    ap.add_argument("--no-cli", action="store_true", help="skip the end-to-end CLI wall-clock leg")
    ap.add_argument("--no-cull", action="store_true", help="disable wave-uniform bound culling")
    ap.add_argument("--fp32", action="store_true",
                    help="time the NON-PARITY FP32 fast path as the headline (RT_FLAG_FP32); default is FP64")
    ap.add_argument("--fp32-steps", type=int, default=20, help="frames of the FP32 side leg (0 = skip)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    import rendezvous

    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:])
    rank, world, local = rendezvous.env_ranks()
    if world != args.gpus:
        # never print a line whose n_gpus is not the --gpus asked for
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2

    if args.dry_run:
        got = rendezvous.share_bytes(rank, bytes(range(128)) if rank == 0 else None, 128) if world > 1 else b""
        print(json.dumps({"dry_run": True, "rank": rank, "world": world, "local_rank": local,
                          "id_ok": world == 1 or got == bytes(range(128))}), flush=True)
        return 0

    import numpy as np  # noqa: F401

    import rtamd
    import scenes

    # No torch here: librtamd.so brings its own HIP runtime (/opt/rocm's, the
    # one `ray` uses) and does the collectives over RCCL itself; a second,
    # torch-bundled runtime in the same process is refused (rtamd.amd_lib).
    lib = rtamd.amd_lib()
    rtamd.set_device(local)

    text, mode = scenes.config_json(args.config)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    flags = rtamd.RT_FLAG_NO_CULL if args.no_cull else rtamd.RT_FLAG_NONE
    if args.fp32:
        flags |= rtamd.RT_FLAG_FP32

    # the product's distribution: rank 0 makes the RCCL id, every rank binds its GPU
    uid = (C.c_uint8 * 128)()
    if rank == 0 and lib.rt_dist_get_id(uid) != 0:
        raise RuntimeError(rtamd.last_error())
    if world > 1:
        got = rendezvous.share_bytes(rank, bytes(uid) if rank == 0 else None, 128)
        uid = (C.c_uint8 * 128)(*got)
    dh = C.c_void_p()
    if lib.rt_dist_create(uid, world, rank, C.byref(dh)) != 0:
        raise RuntimeError(f"rt_dist_create failed: {rtamd.last_error()}")
    if world > 1:
        if lib.rt_dist_barrier(dh) != 0:   # every rank holds the communicator: the id file can go
            raise RuntimeError(f"rt_dist_barrier failed: {rtamd.last_error()}")
        rendezvous.cleanup(rank)

    def reduce_max(vals):
        v = (C.c_double * len(vals))(*[float(x) for x in vals])
        if lib.rt_dist_reduce_max(dh, v, len(vals)) != 0:
            raise RuntimeError(f"rt_dist_reduce_max failed: {rtamd.last_error()}")
        return list(v)

    def reduce_sum(vals):   # per-rank slots, max-reduced, summed on the host
        slots = [0.0] * (len(vals) * world)
        for i, x in enumerate(vals):
            slots[i * world + rank] = float(x)
        m = reduce_max(slots)
        return [sum(m[i * world:(i + 1) * world]) for i in range(len(vals))]

    def barrier():
        if lib.rt_dist_barrier(dh) != 0:
            raise RuntimeError(f"rt_dist_barrier failed: {rtamd.last_error()}")

    n_rows = len(rtamd.dist_rows(H, world, rank, mode))
    frame = rtamd.DeviceBuffer(H * W * 3 * 8) if rank == 0 else None
    frame_ptr = frame.ptr if frame is not None else None
    stream = rtamd.Stream()
    st = rtamd.Stats()

    def step(f=flags, stats=st):
        rc = lib.rt_render_dist(dh, sc.handle, W, H, mode, f, frame_ptr, stream.handle, C.byref(stats))
        if rc != 0:
            raise RuntimeError(f"rt_render_dist failed ({rc}): {rtamd.last_error()}")

    t_first = time.perf_counter()
    step()   # first frame: kernels load, jitter plan + checkpoint table, scene upload
    first_ms = (time.perf_counter() - t_first) * 1e3
    for _ in range(max(0, args.warmup - 1)):
        step()
    rtamd.device_synchronize()
    barrier()
    rtamd.device_synchronize()
    kernel_ms, rng_ms, gather_ms, rays_local, traced_local = [], [], [], 0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kernel_ms.append(st.ms_kernel)
        rng_ms.append(st.ms_rng)
        gather_ms.append(st.ms_gather)
        rays_local += st.rays_intersect + st.rays_occluded
        traced_local += st.rays_traced
    rtamd.device_synchronize()
    barrier()
    rtamd.device_synchronize()
    elapsed = time.perf_counter() - t0
    k_ms = sum(kernel_ms) / len(kernel_ms)
    ranks = None
    if world > 1:
        elapsed, k_ms_max = reduce_max([elapsed, k_ms])
        rays_total, traced_total = reduce_sum([rays_local, traced_local])
        # every rank's split of its last timed frame (after the timed region)
        sp = (C.c_double * len(SPLIT_NAMES))()
        if lib.rt_dist_frame_split(dh, sp, len(SPLIT_NAMES)) < 0:
            raise RuntimeError(f"rt_dist_frame_split failed: {rtamd.last_error()}")
        mine = [k_ms, sum(rng_ms) / len(rng_ms)] + list(sp)
        per = len(mine)
        slots = [-1e300] * (per * world)
        slots[rank * per:(rank + 1) * per] = mine
        allv = reduce_max(slots)
        rows_v = [allv[r * per:(r + 1) * per] for r in range(world)]
        ranks = ranks_block([v[0] for v in rows_v], [v[1] for v in rows_v], [v[2:] for v in rows_v])
    else:
        k_ms_max, rays_total, traced_total = k_ms, float(rays_local), float(traced_local)

    # Instrumented passes (outside the timed region) for the FLOP model:
    # culling off = the reference's own primitive calls one for one
    # (tests/test_gpu_parity.py::test_opcounts_match_reference_without_cull),
    # culling on = what this kernel actually executed.
    def counted_pass(f):
        s = rtamd.Stats()
        step(f, s)
        v = [int(s.ops[i]) for i in range(16)] + [int(s.rays_occluded)]
        if world > 1:
            v = [int(x) for x in reduce_sum(v)]
        d = {rtamd.OP_NAMES[i]: v[i] for i in range(16)}
        d["_occluded"] = v[16]
        return d

    ops_ref = counted_pass(flags | rtamd.RT_FLAG_COUNT_OPS | rtamd.RT_FLAG_NO_CULL)
    ops_exe = counted_pass(flags | rtamd.RT_FLAG_COUNT_OPS)
    rtamd.device_synchronize()

    # Side leg (outside the timed region, not the headline): the NON-PARITY
    # FP32 fast path (RT_FLAG_FP32) on the same frame.
    fp32 = None
    if args.fp32_steps > 0 and not args.fp32:
        st32 = rtamd.Stats()
        f32 = flags | rtamd.RT_FLAG_FP32
        step(f32, st32)
        rtamd.device_synchronize()
        barrier()
        t32 = time.perf_counter()
        rays32, k32 = 0, []
        for _ in range(args.fp32_steps):
            step(f32, st32)
            rays32 += st32.rays_intersect + st32.rays_occluded
            k32.append(st32.ms_kernel)
        rtamd.device_synchronize()
        barrier()
        e32 = time.perf_counter() - t32
        if world > 1:
            e32 = reduce_max([e32])[0]
            rays32 = reduce_sum([rays32])[0]
        fp32 = {"value": round(rays32 / e32 / 1e6, 3), "unit": "Mrays/s",
                "ms_per_step": round(e32 / args.fp32_steps * 1e3, 3),
                "kernel_ms": round(sum(k32) / len(k32), 3), "steps": args.fp32_steps,
                "note": "RT_FLAG_FP32: non-parity fast path, not within the 1e-5 tolerance (tests/test_gpu_fp32.py)"}

    def teardown():
        stream.destroy()
        if frame is not None:
            frame.free()
        lib.rt_dist_destroy(dh)
        rtamd.shutdown()

    if rank != 0:
        barrier()
        teardown()
        return 0

    primary = H * W * (1 if mode == 1 else 8)
    flops, transc = model_flops(ops_ref, primary, mode == 1)
    flops_exe, _ = model_flops(ops_exe, primary, mode == 1)
    achieved = flops / (k_ms_max * 1e-3) / 1e12 / world   # per GPU: each rank's kernel covers 1/world of the frame
    value = rays_total / elapsed / 1e6
    rays_per_frame = rays_total / args.steps

    # Wall-clock split of the CLI's end-to-end path, N = 1:
    # render + device toByte + D2H of 3 B/px (rt_render_rgb8), the parallel
    # PNG deflate, and the `ray` binary itself (process start to exit).
    wall = {"rng": round(sum(rng_ms) / len(rng_ms), 3), "kernel": round(k_ms, 3),
            "gather": round(sum(gather_ms) / len(gather_ms), 3)}
    if world == 1:
        s8 = rtamd.Stats()
        rtamd.render_rgb8(sc, W, H, mode, 1, flags, s8)
        tr = time.perf_counter()
        rgb = rtamd.render_rgb8(sc, W, H, mode, 1, flags, s8)
        wall["render_rgb8_total"] = round((time.perf_counter() - tr) * 1e3, 3)
        wall["tobyte"] = round(s8.ms_tobyte, 3)
        wall["d2h"] = round(s8.ms_d2h, 3)
        nt = max(1, min(16, os.cpu_count() or 1))
        with tempfile.TemporaryDirectory() as td:
            tp = time.perf_counter()
            rtamd.write_png(os.path.join(td, "f.png"), rgb, threads=nt)
            wall["png"] = round((time.perf_counter() - tp) * 1e3, 3)
            wall["png_threads"] = nt
            if not args.no_cli:
                js = os.path.join(td, "scene.json")
                with open(js, "w") as f:
                    f.write(text)
                cmd = [os.path.join(REPO, "raytracing-project_amd", "bin", "ray"), js, os.path.join(td, "cli.png")]
                cmd += (["--paper"] if mode == 1 else []) + ["--stats", "--threads", str(nt)]
                tc = time.perf_counter()
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
                wall["cli_total"] = round((time.perf_counter() - tc) * 1e3, 3)
                if r.returncode == 0:
                    lines = r.stdout.strip().splitlines()
                    cs = json.loads(lines[-1])
                    wall["cli_split"] = {k: cs[k] for k in ("ms_load", "ms_rng", "ms_kernel", "ms_tobyte", "ms_d2h",
                                                            "ms_render", "ms_png", "ms_main")}
                    if len(lines) >= 2 and lines[-2].startswith("{"):
                        wall["cli_setup"] = json.loads(lines[-2])   # one-time costs inside ms_render
                else:
                    wall["cli_error"] = r.stderr[-300:]
        wall["note"] = ("cli_total = the `ray` process end to end (HIP init, JSON load, first-frame device "
                        "setup, render, PNG); cli_split = its own timers")

    # Kernel resources / occupancy of the timed trace kernel.
    ki = (C.c_int32 * 8)()
    occupancy = None
    if lib.rt_test_kernel_info(sc.handle, mode, flags, ki) == 0:
        occupancy = {"vgprs": ki[0], "scratch_bytes_per_lane": ki[1], "lds_bytes": ki[2],
                     "workgroups_per_cu": ki[3], "waves_per_simd": ki[4], "max_waves_per_simd": 8}
    kname = C.create_string_buffer(160)
    kernel_name = "k_std" if mode == 0 else "k_paper_primary"
    if hasattr(lib, "rt_test_kernel_name") and lib.rt_test_kernel_name(sc.handle, mode, flags, kname, 160) == 0:
        kernel_name = kname.value.decode()   # as rocprofv3 names it (profiles/*kernel_stats.csv)

    # HBM: algorithmic bytes of the trace kernel per launch vs counter-measured traffic.
    px = n_rows * W
    alg_bytes = px * (FB_BYTES_PER_PX + (JITTER_BYTES_PER_PX if mode == 0 else 0))
    traffic = None
    if world == 1 and not args.no_pmc:
        try:
            traffic = pmc_traffic(args.config)
        except Exception as e:   # profiler unavailable: report, do not fail the bench
            traffic = {"error": str(e)[:200]}

    cpu = None
    if not args.no_cpu and world == 1:
        nt = max(1, min(16, os.cpu_count() or 1))
        tc = time.perf_counter()
        _, ostm = rtamd.oracle_render(sc, W, H, mode, 0, H, threads=nt)
        dtm = time.perf_counter() - tc
        raysm = ostm.rays_intersect + ostm.rays_occluded
        cpu = {"value": round(raysm / dtm / 1e6, 4), "unit": "Mrays/s", "cores": nt, "kind": "port",
               "sample": f"whole config-{args.config} frame {W}x{H}: {raysm} rays in {dtm:.1f} s on {nt} threads "
                         f"(oracle/oracle.c, rows split across threads; {platform.machine()} host)",
               "host": host_cpu()}
        # faithful to the reference: one thread, a band through the middle of the frame
        r0 = max(0, H // 2 - args.cpu_rows // 2)
        r1 = min(H, r0 + args.cpu_rows)
        tc = time.perf_counter()
        _, ost = rtamd.oracle_render(sc, W, H, mode, r0, r1, threads=1)
        dt = time.perf_counter() - tc
        cpu_rays = ost.rays_intersect + ost.rays_occluded
        cpu["one_thread"] = {"value": round(cpu_rays / dt / 1e6, 4), "cores": 1,
                             "sample": f"output rows [{r0},{r1}) x {W} px, {cpu_rays} rays in {dt:.1f} s"}

    name = scenes.CONFIGS[args.config][0]
    hbm = {"algorithmic_bytes_per_launch": alg_bytes,
           "algorithmic_GBs": round(alg_bytes / (k_ms * 1e-3) / 1e9, 1),
           "algorithmic_frac": round(alg_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    traffic_bytes = None
    if traffic and "bytes" in traffic:
        traffic_bytes = traffic["bytes"]
        hbm.update({"counter_fetch_bytes": traffic["fetch_bytes"], "counter_write_bytes": traffic["write_bytes"],
                    "counter_frac": round(traffic_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                    "counter_source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/one_frame.py in "
                                      "this run (FETCH x2, KiB -> B: MI355X_MICROARCH.md §HBM)"})
    elif traffic:
        hbm["counter_error"] = traffic.get("error")
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
                   "rays_per_frame": int(rays_per_frame), "rays_traced_per_frame": int(traced_total / args.steps),
                   "parallelism": f"{world} ranks, 1 GPU each: row-strips{30 if mode == 1 else 8}x{world}" +
                                  (", RCCL ncclGather to rank 0 in 4 chunks" if world > 1 else ""),
                   "cull": not args.no_cull},
        "roofline": {"bound": "fp64-valu", "achieved": round(achieved, 3), "peak": FP64_VALU_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / FP64_VALU_PEAK_TFLOPS, 4),
                     "traffic": traffic_bytes, "kernel": kernel_name,
                     "kernel_ms": round(k_ms, 3), "flops_per_launch": flops / world, "transcendentals": transc,
                     "flops_model": "SURVEY.md 8d table x the reference's own primitive calls (GPU counters, "
                                    "culling off; equal to the CPU oracle's by test)",
                     "executed_flops_per_launch": flops_exe / world,
                     "executed_frac": round(flops_exe / world / (k_ms_max * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS, 4),
                     "occupancy": occupancy, "hbm": hbm},
        "wall_clock_ms": wall,
        "first_frame_ms": round(first_ms, 1),
        "cpu_baseline": cpu,
        "fp32_fast_path": fp32,
    }
    if ranks is not None:
        out["ranks"] = ranks
    print(json.dumps(out), flush=True)
    barrier()
    teardown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
