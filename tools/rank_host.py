#!/usr/bin/env python3
"""Host-side split of one simulated rank's frame (GPU box): runs
rt_test_dist_sim_rank for one rank of an N-rank split repeatedly and reads
rt_setup_times' per-frame slots (7: frame begin, 8: trace launches, 9: frame
end, 10: device-group setup; ms) after each call, next to the call's wall
time.  Usage: python tools/rank_host.py [--config 4] [--world 8] [--rank 7] [--reps 20]"""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
import rtamd  # noqa: E402
import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    text, mode = scenes.config_json(a.config)
    sc = rtamd.load_scene_from_json_text(text)
    lib = rtamd.amd_lib()
    lib.rt_test_dist_sim_rank.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(rtamd.Stats)]
    lib.rt_setup_times.argtypes = [C.POINTER(C.c_double), C.c_int]
    st = rtamd.Stats()
    slots = (C.c_double * 11)()
    rows = []
    for i in range(a.reps + 2):
        rtamd.device_synchronize()
        t0 = time.perf_counter()
        rc = lib.rt_test_dist_sim_rank(sc.handle, sc.width, sc.height, mode, 0, a.world, a.rank, 0, C.byref(st))
        wall = (time.perf_counter() - t0) * 1e3
        assert rc == 0, rtamd.last_error()
        lib.rt_setup_times(slots, 11)
        if i >= 2:
            rows.append((wall, slots[7], slots[8], slots[9], slots[10], st.ms_kernel, st.ms_rng))
    med = [statistics.median(c) for c in zip(*rows)]
    print(f"config {a.config} world {a.world} rank {a.rank} (median of {a.reps}): wall {med[0]:.3f} ms | "
          f"frame_begin {med[1]:.3f} trace launches {med[2]:.3f} frame_end {med[3]:.3f} group {med[4]:.3f} | "
          f"kernel {med[5]:.3f} rng {med[6]:.3f}")


if __name__ == "__main__":
    main()
