"""N>1 path on CPU: world_size 2 with the gloo backend.

Each rank renders its interleaved row strips (standard mode: every strip
starts its own mt19937 stream offset; paper mode: neighbour rows outside the
strip are re-traced), the padded row buffers go through frame_dist.DistFrame
- a Python twin of the product's partition and chunked gather-to-rank-0
layout (rt_dist.hip; tests/test_host_lib.py pins the partitions equal) - and
rank 0 scatters them into the frame.  The per-rank renderer here is the CPU
oracle (test infrastructure), so this test pins the partition / stream
offsets / gather / scatter LOGIC over a real two-process torch.distributed
group; it does not run the product's C++ rank protocol (dist_frame: frame
agreements, RCCL gathers, placement, failure verdicts), which
tests/test_gpu_dist_threads.py executes with concurrent ranks on one GPU, nor
the GPU kernels (tests/test_gpu_jitter_rows.py)."""
import os
import socket

import multiprocessing as mp

import numpy as np
import pytest

# torch is imported only inside the spawned ranks: the pytest process itself
# keeps one HIP runtime (/opt/rocm's, the one librtamd.so binds; rtamd
# refuses a process where torch's bundled runtime is mapped too).


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, text, mode, out_path):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "raytracing-project_amd", "python"))
    import torch
    import torch.distributed as dist

    import frame_dist
    import rtamd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = rtamd.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    df = frame_dist.DistFrame(W, H, rank, world, "cpu", chunks=3, strip=frame_dist.strip_for(mode))

    def trace_chunk(a, b, out, stream):   # row by row: arbitrary stream offsets
        for k in range(a, b):
            r = df.rows[k]
            fb, _ = rtamd.oracle_render(sc, W, H, mode, r, r + 1)
            out[k - a] = torch.from_numpy(fb[0])

    def scatter(src, slot_rows, full):
        keep = slot_rows >= 0
        full[slot_rows[keep].long()] = src[keep]

    frame = df.run(trace_chunk, dist, scatter)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", [0, 1])
def test_two_rank_strip_frame_matches_single(rt, tmp_path, mode):
    import scenes

    text, _ = scenes.config_json(4, dpi=12)   # 48x27 snorlax, 5 lights
    out = str(tmp_path / "frame.npy")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, text, mode, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = np.load(out)
    sc = rt.load_scene_from_json_text(text)
    want, _ = rt.oracle_render(sc, sc.width, sc.height, mode)
    assert np.array_equal(got, want)


def test_strip_partition_covers_frame():
    import frame_dist

    for H in (1, 7, 8, 9, 90, 2160):
        for world in (1, 2, 3, 8):
            allr = sorted(r for k in range(world) for r in frame_dist.strip_rows(H, k, world))
            assert allr == list(range(H))
            idx = frame_dist.gather_row_index(H, world)
            assert len(idx) == world * frame_dist.max_rows(H, world)
            assert sorted(r for r in idx if r >= 0) == list(range(H))
            m = frame_dist.max_rows(H, world)
            for chunks in (1, 3, 4, 64):
                for strip in (1, 8, 30):
                    b = frame_dist.chunk_bounds(m, chunks, strip)
                    assert b[0][0] == 0 and b[-1][1] == m
                    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
                    assert all(a % strip == 0 for a, _ in b)   # chunks never split a strip


def _rdv_worker(rank, tag, out):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "raytracing-project_amd", "python"))
    import rendezvous

    data = bytes(range(128)) if rank == 0 else None
    got = rendezvous.share_bytes(rank, data, 128, tag=tag, timeout=60)
    with open(f"{out}.{rank}", "wb") as f:
        f.write(got)


def test_rendezvous_hands_rank0_bytes_to_every_rank(tmp_path):
    """bench.py's torch-free id exchange (rendezvous.share_bytes): three
    processes, rank 0 publishing after the others start polling."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "raytracing-project_amd", "python"))
    import rendezvous

    tag = f"test_{os.getpid()}"
    out = str(tmp_path / "got")
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rdv_worker, args=(r, tag, out)) for r in (2, 1, 0)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(3):
        assert open(f"{out}.{r}", "rb").read() == bytes(range(128))
    rendezvous.cleanup(0, tag=tag)
    assert not os.path.exists(rendezvous._path(tag))
