"""GPU: the parallel mt19937 jitter stream and row-subset rendering.

The jitter KAT is the reference's serial stream (std::mt19937(12345) through
uniform_real_distribution(-0.5, 0.5), tracer.cpp:284-293) as restated by the
oracle, which tests/test_oracle_golden.py pins to the reference's own
libstdc++ draws.  Offsets cover the first draws, segment and checkpoint
boundaries (K = 1024 twist blocks = 638,976 outputs) and the last pixels of
4K and 8K standard-mode frames."""
import ctypes as C

import numpy as np
import pytest

SEG = 1024 * 624
FRAME_4K = 32 * 3840 * 2160
FRAME_8K = 32 * 7680 * 4320


def _device_draws(q0, q1, first, count, K=1024):
    import rtamd

    lib = rtamd.amd_lib()
    lib.rt_test_jitter_device.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                          C.POINTER(C.c_double)]
    out = np.zeros(count)
    rc = lib.rt_test_jitter_device(K, q0, q1, first, count, out.ctypes.data_as(C.POINTER(C.c_double)))
    assert rc == 0, rtamd.last_error()
    return out


def _oracle_draws(first, count):
    import rtamd

    out = np.zeros(count)
    rtamd.oracle_lib().oracle_jitter(first, count, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("q0,q1,first,count", [
    (0, 2 * SEG, 0, 4096),                        # first draws + first segment boundary
    (0, 6 * SEG, SEG // 2 - 100, 400),            # around segment 1 start
    (5 * SEG - 64, 5 * SEG + 4096, 5 * SEG // 2 - 32, 2048),   # band starting mid-frame (checkpoint 5)
    (FRAME_4K - 32 * 3840, FRAME_4K, FRAME_4K // 2 - 16 * 3840, 16 * 3840),   # last row of 4K
    (FRAME_8K - 64, FRAME_8K, FRAME_8K // 2 - 32, 32),                          # last pixels of 8K
])
def test_jitter_stream_matches_serial(gpu, q0, q1, first, count):
    dev = _device_draws(q0, q1, first, count)
    ref = _oracle_draws(first, count)
    assert np.array_equal(dev, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [64, 256, 512])
@pytest.mark.parametrize("q0,q1,first,count", [
    (0, 40 * SEG, 0, 2048),
    (FRAME_4K - 32 * 3840 * 8, FRAME_4K, FRAME_4K // 2 - 16 * 3840 * 8, 16 * 3840 * 8),   # last strip of 4K
])
def test_jitter_stream_short_segments(gpu, K, q0, q1, first, count):
    """The multi-GPU segment lengths (more checkpoints, one more tree level)."""
    assert np.array_equal(_device_draws(q0, q1, first, count, K), _oracle_draws(first, count))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_row_subset_matches_full_frame(gpu, mode):
    """rt_render_rows_device on interleaved 8-row strips (the multi-GPU split)
    reproduces the same rows of the full frame bit for bit."""
    import scenes
    rt = gpu
    text, _ = scenes.config_json(4, dpi=40)   # 160x90 snorlax, 5 lights
    sc = rt.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    full = rt.Tracer(sc, W, H, mode).render()
    lib = rt.amd_lib()
    for world in (2, 3, 5):
        for rank in range(world):
            rows = [r for s in range((H + 7) // 8) if s % world == rank for r in range(s * 8, min(H, s * 8 + 8))]
            buf = rt.DeviceBuffer(len(rows) * W * 3 * 8)
            rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                           buf.ptr, None, None)
            assert rc == 0, rt.last_error()
            got = buf.to_host(np.float64, (len(rows), W, 3))
            assert np.array_equal(got, full[rows]), (world, rank)


@pytest.mark.gpu
def test_unordered_row_subset_and_duplicates(gpu):
    """Rows in arbitrary order (jitter ranges sorted on the host, written to
    their own jitter row) match the full frame; a duplicated row is rejected."""
    import scenes
    rt = gpu
    text, _ = scenes.config_json(4, dpi=40)
    sc = rt.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    full = rt.Tracer(sc, W, H, 0).render()
    lib = rt.amd_lib()
    rng = np.random.default_rng(7)
    rows = [int(r) for r in rng.permutation(H)[: H // 3]]
    buf = rt.DeviceBuffer(len(rows) * W * 3 * 8)
    rc = lib.rt_render_rows_device(sc.handle, W, H, 0, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                   buf.ptr, None, None)
    assert rc == 0, rt.last_error()
    assert np.array_equal(buf.to_host(np.float64, (len(rows), W, 3)), full[rows])
    dup = rows[:4] + rows[:1]
    rc = lib.rt_render_rows_device(sc.handle, W, H, 0, 0, (C.c_int32 * len(dup))(*dup), len(dup),
                                   buf.ptr, None, None)
    assert rc == rt.RT_ERR_INVALID_ARG
    assert "duplicate" in rt.last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_frame_chunks_on_two_streams(gpu, mode):
    """rt_frame_begin / trace (chunks alternating between two HIP streams) /
    end reproduces the rows of the full frame bit for bit, with the same ray
    counts as one rt_render_rows_device call (the bench's multi-GPU path)."""
    import frame_dist
    import scenes
    rt = gpu
    text, _ = scenes.config_json(4, dpi=40)
    sc = rt.load_scene_from_json_text(text)
    W, H = sc.width, sc.height
    full = rt.Tracer(sc, W, H, mode).render()
    lib = rt.amd_lib()
    rows = frame_dist.strip_rows(H, 1, 3)
    streams = [rt.Stream(), rt.Stream()]
    row_bytes = W * 3 * 8
    buf = rt.DeviceBuffer(len(rows) * row_bytes)
    fr = C.c_void_p()
    rc = lib.rt_frame_begin(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                            streams[0].handle, C.byref(fr))
    assert rc == 0, rt.last_error()
    for k, (a, b) in enumerate(frame_dist.chunk_bounds(len(rows), 5)):
        rc = lib.rt_frame_trace(fr, a, b, C.c_void_p(buf.ptr.value + a * row_bytes), streams[k % 2].handle)
        assert rc == 0, rt.last_error()
    st = rt.Stats()
    assert lib.rt_frame_end(fr, C.byref(st)) == 0
    rt.device_synchronize()
    assert np.array_equal(buf.to_host(np.float64, (len(rows), W, 3)), full[rows])
    st1 = rt.Stats()
    buf2 = rt.DeviceBuffer(len(rows) * row_bytes)
    rc = lib.rt_render_rows_device(sc.handle, W, H, mode, 0, (C.c_int32 * len(rows))(*rows), len(rows),
                                   buf2.ptr, None, C.byref(st1))
    assert rc == 0
    assert (st.rays_intersect, st.rays_occluded) == (st1.rays_intersect, st1.rays_occluded)


TSEG = 16 * 624   # checkpoint-table segment: rtamd::kTableK = 16 twist blocks of 624 words (mt_jump.hpp)


@pytest.mark.gpu
@pytest.mark.parametrize("q0,q1,first,count", [
    (0, 3 * TSEG, 0, 4096),                                  # first draws, first table segments
    (0, 6 * TSEG, TSEG // 2 - 100, 400),                     # across a segment start
    (7 * TSEG - 64, 9 * TSEG + 4096, 7 * TSEG // 2 - 32, 2048),   # range starting mid-segment
    (FRAME_4K - 32 * 3840 * 3, FRAME_4K, FRAME_4K // 2 - 16 * 3840 * 3, 16 * 3840 * 3),   # last rows of 4K
    (FRAME_8K - 64, FRAME_8K, FRAME_8K // 2 - 32, 32),       # last pixels of 8K (table of 26.6k checkpoints)
])
def test_jitter_table_path_matches_serial(gpu, q0, q1, first, count):
    """The frame path (K = 0 in the hook): resident checkpoint table every
    kTableK = 16 twist blocks + the one-wavefront fill kernel, draw for draw
    against the serial stream; the cases land on and across segment edges."""
    dev = _device_draws(q0, q1, first, count, K=0)
    ref = _oracle_draws(first, count)
    assert np.array_equal(dev, ref)
