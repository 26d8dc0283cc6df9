"""The world >= 2 rank protocol of distributed frames, executed (SURVEY.md
§8e; the reference's frame loop is raytracer/src/tracer.cpp:247-300).

rt_test_dist_threads runs the ranks of a distributed frame CONCURRENTLY on
one GPU: one host thread per rank, each with its own streams and device
workspace, through the product's rank path (rt_dist.hip dist_frame) with RCCL
replaced by a same-device transport that keeps its contract (every rank issues
the same collectives, each ordered on the rank's collective stream; host
rendezvous + device copies / max reduction; rendezvous bounded by the rank's
timeout).  So the code the first multi-GPU run executes - the partition, the
chunked gathers and the root's placement, the frame agreement (descriptor as
v / -v maxima + setup status) and the trace-status agreement, their verdicts
for world >= 2, and the timeouts - runs here at world 2, 3 and 8 on config 4
(dpi 40) and config 5 in paper mode:

* fault-free frames are bit-exact to rt_render, frame after frame;
* ranks that disagree on the frame descriptor all return RT_ERR_INVALID_ARG
  naming the field;
* a rank failing before its frame begins makes every rank return RT_ERR_HIP,
  the others naming it; the next frame is bit-exact;
* a rank failing mid-trace (after the agreement) makes every rank return
  RT_ERR_HIP, the others naming it "failed while tracing" (frames of >= 2
  chunks per rank at every world); the next frame is bit-exact;
* a rank that loaded another scene, or whose root strip shed differs, makes
  every rank refuse the frame naming "scene" / the shed;
* one set of ranks renders several scenes in sequence, each bit-exact;
* a rank that never takes part (a dead peer) makes every other rank give up
  with RT_ERR_HIP within its timeout - no thread outlives it.
"""
import ctypes as C
import json

import numpy as np
import pytest

import scenes

RT_ERR_INVALID_ARG = -1
RT_ERR_HIP = -5

CASES = {
    "cfg4_std": (lambda: scenes.config_json(4, dpi=40)[0], 0),
    "cfg5_paper": (lambda: scenes.config_json(5, dpi=40)[0], 1),
    # (mid-trace failures: >= 2 row chunks per rank at world 8 needs a rank
    # owning 2 strips; paper strips are 30 rows, so 360 rows = 12 strips)
    "cfg5_paper_tall": (lambda: scenes.config_json(5, dpi=160)[0], 1),
}
BASE_CASES = ["cfg4_std", "cfg5_paper"]
WORLDS = [2, 3, 8]

_want_cache = {}


def _case(gpu, name):
    text, mode = CASES[name]
    sc = gpu.load_scene_from_json_text(text())
    W, H = sc.width, sc.height
    if name not in _want_cache:
        _want_cache[name] = gpu.Tracer(sc, W, H, mode).render()
    return sc, mode, W, H, _want_cache[name]


def _others(world, k):
    return [r for r in range(world) if r != k]


@pytest.mark.gpu
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("name", BASE_CASES)
def test_concurrent_ranks_bit_exact(gpu, name, world):
    """Frame after frame (paper frames launch their primary blocks
    costliest first from the second frame on)."""
    sc, mode, W, H, want = _case(gpu, name)
    out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=4)
    assert (rc == 0).all(), msg
    for f in range(4):
        assert np.array_equal(out[f], want), f"frame {f}"
    out8, rc8, _, msg8 = gpu.dist_threads(sc, W, H, mode, world, frames=1, rgb8=True)
    assert (rc8 == 0).all(), msg8
    assert np.array_equal(out8[0], gpu.to_rgb8(want))


@pytest.mark.gpu
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("name", BASE_CASES)
@pytest.mark.parametrize("fault,field", [(4, "flags"), (3, "H")])
def test_descriptor_mismatch_every_rank_invalid_arg(gpu, name, world, fault, field):
    sc, mode, W, H, want = _case(gpu, name)
    k = world - 1 if fault == 3 else 0   # (the root itself may be the odd one)
    out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2, fault=fault, fault_rank=k)
    assert (rc[0] == RT_ERR_INVALID_ARG).all(), (rc[0], msg[0])
    for r in range(world):
        assert "disagree on the frame" in msg[0][r] and field in msg[0][r], msg[0][r]
    assert (rc[1] == 0).all(), msg[1]
    assert np.array_equal(out[1], want)


@pytest.mark.gpu
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("name", BASE_CASES)
def test_setup_failure_named_by_every_rank(gpu, name, world):
    sc, mode, W, H, want = _case(gpu, name)
    k = world // 2
    out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2, fault=gpu.FAULT_SETUP, fault_rank=k)
    assert (rc[0] == RT_ERR_HIP).all(), (rc[0], msg[0])
    assert "injected setup failure" in msg[0][k], msg[0][k]
    for r in _others(world, k):
        assert f"rank(s) {k} failed to set up" in msg[0][r], msg[0][r]
    assert (rc[1] == 0).all(), msg[1]
    assert np.array_equal(out[1], want)


@pytest.mark.gpu
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("name", ["cfg4_std", "cfg5_paper_tall"])
def test_mid_frame_trace_failure_then_next_frame_exact(gpu, name, world):
    """The failure hits the middle of the frame's row chunks (rt_dist.hip
    chunk_bounds: <= 4, whole strips of the largest share), after the first
    agreement: every world here has >= 2 chunks, so the verdict always comes
    from the trace-status agreement."""
    sc, mode, W, H, want = _case(gpu, name)
    k = 0 if world == 2 else world - 2
    rows = (C.c_int32 * H)()
    m = max(gpu.amd_lib().rt_dist_rows_mode(H, world, r, mode, rows) for r in range(world))
    strip = 30 if mode == 1 else 8
    assert min(4, (m + strip - 1) // strip) >= 2, (name, world, m)
    out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2, fault=gpu.FAULT_TRACE, fault_rank=k)
    assert (rc[0] == RT_ERR_HIP).all(), (rc[0], msg[0])
    assert "injected trace failure" in msg[0][k], msg[0][k]
    for r in _others(world, k):
        assert f"rank(s) {k} failed while tracing" in msg[0][r], msg[0][r]
    assert (rc[1] == 0).all(), msg[1]
    assert np.array_equal(out[1], want)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("name", BASE_CASES)
@pytest.mark.parametrize("fault,field", [("scene", "scene"), ("shed", "RT_ROOT_SHED_STD, RT_ROOT_SHED_PAPER")])
def test_scene_or_shed_mismatch_every_rank_invalid_arg(gpu, name, world, fault, field):
    """A rank that loaded another scene (its content hash differs), or whose
    root strip shed differs (it would trace another partition than the root
    places), is refused by every rank; the next frame is bit-exact."""
    sc, mode, W, H, want = _case(gpu, name)
    k = world - 1
    if fault == "scene":
        d = json.loads(CASES[name][0]())
        d.setdefault("medium", {})["ambient"] = [0.123, 0.123, 0.123]
        alt = gpu.load_scene_from_json_text(json.dumps(d))
        out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2, fault=gpu.FAULT_DESC_SCENE, fault_rank=k,
                                            alt_scene=alt)
    else:
        out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2, fault=gpu.FAULT_DESC_SHED, fault_rank=k)
    assert (rc[0] == RT_ERR_INVALID_ARG).all(), (rc[0], msg[0])
    for r in range(world):
        assert "disagree on the frame" in msg[0][r] and f"({field})" in msg[0][r], msg[0][r]
    assert (rc[1] == 0).all(), msg[1]
    assert np.array_equal(out[1], want)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [3])
def test_same_ranks_render_scenes_in_sequence(gpu, world):
    """One set of rank handles renders A, B, A, B (a rank's scene cache and
    content-hash cache reused across scenes): every frame bit-exact."""
    a, mode, W, H, want_a = _case(gpu, "cfg4_std")
    d = json.loads(scenes.config_json(4, dpi=40)[0])
    d["background"] = [0.3, 0.2, 0.1]
    b = gpu.load_scene_from_json_text(json.dumps(d))
    assert (b.width, b.height) == (W, H)
    want_b = gpu.Tracer(b, W, H, mode).render()
    assert not np.array_equal(want_a, want_b)
    out, rc, ms, msg = gpu.dist_threads(a, W, H, mode, world, frames=4, frame_scenes=[a, b, a, b])
    assert (rc == 0).all(), msg
    for f, w in enumerate([want_a, want_b, want_a, want_b]):
        assert np.array_equal(out[f], w), f"frame {f}"


@pytest.mark.gpu
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("name", BASE_CASES)
def test_absent_rank_every_other_rank_gives_up_in_time(gpu, name, world):
    """A peer that never takes part: every other rank returns RT_ERR_HIP,
    naming the timeout, within its timeout plus its own frame setup (a warm
    frame first, so setup is the steady-state cost)."""
    sc, mode, W, H, want = _case(gpu, name)
    timeout = 400
    k = world - 1
    out, rc, ms, msg = gpu.dist_threads(sc, W, H, mode, world, frames=2, fault=gpu.FAULT_ABSENT, fault_rank=k,
                                        fault_frame=1, timeout_ms=timeout)
    assert (rc[0] == 0).all(), msg[0]
    assert np.array_equal(out[0], want)
    assert rc[1][k] == gpu.RANK_ABSENT
    for r in _others(world, k):
        assert rc[1][r] == RT_ERR_HIP, (r, msg[1][r])
        assert "timed out after 400 ms" in msg[1][r] or "aborted" in msg[1][r], msg[1][r]
        # the call gives up at its deadline: the timeout plus this rank's own
        # (warm) work before its first rendezvous, never the peers' lifetime
        assert ms[1][r] < timeout + 600, (r, ms[1][r], msg[1][r])
    print(f"absent rank {k} of {world}: others returned after "
          f"{', '.join(f'{ms[1][r]:.0f}' for r in _others(world, k))} ms")


@pytest.mark.gpu
def test_concurrent_ranks_odd_frames(gpu):
    """Partial strips, ranks without rows and chunk counts that differ between
    ranks, concurrently (paper mode traces each strip's neighbour rows)."""
    d = json.loads(scenes.config_json(4, dpi=24)[0])
    for (w, h, world) in [(37, 29, 3), (24, 5, 8), (64, 61, 2)]:
        scr = d["screen"]
        dims = scr.get("dimensions", [1, 1])
        cx, cy = scr["position"][0] + dims[0] / 2, scr["position"][1] + dims[1] / 2
        e = json.loads(json.dumps(d))
        e["screen"]["dpi"] = 16
        e["screen"]["dimensions"] = [w / 16, h / 16]
        e["screen"]["position"] = [cx - w / 32, cy - h / 32, scr["position"][2]]
        sc = gpu.load_scene_from_json_text(json.dumps(e))
        assert (sc.width, sc.height) == (w, h)
        for mode in (0, 1):
            want = gpu.Tracer(sc, w, h, mode).render()
            out, rc, ms, msg = gpu.dist_threads(sc, w, h, mode, world, frames=2)
            assert (rc == 0).all(), msg
            assert np.array_equal(out[0], want) and np.array_equal(out[1], want)
