"""C-ABI libraries: exports, host helpers (PNG writer, toByte), CLI error
paths and the jump-ahead polynomials.  No GPU compute here."""
import ctypes as C
import json
import os
import re
import struct
import subprocess
import zlib

import numpy as np
import pytest

from conftest import REPO

INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(REPO, "raytracing-project_amd", "lib")
RAY = os.path.join(REPO, "raytracing-project_amd", "bin", "ray")


def _declared_functions(header):
    text = open(os.path.join(INCLUDE, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rt_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_libraries_export_every_declared_symbol():
    host = C.CDLL(os.path.join(LIB, "librt_host.so"), mode=C.RTLD_GLOBAL)
    amd = C.CDLL(os.path.join(LIB, "librtamd.so"), mode=C.RTLD_GLOBAL)
    declared = _declared_functions("rt.h") + _declared_functions("rt_test.h")
    assert len(declared) >= 18 and "rt_render" in declared and "rt_last_error" in declared
    for name in declared:
        assert hasattr(host, name) or hasattr(amd, name), name
    assert amd.rt_abi_version() == 6


@pytest.mark.parametrize("H,world", [(2160, 8), (2160, 3), (1080, 2), (17, 4), (5, 8), (1, 1), (4320, 8)])
@pytest.mark.parametrize("mode,S", [(0, 8), (1, 30)])
def test_dist_partition(rt, H, world, mode, S):
    """rt_dist_rows_mode: interleaved strips of RT_STRIP_ROWS
    (paper mode RT_PAPER_STRIP_ROWS), every output row on exactly one rank,
    ascending per rank, balanced to a strip."""
    import frame_dist

    rows = [rt.dist_rows(H, world, r, mode) for r in range(world)]
    flat = sorted(x for rr in rows for x in rr)
    assert flat == list(range(H))
    own = frame_dist.strip_owners((H + S - 1) // S, world, mode)
    for r, rr in enumerate(rows):
        assert rr == sorted(rr)
        assert all(own[x // S] == r for x in rr)   # whole strips
    # the non-root ranks balanced to a strip; the root near its weight
    n_strips = [sum(1 for o in own if o == r) for r in range(world)]
    if world > 1:
        assert max(n_strips[1:]) - min(n_strips[1:]) <= 1
        w0 = max(500, 1000 - frame_dist.ROOT_SHED[mode] * world) / 1000
        assert abs(n_strips[0] - w0 * (len(own) - n_strips[0]) / (world - 1)) <= 1.5
    if mode == 0:
        assert rows == [rt.dist_rows(H, world, r) for r in range(world)]   # rt_dist_rows = standard


def test_strip_owners_rotate_per_round():
    """Equal weights (RGB8 output): round k of `world` strips starts at rank
    k mod world, so no rank owns one phase of the world*S-row period."""
    import frame_dist

    own = frame_dist.strip_owners(64, 8, mode=0, kind=1)
    for k in range(8):
        assert own[8 * k:8 * k + 8] == [(k + i) % 8 for i in range(8)]


def test_dist_partition_matches_python_mirror(rt):
    import frame_dist
    for H, world in [(2160, 8), (1081, 3), (7, 2), (4320, 8), (4320, 5)]:
        for mode in (0, 1):
            for r in range(world):
                assert rt.dist_rows(H, world, r, mode) == frame_dist.strip_rows(H, r, world, frame_dist.strip_for(mode))


def _decode_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, W = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc
        if typ == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype == 2
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, dtype=np.uint8).reshape(H, 1 + 3 * W)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(H, W, 3)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_png_roundtrip(rt, tmp_path, threads):
    rng = np.random.default_rng(threads)
    img = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    p = str(tmp_path / "x.png")
    rt.write_png(p, img, threads=threads)
    assert np.array_equal(_decode_png(p), img)


def test_to_rgb8_matches_toByte(rt):
    # toByte(v) = (int)std::round(clamp01(v) * 255): round half away from zero (core.h:313-316)
    v = np.array([-1.0, 0.0, 0.5 / 255, 1.5 / 255, 0.5, 127.5 / 255, 1.0, 1.2, np.nan, 0.999999, 2.5 / 255, 1e-300])
    v = np.pad(v, (0, (-len(v)) % 3)).reshape(-1, 1, 3)
    got = rt.to_rgb8(v).reshape(-1)
    flat = v.reshape(-1)
    clamped = np.where(flat < 1.0, flat, 1.0)   # std::min(1.0, v) maps NaN to 1
    clamped = np.where(0.0 < clamped, clamped, 0.0)
    want = np.floor(clamped * 255.0 + 0.5).astype(np.uint8)
    assert np.array_equal(got, want)


def test_mt19937_jump_polynomials_cpu():
    amd = C.CDLL(os.path.join(LIB, "librtamd.so"), mode=C.RTLD_GLOBAL)
    assert amd.rt_test_mt_jump_cpu(64, 2) == 0   # radix-64 tree: m*64^j*K blocks, j < 2
    assert amd.rt_test_mt_jump_cpu(3, 3) == 0   # non power-of-two segment length


def _compile_info(rt, text):
    amd = rt.amd_lib()
    amd.rt_test_compile_info.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
    sc = rt.load_scene_from_json_text(text)
    out = (C.c_int32 * 8)()
    assert amd.rt_test_compile_info(sc.handle, out) == 0
    keys = ("objects", "obj_groups", "obj_group_members", "ops", "ivl_groups", "ivl_group_members",
            "has_eager", "max_ivl_depth")
    return dict(zip(keys, out))


def test_compiled_cull_groups(rt):
    """Host compile of the device object table: object cull headers and CSG
    operand groups (scene_compile.cpp) appear where the bench scene needs
    them and never in scenes without CSG."""
    import scenes
    cfg4 = _compile_info(rt, scenes.config_json(4, dpi=8)[0])
    # 15 objects + 2 headers; the 20-sphere union gets operand groups
    assert cfg4["objects"] == 17 and cfg4["obj_groups"] == 2
    assert cfg4["ivl_groups"] >= 3 and cfg4["ivl_group_members"] >= 10
    tort = scenes.torture_scenes(dpi=8)
    g = _compile_info(rt, json.dumps(tort["csg_groups"]))
    assert g["ivl_groups"] >= 3
    assert _compile_info(rt, json.dumps(tort["rotation_scaling"]))["ivl_groups"] == 0
    assert _compile_info(rt, json.dumps(tort["xform_in_csg"]))["has_eager"] == 1


def test_cli_usage_and_load_errors(tmp_path):
    r = subprocess.run([RAY], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage:" in r.stderr and "--paper" in r.stderr
    r = subprocess.run([RAY, str(tmp_path / "missing.json"), str(tmp_path / "o.png")], capture_output=True, text=True)
    assert r.returncode == 3 and r.stderr.startswith("[error] Cannot open JSON file: ")
    bad = tmp_path / "bad.json"
    bad.write_text("{ invalid json }")
    r = subprocess.run([RAY, str(bad), str(tmp_path / "o.png")], capture_output=True, text=True)
    assert r.returncode == 3 and r.stderr.startswith("[error] JSON parse error: ")
    bad.write_text(json.dumps({"objects": [{"sphere": {"position": [0, 0, 0], "radius": 1, "color": [1, 0, 0]}}]}))
    r = subprocess.run([RAY, str(bad), str(tmp_path / "o.png")], capture_output=True, text=True)
    assert r.returncode == 3 and "JSON processing error: color must be an object" in r.stderr


def test_render_without_device_fails_loudly(rt):
    """On a host without a HIP device the product path errors out (no CPU fallback)."""
    amd = rt.amd_lib()
    if amd.rt_device_count() > 0:
        pytest.skip("a GPU is present")
    sc = rt.load_scene_from_json_text(json.dumps({"objects": []}))
    with pytest.raises(rt.RTError) as e:
        rt.Tracer(sc, 4, 4, 0).render()
    assert e.value.code == -7


def test_runtime_guard_refuses_two_runtimes(rt, monkeypatch):
    """rtamd.check_one_hip_runtime: a second HIP runtime (torch's bundled copy)
    or a foreign one bound instead of /opt/rocm's is refused."""
    rocm = rt.ROCM_DIR
    monkeypatch.setattr(rt, "mapped_libraries",
                        lambda stem: [rocm + "/lib/libamdhip64.so.7", "/x/torch/lib/libamdhip64.so"])
    with pytest.raises(RuntimeError, match="two HIP runtimes"):
        rt.check_one_hip_runtime()
    monkeypatch.setattr(rt, "mapped_libraries", lambda stem: ["/x/torch/lib/libamdhip64.so"])
    with pytest.raises(RuntimeError, match="not"):
        rt.check_one_hip_runtime()
    monkeypatch.setattr(rt, "mapped_libraries", lambda stem: [rocm + "/lib/libamdhip64.so.7"])
    assert rt.check_one_hip_runtime().startswith(rocm)


def test_paper_code_decoder_matches_reference_expression(rt):
    """Distributed paper-mode frames gather one code byte per pixel; the root
    decodes it (rtamd::paper_code_value) into the value tracer.cpp:258-281
    computes from the edge strength (tracer.cpp:133-178: the max of 0.9 /
    0.6 / 0.5 / 0.3 or 0, halved when a neighbour is outside the frame) and
    the hatch bit (tracer.cpp:188-205), bit for bit in FP64."""
    lib = rt.amd_lib()
    lib.rt_test_paper_code_value.restype = C.c_double
    lib.rt_test_paper_code_value.argtypes = [C.c_int]
    raw = [0.0, 0.3, 0.5, 0.6, 0.9]
    seen = set()
    for i, e0 in enumerate(raw):
        for half in (0, 1):
            for h in (0, 1):
                edge = e0 * 0.5 if half else e0
                if edge > 0.8:
                    want = 0.0
                elif edge > 0.5:
                    want = 0.2
                else:
                    want = 1.0 if h else 0.0
                    if edge > 0.3:
                        want *= (1.0 - (edge - 0.3) * 0.4)
                got = lib.rt_test_paper_code_value(i | (8 if half else 0) | (16 if h else 0))
                assert struct.pack("<d", got) == struct.pack("<d", want), (i, half, h, got, want)
                seen.add(got)
    assert {0.0, 0.2, 1.0} <= seen and len(seen) >= 5   # incl. the darkened whites of edges 0.45 / 0.6*0.5...


def test_paper_launch_order_permutes_whole_blocks(rt):
    """rt_render.hip order_paper_groups: a paper frame's primary list is
    relaunched in 16-entry blocks (one workgroup row), costliest first by the
    previous frame's measured 8-entry group costs (keyed by each group's first
    ext index), ties in list order, padding blocks last; any unmeasured group
    keeps the whole list in row order."""
    lib = rt.amd_lib()
    lib.rt_test_paper_order.argtypes = [C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_uint32), C.c_int]
    rng = np.random.default_rng(7)
    n_ext = 96
    # runs of consecutive ext rows padded to 8, the list padded to 16 (frame_trace)
    lst = []
    for a, b in [(0, 30), (30, 61), (61, 90), (90, 96)]:
        while len(lst) % 8:
            lst.append(-1)
        lst.extend(range(a, b))
    while len(lst) % 16:
        lst.append(-1)
    lst.extend([-1] * 16)   # an all-padding block
    cost = np.zeros(n_ext, dtype=np.uint32)
    groups = [lst[i:i + 8] for i in range(0, len(lst), 8)]
    for g in groups:
        e = next((v for v in g if v >= 0), -1)
        if e >= 0:
            cost[e] = rng.integers(1, 5)   # small values: ties happen

    def run(lst, cost):
        arr = (C.c_int32 * len(lst))(*lst)
        c = (C.c_uint32 * len(cost))(*[int(v) for v in cost])
        assert lib.rt_test_paper_order(arr, len(lst), c, len(cost)) == 0
        return list(arr)

    got = run(lst, cost)
    blocks = [lst[i:i + 16] for i in range(0, len(lst), 16)]

    def bcost(b):
        s = 0
        for g in (b[:8], b[8:]):
            e = next((v for v in g if v >= 0), -1)
            s += int(cost[e]) if e >= 0 else 0
        return s
    want = [v for b in sorted(blocks, key=lambda b: -bcost(b)) for v in b]   # (sorted is stable)
    assert got == want
    assert sorted(got) == sorted(lst) and got[-16:] == [-1] * 16
    # one unmeasured group: row order kept
    cost2 = cost.copy()
    cost2[next(v for v in lst if v >= 0)] = 0
    assert run(lst, cost2) == lst
    # bad arguments
    assert lib.rt_test_paper_order((C.c_int32 * 8)(), 8, (C.c_uint32 * 1)(), 1) != 0
