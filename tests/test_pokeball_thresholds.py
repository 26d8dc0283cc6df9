"""Pokeball::pick_region_material (raytracer/src/geometry.cpp:163-180)
compares ang = std::acos(clamp1(u . btnDir)) with btnOuter and with
inner = max(0, btnOuter - ringWidth).  The device never evaluates acos: it
compares x with two thresholds the host derives from its own acos (glibc,
the reference's), rtamd::pokeball_thresholds (scene_compile.hpp).  Here,
with Python's math.acos (the same glibc acos), the thresholds reproduce both
comparisons exactly: densely around each threshold, at the ends of [-1, 1],
and over random x - for the loader's defaults, the reference example scene's
values, this repo's scenes, and random parameters."""
import ctypes as C
import math
import random
import struct

import numpy as np
import pytest


def _thr(rt, b, w):
    out = (C.c_double * 2)()
    assert rt.amd_lib().rt_test_pokeball_thresholds(C.c_double(b), C.c_double(w), out) == 0
    return out[0], out[1]


def _step(x, k):
    """x moved by k ulps (ordered doubles)."""
    i = struct.unpack("<q", struct.pack("<d", x))[0]
    key = i if i >= 0 else -(i & 0x7FFFFFFFFFFFFFFF)
    key += k
    i2 = key if key >= 0 else ((-key) | -0x8000000000000000)
    return struct.unpack("<d", struct.pack("<q", i2))[0]


def _check(rt, b, w, rng, dense=3000, n_random=20000):
    xb, xi = _thr(rt, b, w)
    inner = max(0.0, b - w)
    xs = [-1.0, 1.0, 0.0, -0.0, math.cos(b), math.cos(inner)]
    for t in (xb, xi, math.cos(b), math.cos(inner)):
        if -1.0 <= t <= 1.0:
            xs += [_step(t, k) for k in range(-dense, dense + 1)]
    xs += [rng.uniform(-1.0, 1.0) for _ in range(n_random)]
    for x in xs:
        if not (-1.0 <= x <= 1.0):
            continue
        a = math.acos(x)
        assert (a <= b) == (x >= xb), (b, w, x, xb)
        assert (a >= inner) == (x <= xi), (b, w, x, xi)


PARAMS = [(0.28, 0.06), (0.25, 0.05), (0.35, 0.08), (0.3, 0.3), (0.3, 0.5), (0.0, 0.0), (math.pi, 0.1),
          (4.0, 0.1), (-0.1, 0.05), (1e-9, 1e-10), (math.pi / 2, 0.2)]


@pytest.mark.parametrize("b,w", PARAMS)
def test_thresholds_reproduce_glibc_acos_decisions(rt, b, w):
    _check(rt, b, w, random.Random(hash((b, w)) & 0xffff))


def test_thresholds_random_parameters(rt):
    rng = random.Random(7)
    for _ in range(40):
        b = rng.uniform(0.0, 3.2)
        w = rng.uniform(0.0, 1.0)
        _check(rt, b, w, rng, dense=300, n_random=2000)


def test_nan_parameters(rt):
    xb, xi = _thr(rt, float("nan"), 0.1)
    assert xb == 2.0   # acos(x) <= NaN never holds: no button / ring
    assert np.isfinite(xi)
