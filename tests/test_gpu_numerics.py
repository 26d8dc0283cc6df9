"""Device arithmetic helpers that must round exactly like the plain FP64
operations they replace.

div3 (rt_device.hpp) divides three numerators by one denominator with the
compiler's own v_div_scale / v_rcp / Newton / v_div_fmas / v_div_fixup
sequence, doing the reciprocal refinement once; it replaces every
normalisation (Dir3::normalized, core.h:95-101), the light direction
tl / dist (shading.cpp:81-83) and the sphere normal (p - c) / r
(geometry.cpp:30, 67-77).  It must equal `/` bit for bit on every input,
including zeros of both signs, denormals, infinities, NaN and the exponent
extremes where the scaled denominator depends on the numerator."""
import ctypes as C

import numpy as np
import pytest


def _run(rt, a, b):
    lib = rt.amd_lib()
    dp = C.POINTER(C.c_double)
    lib.rt_test_div3.argtypes = [dp, dp, C.c_int, dp, dp]
    n = len(b)
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(n, 3)
    b = np.ascontiguousarray(b, dtype=np.float64)
    o3 = np.zeros((n, 3))
    op = np.zeros((n, 3))
    rc = lib.rt_test_div3(a.ctypes.data_as(dp), b.ctypes.data_as(dp), n, o3.ctypes.data_as(dp), op.ctypes.data_as(dp))
    assert rc == 0
    return o3, op


@pytest.mark.gpu
def test_div3_bit_identical_to_division(gpu):
    rng = np.random.default_rng(11)
    n = 1 << 20
    # geometry-like values: unit-ish vectors, distances, radii
    a = rng.normal(size=(n, 3)) * np.exp(rng.uniform(-20, 20, size=(n, 1)))
    b = np.abs(rng.normal(size=n)) * np.exp(rng.uniform(-20, 20, size=n)) + 1e-12
    o3, op = _run(gpu, a, b)
    assert np.array_equal(o3.view(np.uint64), op.view(np.uint64))


@pytest.mark.gpu
def test_div3_edge_values(gpu):
    specials = np.array([0.0, -0.0, 5e-324, -5e-324, 2.2250738585072014e-308, 1e-300, 1e-310, 1.0, -1.0,
                         1e300, 1.7976931348623157e308, np.inf, -np.inf, np.nan, 3.0, 1e-17, 2.0 ** -969,
                         2.0 ** -970, 2.0 ** 1023], dtype=np.float64)
    rng = np.random.default_rng(5)
    n = 64 * 2048
    a = rng.choice(specials, size=(n, 3))
    b = rng.choice(specials, size=n)
    # one wave in four gets ordinary values mixed with extremes in the same wave
    a[::4] = rng.normal(size=(len(a[::4]), 3))
    o3, op = _run(gpu, a, b)
    assert np.array_equal(o3.view(np.uint64), op.view(np.uint64))
