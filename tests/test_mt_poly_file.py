"""The precomputed mt19937 checkpoint-tree jump polynomials (build output
lib/mt19937_tree.polys, read by the jitter generator instead of computing
them on a process's first frame) equal the polynomials computed from the
characteristic polynomial, and a damaged file is refused (the generator then
computes them).  Host only: no GPU."""
import ctypes as C
import os
import shutil

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POLYS = os.path.join(REPO, "raytracing-project_amd", "lib", "mt19937_tree.polys")


@pytest.fixture(scope="module")
def lib(rt):
    L = rt.amd_lib()
    L.rt_test_mt_poly_file.argtypes = [C.c_char_p, C.c_int]
    return L


def test_poly_file_matches_computed(lib):
    assert os.path.exists(POLYS), "build() writes lib/mt19937_tree.polys"
    # levels 1-2 cover every frame up to 4096 segments (8K); level 3+ are
    # the same recurrence, checked on the GPU by the jitter-stream tests
    assert lib.rt_test_mt_poly_file(POLYS.encode(), 2) == 0


def test_poly_file_damaged_or_short_is_refused(lib, tmp_path):
    bad = tmp_path / "bad.polys"
    shutil.copy(POLYS, bad)
    with open(bad, "r+b") as f:
        f.seek(24 + 4 * 1000)
        b = f.read(1)
        f.seek(24 + 4 * 1000)
        f.write(bytes([b[0] ^ 1]))
    assert lib.rt_test_mt_poly_file(str(bad).encode(), 1) == 2       # checksum
    assert lib.rt_test_mt_poly_file(POLYS.encode(), 9) == 2            # more levels than stored
    assert lib.rt_test_mt_poly_file(str(tmp_path / "none").encode(), 1) == 2
