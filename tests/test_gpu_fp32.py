"""The optional FP32 fast path (RT_FLAG_FP32).

NON-PARITY by design: the survey measured that FP32 misses the 1e-5 bar on
0.155 % of snorlax pixels.  These tests pin what the flag does promise: the
same algorithm (ray counts within a small fraction of the FP64 path's), an
image that matches the CPU oracle closely everywhere but on a thin set of
silhouette / CSG-seam / shadow-edge pixels, and the same output contract
(shape, paper-mode value set).  The FP64 path stays the parity path
(tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from test_gpu_parity import SMALL

# fraction of framebuffer channels allowed to differ from the oracle by more
# than 1e-3 (silhouettes / seams flip between hit and miss in FP32).  Measured
# on MI355X: <= 0.33 % on every scene but reflect_refract (4.3 %: refraction
# at recursion 6 amplifies a flipped TIR decision down the ray tree).
FAR_FRAC = 0.01
FAR_FRAC_SECONDARY = 0.06
# mean |d| over the whole framebuffer
MEAN_TOL = 5e-3


def _render(rt, text, mode, flags):
    sc = rt.load_scene_from_json_text(text)
    st = rt.Stats()
    fb = rt.Tracer(sc, sc.width, sc.height, mode, flags=flags).render(st)
    return sc, fb, st


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SMALL))
@pytest.mark.parametrize("mode", [0, 1])
def test_fp32_close_to_oracle(gpu, name, mode):
    text = SMALL[name]()
    sc, fb, st = _render(gpu, text, mode, gpu.RT_FLAG_FP32)
    ref, ost = gpu.oracle_render(sc, sc.width, sc.height, mode, threads=8)
    d = np.abs(fb - ref)
    far = float(np.mean(d > 1e-3))
    n_ref = ost.rays_intersect + ost.rays_occluded
    n_gpu = st.rays_intersect + st.rays_occluded
    print(f"  {name} mode={mode} far={far:.5f} mean={d.mean():.2e} max={d.max():.3g} "
          f"within1e-5={float(np.mean(d <= 1e-5)):.4f} rays gpu={n_gpu} oracle={n_ref}")
    assert fb.shape == ref.shape and np.isfinite(fb).all()
    assert far <= (FAR_FRAC_SECONDARY if name == "reflect_refract" else FAR_FRAC)
    assert d.mean() <= MEAN_TOL
    assert abs(n_gpu - n_ref) <= 0.05 * n_ref + 16


@pytest.mark.gpu
def test_fp32_flag_changes_kernel_only(gpu):
    """FP32 and FP64 frames of the same scene agree to FP32 accuracy on
    ordinary pixels and the FP64 frame is unaffected by a preceding FP32 run
    (separate scene copies in the workspace)."""
    text = SMALL["cfg4"]()
    sc, a, _ = _render(gpu, text, 0, gpu.RT_FLAG_NONE)
    _, b, _ = _render(gpu, text, 0, gpu.RT_FLAG_FP32)
    _, c, _ = _render(gpu, text, 0, gpu.RT_FLAG_NONE)
    assert np.array_equal(a, c)
    assert float(np.median(np.abs(a - b))) <= 1e-5
