"""rtamd — ctypes bindings over the C-ABI in include/rt.h.

This is test/bench plumbing, not the product: the product is the C-ABI
(lib/librtamd.so, lib/librt_host.so) and the `ray` CLI.  The Python names
mirror the reference's interface for the hot path:

* ``load_scene_from_json_text`` / ``load_scene_from_json`` ->
  ``jsonio::load_scene_from_json_text`` / ``load_scene_from_json``
  (raytracer/src/json_loader.cpp:458-503)
* ``Tracer(scene, width, height, mode).render()`` -> ``Tracer::render``
  (raytracer/src/tracer.h:18-35, tracer.cpp:247-305)

The GPU path fails loudly (RuntimeError) when librtamd.so is missing or no HIP
device is present; there is no CPU fallback.  The CPU oracle (oracle/) and the
reference harness (oracle/_ref) are exposed separately for tests only.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
BIN_DIR = os.path.join(PKG_DIR, "bin")
ORACLE_DIR = os.path.join(REPO_DIR, "oracle")

RT_OK = 0
RT_MODE_STANDARD = 0
RT_MODE_PAPER = 1
RT_OK = 0
RT_ERR_INVALID_ARG = -1
RT_ERR_NO_DEVICE = -7
RT_FLAG_NONE = 0
RT_FLAG_COUNT_OPS = 1
RT_FLAG_NO_CULL = 2
RT_FLAG_FP32 = 4   # non-parity FP32 fast path
RT_FLAG_NO_BVH = 8   # wave culls without the wave BVH (A/B; identical results)
RT_FLAG_FORCE_BVH = 16   # the wave BVH on every frame (no on/off trial frames)

NODE_SPHERE, NODE_HALFSPACE, NODE_POKEBALL, NODE_TRANSLATION, NODE_SCALING, NODE_ROTATION, NODE_CSG = range(7)
CSG_UNION, CSG_INTERSECTION, CSG_DIFFERENCE = range(3)

OP_NAMES = [
    "sphere_isect", "sphere_isect_hit", "sphere_ivl", "sphere_ivl_hit", "half_isect", "half_isect_hit",
    "half_ivl", "poke_region", "csg_combine", "xform", "shade_light", "shade_spec", "secondary", "culled",
    "light_eval", "shade_call",
]


class Material(C.Structure):
    _fields_ = [("albedo", C.c_double * 3), ("ambient", C.c_double * 3), ("kd", C.c_double), ("ks", C.c_double),
                ("kr", C.c_double), ("kt", C.c_double), ("shininess", C.c_double),
                ("refractive_index", C.c_double)]


class Node(C.Structure):
    _fields_ = [("kind", C.c_int32), ("a", C.c_int32), ("b", C.c_int32), ("op", C.c_int32), ("mat", C.c_int32),
                ("mats", C.c_int32 * 5), ("v", C.c_double * 24), ("aux", C.c_double * 4)]


class Light(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("intensity", C.c_double * 3)]


class DirLight(C.Structure):
    _fields_ = [("dir", C.c_double * 3), ("radiance", C.c_double * 3)]


class Camera(C.Structure):
    _fields_ = [("eye", C.c_double * 3), ("P", C.c_double * 3), ("Lx", C.c_double), ("Ly", C.c_double),
                ("dpi", C.c_int32), ("pad_", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("camera", Camera), ("background", C.c_double * 3), ("ambient", C.c_double * 3),
                ("medium_index", C.c_double), ("recursion_limit", C.c_int32), ("n_lights", C.c_int32),
                ("lights", C.POINTER(Light)), ("n_materials", C.c_int32), ("n_nodes", C.c_int32),
                ("materials", C.POINTER(Material)), ("nodes", C.POINTER(Node)), ("n_objects", C.c_int32),
                ("pad_", C.c_int32), ("objects", C.POINTER(C.c_int32)), ("n_dir_lights", C.c_int32),
                ("pad2_", C.c_int32), ("dir_lights", C.POINTER(DirLight))]


class Stats(C.Structure):
    _fields_ = [("rays_intersect", C.c_uint64), ("rays_occluded", C.c_uint64), ("rays_traced", C.c_uint64),
                ("pixels", C.c_uint64), ("ms_rng", C.c_double), ("ms_kernel", C.c_double),
                ("ms_total", C.c_double), ("ops", C.c_uint64 * 16),
                ("ms_gather", C.c_double), ("ms_tobyte", C.c_double), ("ms_d2h", C.c_double),
                ("n_gpus", C.c_int32), ("pad_", C.c_int32)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "ops"}
        d["ops"] = {OP_NAMES[i]: int(self.ops[i]) for i in range(16)}
        return d


class OracleStats(C.Structure):
    _fields_ = [("rays_intersect", C.c_uint64), ("rays_occluded", C.c_uint64), ("ops", C.c_uint64 * 16)]


class OracleHit(C.Structure):
    _fields_ = [("t", C.c_double), ("p", C.c_double * 3), ("n", C.c_double * 3), ("mat", C.c_int32),
                ("front_face", C.c_int32)]

    def as_tuple(self):
        return (self.t, tuple(self.p), tuple(self.n), self.mat, self.front_face)


_dp = C.POINTER(C.c_double)


def _load(path: str, mode=C.RTLD_GLOBAL):
    if not os.path.exists(path):
        raise RuntimeError(f"required library not built: {path} (run __graft_entry__.build())")
    return C.CDLL(path, mode=mode)


_host = None
_amd = None
_oracle = None
_ref = None


def host_lib():
    global _host
    if _host is None:
        lib = _load(os.path.join(LIB_DIR, "librt_host.so"))
        lib.rt_last_error.restype = C.c_char_p
        lib.rt_scene_load_json_text.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p)]
        lib.rt_scene_load_json_file.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        lib.rt_scene_from_desc.argtypes = [C.POINTER(SceneDesc), C.POINTER(C.c_void_p)]
        lib.rt_scene_get_desc.argtypes = [C.c_void_p]
        lib.rt_scene_get_desc.restype = C.POINTER(SceneDesc)
        lib.rt_scene_destroy.argtypes = [C.c_void_p]
        lib.rt_camera_width.argtypes = [C.POINTER(Camera)]
        lib.rt_camera_height.argtypes = [C.POINTER(Camera)]
        lib.rt_framebuffer_to_rgb8.argtypes = [_dp, C.c_size_t, C.POINTER(C.c_uint8)]
        lib.rt_write_png.argtypes = [C.c_char_p, C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_int]
        _host = lib
    return _host


def amd_lib():
    """The HIP renderer.  Raises if the extension is missing (no fallback)."""
    global _amd
    if _amd is None:
        host_lib()
        # RTAMD_LIB: diagnostic override (tools/ build experiments); never a fallback
        lib = _load(os.environ.get("RTAMD_LIB") or os.path.join(LIB_DIR, "librtamd.so"))
        lib.rt_render.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, C.POINTER(Stats)]
        lib.rt_render_rows_device.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                              C.POINTER(C.c_int32), C.c_int, C.c_void_p, C.c_void_p,
                                              C.POINTER(Stats)]
        lib.rt_scatter_rows_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        if hasattr(lib, "rt_frame_begin"):   # (absent only in RTAMD_LIB builds of older sources)
            lib.rt_frame_begin.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int32),
                                           C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
            lib.rt_frame_trace.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
            lib.rt_frame_end.argtypes = [C.c_void_p, C.POINTER(Stats)]
        lib.rt_framebuffer_to_rgb8_device.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
        lib.rt_device_count.restype = C.c_int
        lib.rt_render_multi.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp,
                                        C.POINTER(Stats)]
        lib.rt_render_rgb8.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_uint8), C.POINTER(Stats)]
        lib.rt_dist_get_id.argtypes = [C.POINTER(C.c_uint8)]
        lib.rt_dist_create.argtypes = [C.POINTER(C.c_uint8), C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        lib.rt_dist_destroy.argtypes = [C.c_void_p]
        lib.rt_dist_destroy.restype = None
        lib.rt_render_dist.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                       C.c_void_p, C.POINTER(Stats)]
        lib.rt_render_dist_rgb8.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.POINTER(Stats)]
        lib.rt_dist_rows.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int32)]
        lib.rt_dist_rows_mode.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int32)]
        lib.rt_test_render_dist_sim.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                _dp, C.POINTER(C.c_uint8)]
        lib.rt_test_dist_threads.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, _dp,
                                             C.POINTER(C.c_uint8)]
        lib.rt_dist_reduce_max.argtypes = [C.c_void_p, _dp, C.c_int]
        lib.rt_dist_barrier.argtypes = [C.c_void_p]
        lib.rt_dist_frame_split.argtypes = [C.c_void_p, _dp, C.c_int]
        lib.rt_set_device.argtypes = [C.c_int]
        lib.rt_device_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
        lib.rt_device_free.argtypes = [C.c_void_p]
        lib.rt_memcpy_h2d.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        lib.rt_memcpy_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        lib.rt_stream_create.argtypes = [C.POINTER(C.c_void_p)]
        lib.rt_stream_destroy.argtypes = [C.c_void_p]
        lib.rt_test_dist_create_rccl1.argtypes = [C.POINTER(C.c_void_p)]
        check_one_hip_runtime()
        _amd = lib
    return _amd


def mapped_libraries(stem: str) -> list[str]:
    """Real paths of the shared objects whose file name starts with `stem`
    mapped into this process (/proc/self/maps)."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6:
                    path = parts[5].strip()
                    if os.path.basename(path).startswith(stem):
                        out.add(os.path.realpath(path))
    except OSError:
        return []
    return sorted(out)


ROCM_DIR = os.path.realpath(os.environ.get("ROCM_PATH", "/opt/rocm"))


def check_one_hip_runtime() -> str:
    """librtamd.so must run on ONE HIP runtime, the one `ray` and the
    INTEGRATION binding use: /opt/rocm's.  A process that imported torch
    first has torch's bundled runtime (same soname) already mapped, and
    librtamd.so binds to it; loading torch afterwards maps a second runtime
    (two runtimes torn down at exit aborted the process).  Raises in both
    cases; a single runtime outside ROCM_PATH only warns.  Returns the
    runtime's path."""
    hips = mapped_libraries("libamdhip64.so")
    if len(hips) > 1:
        raise RuntimeError("two HIP runtimes mapped in this process: " + ", ".join(hips) +
                           " (do not import torch in a process that uses librtamd.so)")
    if hips and os.sep + "torch" + os.sep in hips[0]:
        raise RuntimeError(f"librtamd.so is bound to torch's bundled HIP runtime {hips[0]} "
                           "(import torch after, or not at all in, a process that uses librtamd.so)")
    if hips and not hips[0].startswith(ROCM_DIR + os.sep):
        # one runtime, not a torch wheel's: another ROCm install (/opt/rocm-X.Y without the
        # /opt/rocm link, a distro package) is legitimate
        import warnings

        warnings.warn(f"librtamd.so runs on the HIP runtime {hips[0]}, outside ROCM_PATH={ROCM_DIR}")
    return hips[0] if hips else ""


def oracle_lib():
    """CPU oracle (TEST INFRASTRUCTURE ONLY)."""
    global _oracle
    if _oracle is None:
        lib = _load(os.path.join(ORACLE_DIR, "liboracle.so"), mode=C.RTLD_LOCAL)
        lib.oracle_render_rows.argtypes = [C.POINTER(SceneDesc), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp,
                                           C.POINTER(OracleStats), C.c_int]
        lib.oracle_node_intersect.argtypes = [C.POINTER(SceneDesc), C.c_int, _dp, _dp, C.c_double, C.c_double,
                                              C.POINTER(OracleHit)]
        lib.oracle_node_interval.argtypes = [C.POINTER(SceneDesc), C.c_int, _dp, _dp, _dp, _dp,
                                             C.POINTER(OracleHit), C.POINTER(OracleHit)]
        lib.oracle_scene_intersect.argtypes = [C.POINTER(SceneDesc), _dp, _dp, C.c_double, C.c_double,
                                               C.POINTER(OracleHit)]
        lib.oracle_scene_occluded.argtypes = [C.POINTER(SceneDesc), _dp, _dp, C.c_double, C.c_double]
        lib.oracle_camera_ray.argtypes = [C.POINTER(SceneDesc), C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                          _dp, _dp]
        lib.oracle_jitter.argtypes = [C.c_uint64, C.c_uint64, _dp]
        lib.oracle_mt_words.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32)]
        _oracle = lib
    return _oracle


def ref_lib():
    """The reference's own sources compiled by oracle/Makefile (container only)."""
    global _ref
    if _ref is None:
        lib = _load(os.path.join(ORACLE_DIR, "_ref", "libref.so"), mode=C.RTLD_LOCAL)
        lib.ref_render.argtypes = [C.POINTER(SceneDesc), C.c_int, C.c_int, C.c_int, _dp, C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64)]
        lib.ref_node_intersect_batch.argtypes = [C.POINTER(SceneDesc), C.c_int, C.c_int, _dp, _dp, C.c_double,
                                                 C.c_double, C.POINTER(C.c_int), C.POINTER(OracleHit)]
        lib.ref_node_interval_batch.argtypes = [C.POINTER(SceneDesc), C.c_int, C.c_int, _dp, _dp,
                                                C.POINTER(C.c_int), _dp, _dp, C.POINTER(OracleHit),
                                                C.POINTER(OracleHit)]
        lib.ref_camera_ray.argtypes = [C.POINTER(SceneDesc), C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                       _dp, _dp]
        lib.ref_jitter.argtypes = [C.c_uint64, C.c_uint64, _dp]
        lib.ref_mt_words.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32)]
        if hasattr(lib, "ref_roundtrip"):
            lib.ref_roundtrip.argtypes = [C.POINTER(SceneDesc), C.POINTER(C.c_void_p)]
        _ref = lib
    return _ref


class RTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def last_error() -> str:
    return host_lib().rt_last_error().decode("utf-8", "replace")


class Scene:
    """Owned rt_scene handle (scene IR)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @property
    def handle(self):
        return self._h

    @property
    def desc(self) -> SceneDesc:
        return host_lib().rt_scene_get_desc(self._h).contents

    @property
    def desc_ptr(self):
        return host_lib().rt_scene_get_desc(self._h)

    @property
    def width(self) -> int:
        return host_lib().rt_camera_width(C.byref(self.desc.camera))

    @property
    def height(self) -> int:
        return host_lib().rt_camera_height(C.byref(self.desc.camera))

    def close(self):
        if self._h and self._h.value:
            host_lib().rt_scene_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_scene_from_json_text(text: str) -> Scene:
    """jsonio::load_scene_from_json_text (json_loader.cpp:458); raises RTError."""
    raw = text.encode("utf-8")
    out = C.c_void_p()
    rc = host_lib().rt_scene_load_json_text(raw, len(raw), C.byref(out))
    if rc != RT_OK:
        raise RTError(rc, last_error())
    return Scene(out.value)


def load_scene_from_json(path: str) -> Scene:
    """jsonio::load_scene_from_json (json_loader.cpp:499)."""
    out = C.c_void_p()
    rc = host_lib().rt_scene_load_json_file(path.encode(), C.byref(out))
    if rc != RT_OK:
        raise RTError(rc, last_error())
    return Scene(out.value)


def scene_from_desc(desc: SceneDesc) -> Scene:
    out = C.c_void_p()
    rc = host_lib().rt_scene_from_desc(C.byref(desc), C.byref(out))
    if rc != RT_OK:
        raise RTError(rc, last_error())
    return Scene(out.value)


def with_dir_lights(scene: Scene, lights) -> Scene:
    """Copy of `scene` with directional lights [(dir, radiance), ...]: the
    reference's Scene::dir_lights (scene.h:10-15, 36), which its JSON loader
    never fills; reachable here through rt_scene_from_desc as there through
    the Scene API."""
    d = SceneDesc.from_buffer_copy(scene.desc)   # arrays are deep-copied by rt_scene_from_desc
    arr = (DirLight * max(1, len(lights)))()
    for i, (dv, rad) in enumerate(lights):
        arr[i].dir[:] = [float(v) for v in dv]
        arr[i].radiance[:] = [float(v) for v in rad]
    d.n_dir_lights = len(lights)
    d.dir_lights = C.cast(arr, C.POINTER(DirLight))
    return scene_from_desc(d)


def device_count() -> int:
    return int(amd_lib().rt_device_count())


def _ok(rc: int, what: str):
    if rc != RT_OK:
        raise RTError(rc, f"{what}: {last_error()}")


def set_device(dev: int):
    _ok(amd_lib().rt_set_device(dev), "rt_set_device")


def device_synchronize():
    _ok(amd_lib().rt_device_synchronize(), "rt_device_synchronize")


class DeviceBuffer:
    """A device allocation made by librtamd.so itself (rt_device_alloc): the
    tests and bench need no second HIP runtime (torch) for their buffers."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _ok(amd_lib().rt_device_alloc(self.nbytes, C.byref(p)), "rt_device_alloc")
        self.ptr = p

    def to_host(self, dtype=np.float64, shape=None) -> np.ndarray:
        out = np.empty(self.nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        _ok(amd_lib().rt_memcpy_d2h(out.ctypes.data_as(C.c_void_p), self.ptr, out.nbytes), "rt_memcpy_d2h")
        return out.reshape(shape) if shape is not None else out

    def from_host(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _ok(amd_lib().rt_memcpy_h2d(self.ptr, arr.ctypes.data_as(C.c_void_p), arr.nbytes), "rt_memcpy_h2d")

    def free(self):
        if self.ptr is not None and self.ptr.value:
            amd_lib().rt_device_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    """A non-blocking HIP stream made by librtamd.so (rt_stream_create)."""

    def __init__(self):
        p = C.c_void_p()
        _ok(amd_lib().rt_stream_create(C.byref(p)), "rt_stream_create")
        self.handle = p

    def destroy(self):
        if self.handle is not None and self.handle.value:
            amd_lib().rt_stream_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def shutdown():
    """rt_shutdown: release every device resource the library caches."""
    _ok(amd_lib().rt_shutdown(), "rt_shutdown")


@dataclass
class Tracer:
    """Mirror of the reference's Tracer (tracer.h:18-35) over the GPU C-ABI."""
    scene: Scene
    width: int
    height: int
    mode: int = RT_MODE_STANDARD
    flags: int = RT_FLAG_NONE

    def render(self, stats: Stats | None = None) -> np.ndarray:
        lib = amd_lib()
        fb = np.zeros((self.height, self.width, 3), dtype=np.float64)
        st = stats if stats is not None else Stats()
        rc = lib.rt_render(self.scene.handle, self.width, self.height, self.mode, self.flags,
                           fb.ctypes.data_as(_dp), C.byref(st))
        if rc != RT_OK:
            raise RTError(rc, last_error())
        return fb


def render_multi(scene: Scene, width: int, height: int, mode: int, n_gpus: int, flags: int = RT_FLAG_NONE,
                 stats: Stats | None = None) -> np.ndarray:
    """rt_render_multi: the frame over n_gpus devices of this process."""
    fb = np.zeros((height, width, 3), dtype=np.float64)
    st = stats if stats is not None else Stats()
    rc = amd_lib().rt_render_multi(scene.handle, width, height, mode, flags, n_gpus, fb.ctypes.data_as(_dp),
                                   C.byref(st))
    if rc != RT_OK:
        raise RTError(rc, last_error())
    return fb


def render_rgb8(scene: Scene, width: int, height: int, mode: int, n_gpus: int = 1, flags: int = RT_FLAG_NONE,
                stats: Stats | None = None) -> np.ndarray:
    """rt_render_rgb8: render + toByte on the device(s), RGB bytes."""
    out = np.zeros((height, width, 3), dtype=np.uint8)
    st = stats if stats is not None else Stats()
    rc = amd_lib().rt_render_rgb8(scene.handle, width, height, mode, flags, n_gpus,
                                  out.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(st))
    if rc != RT_OK:
        raise RTError(rc, last_error())
    return out


def dist_rows(H: int, world: int, rank: int, mode: int = RT_MODE_STANDARD) -> list[int]:
    """rt_dist_rows_mode: the output rows rank renders (interleaved strips of
    RT_STRIP_ROWS, paper mode RT_PAPER_STRIP_ROWS)."""
    buf = (C.c_int32 * max(1, H))()
    n = amd_lib().rt_dist_rows_mode(H, world, rank, mode, buf)
    if n < 0:
        raise RTError(n, "rt_dist_rows: bad arguments")
    return list(buf[:n])


class DistRun(C.Structure):
    """rt_test.h rt_test_dist_run."""
    _fields_ = [("world", C.c_int), ("rgb8", C.c_int), ("frames", C.c_int), ("fault_rank", C.c_int),
                ("fault", C.c_int), ("fault_frame", C.c_int), ("timeout_ms", C.c_int), ("msg_cap", C.c_int),
                ("rc", C.POINTER(C.c_int)), ("ms", _dp), ("msgs", C.c_char_p),
                ("frame_scenes", C.POINTER(C.c_void_p)), ("alt_scene", C.c_void_p), ("split", _dp)]


(FAULT_NONE, FAULT_TRACE, FAULT_SETUP, FAULT_DESC_H, FAULT_DESC_FLAGS, FAULT_ABSENT, FAULT_DESC_SCENE,
 FAULT_DESC_SHED) = range(8)
RANK_ABSENT = 1


def dist_threads(scene: Scene, width: int, height: int, mode: int, world: int, frames: int = 1,
                 fault: int = FAULT_NONE, fault_rank: int = -1, fault_frame: int = 0, timeout_ms: int = 0,
                 rgb8: bool = False, flags: int = RT_FLAG_NONE, frame_scenes=None, alt_scene=None,
                 split_out: np.ndarray | None = None):
    """rt_test_dist_threads: `frames` distributed frames with `world` ranks
    running concurrently on the current device (one host thread, stream set
    and workspace per rank; RCCL replaced by a same-device transport), with an
    optional fault on one rank in one frame.  frame_scenes: one Scene (or
    None = `scene`) per frame, rendered in sequence on the same ranks;
    alt_scene: the scene FAULT_DESC_SCENE gives the faulty rank; split_out:
    float64 [frames, world, 10], filled with each rank's rt_dist_frame_split
    after each successful frame.  Returns (root frames
    [frames, H, W, 3] - zeros where the root's call failed -, rc [frames,
    world], ms [frames, world], messages [frames][world])."""
    lib = amd_lib()
    cap = 512
    rc = np.zeros((frames, world), dtype=np.int32)
    ms = np.zeros((frames, world), dtype=np.float64)
    msgs = C.create_string_buffer(frames * world * cap)
    out = np.zeros((frames, height, width, 3), dtype=np.uint8 if rgb8 else np.float64)
    run = DistRun(world, 1 if rgb8 else 0, frames, fault_rank, fault, fault_frame, timeout_ms, cap,
                  rc.ctypes.data_as(C.POINTER(C.c_int)), ms.ctypes.data_as(_dp), C.cast(msgs, C.c_char_p))
    keep = []
    if frame_scenes is not None:
        assert len(frame_scenes) == frames
        arr = (C.c_void_p * frames)(*[(x.handle.value if x is not None else None) for x in frame_scenes])
        keep.append(arr)
        run.frame_scenes = C.cast(arr, C.POINTER(C.c_void_p))
    if alt_scene is not None:
        run.alt_scene = alt_scene.handle.value
    if split_out is not None:
        assert split_out.shape == (frames, world, 10) and split_out.dtype == np.float64 and split_out.flags.c_contiguous
        run.split = split_out.ctypes.data_as(_dp)
    if rgb8:
        r = lib.rt_test_dist_threads(scene.handle, width, height, mode, flags, C.byref(run), None,
                                     out.ctypes.data_as(C.POINTER(C.c_uint8)))
    else:
        r = lib.rt_test_dist_threads(scene.handle, width, height, mode, flags, C.byref(run),
                                     out.ctypes.data_as(_dp), None)
    if r != RT_OK:
        raise RTError(r, last_error())
    raw = msgs.raw
    text = [[raw[(f * world + k) * cap:(f * world + k + 1) * cap].split(b"\0", 1)[0].decode("utf-8", "replace")
             for k in range(world)] for f in range(frames)]
    return out, rc, ms, text


def render_dist_sim(scene: Scene, width: int, height: int, mode: int, world: int, rgb8: bool = False,
                    flags: int = RT_FLAG_NONE) -> np.ndarray:
    """rt_test_render_dist_sim: one distributed frame with `world` ranks
    running concurrently on the current device (rt_test_dist_threads)."""
    lib = amd_lib()
    if rgb8:
        out = np.zeros((height, width, 3), dtype=np.uint8)
        rc = lib.rt_test_render_dist_sim(scene.handle, width, height, mode, flags, world, 1, None,
                                         out.ctypes.data_as(C.POINTER(C.c_uint8)))
    else:
        out = np.zeros((height, width, 3), dtype=np.float64)
        rc = lib.rt_test_render_dist_sim(scene.handle, width, height, mode, flags, world, 0, out.ctypes.data_as(_dp),
                                         None)
    if rc != RT_OK:
        raise RTError(rc, last_error())
    return out


def oracle_render(scene: Scene, width: int, height: int, mode: int, row0: int = 0, row1: int | None = None,
                  threads: int = 1):
    """CPU oracle restricted to output rows [row0,row1).  TEST ONLY."""
    if row1 is None:
        row1 = height
    fb = np.zeros((row1 - row0, width, 3), dtype=np.float64)
    st = OracleStats()
    rc = oracle_lib().oracle_render_rows(scene.desc_ptr, width, height, mode, row0, row1, fb.ctypes.data_as(_dp),
                                         C.byref(st), threads)
    if rc != 0:
        raise RuntimeError("oracle_render_rows failed")
    return fb, st


def ref_render(scene: Scene, width: int, height: int, mode: int):
    """The reference's own Tracer::render (oracle/_ref, container only)."""
    fb = np.zeros((height, width, 3), dtype=np.float64)
    ni, no = C.c_uint64(), C.c_uint64()
    ref_lib().ref_render(scene.desc_ptr, width, height, mode, fb.ctypes.data_as(_dp), C.byref(ni), C.byref(no))
    return fb, int(ni.value), int(no.value)


def to_rgb8(fb: np.ndarray) -> np.ndarray:
    fb = np.ascontiguousarray(fb, dtype=np.float64)
    out = np.zeros(fb.shape, dtype=np.uint8)
    host_lib().rt_framebuffer_to_rgb8(fb.ctypes.data_as(_dp), fb.size // 3, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def write_png(path: str, rgb8: np.ndarray, threads: int = 1) -> None:
    rgb8 = np.ascontiguousarray(rgb8, dtype=np.uint8)
    h, w = rgb8.shape[:2]
    rc = host_lib().rt_write_png(path.encode(), rgb8.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, threads)
    if rc != RT_OK:
        raise RTError(rc, f"rt_write_png failed ({rc})")
