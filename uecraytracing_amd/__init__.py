"""uecraytracing_amd — MI355X (gfx950) renderer for the per-pixel sampling loop of
yaito3014/UECRayTracing.

The product is the C-ABI library ``uecraytracing_amd/lib/libykgpu.so`` (include/ykgpu.h) and the
drop-in CLI ``uecraytracing_amd/lib/raytrace``.  This module is a thin ctypes view of that
library for tests and the benchmark: it has NO fallback — if the library or a GPU is missing,
every render raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import records
from .records import Camera, RenderParams, RenderStats, Sphere, make_params, sphere_array

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libykgpu.so")
# tools/ablate.py loads timing-only variants through this override; tests never set it
LIB_PATH = os.environ.get("YKGPU_LIB_OVERRIDE", LIB_PATH)
CLI_PATH = os.path.join(LIB_DIR, "raytrace")

EXPORTS = (
    "ykgpu_abi_version", "ykgpu_last_error", "ykgpu_device_count", "ykgpu_context_create",
    "ykgpu_context_destroy", "ykgpu_set_scene", "ykgpu_render", "ykgpu_render_async",
    "ykgpu_render_sums", "ykgpu_render_trace", "ykgpu_get_stats", "ykgpu_math_sqrt", "ykgpu_math_sqrt_f32", "ykgpu_math_div", "ykgpu_math_div_f32", "yk_camera_reference", "yk_camera_look",
    "yk_scene_build", "yk_scene_write", "yk_scene_read", "yk_image_height_for",
    "ykgpu_group_create", "ykgpu_group_destroy", "ykgpu_group_size", "ykgpu_group_set_scene",
    "ykgpu_group_render", "ykgpu_group_get_stats", "ykgpu_render_devices",
)
ABI_VERSION = 11
SCENE_DIR = os.path.join(PKG_DIR, "scenes")  # committed scene files of the BASELINE configs

_lib = None


class YkError(RuntimeError):
    pass


def load_library():
    """Loads libykgpu.so (built by __graft_entry__.build / `make -C uecraytracing_amd/csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise YkError(f"{LIB_PATH} is missing: build it with `make -C uecraytracing_amd/csrc` "
                      "(there is no CPU fallback)")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64/libhsa-runtime64
    # (soname libamdhip64.so.7, like /opt/rocm's).  If torch is importable it is loaded FIRST
    # so that libykgpu.so binds to the already-loaded runtime instead of pulling in a second
    # copy, which would leave whichever initialises second without a GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    P, c = ctypes.POINTER, ctypes
    sig = {
        "ykgpu_abi_version": ([], c.c_uint32),
        "ykgpu_last_error": ([], c.c_char_p),
        "ykgpu_device_count": ([P(c.c_int)], c.c_int),
        "ykgpu_context_create": ([c.c_int, P(c.c_void_p)], c.c_int),
        "ykgpu_context_destroy": ([c.c_void_p], c.c_int),
        "ykgpu_set_scene": ([c.c_void_p, P(Sphere), c.c_uint32, P(Camera)], c.c_int),
        "ykgpu_render": ([c.c_void_p, P(RenderParams), c.c_void_p], c.c_int),
        "ykgpu_render_async": ([c.c_void_p, P(RenderParams), c.c_void_p, c.c_void_p], c.c_int),
        "ykgpu_render_sums": ([c.c_void_p, P(RenderParams), c.c_void_p], c.c_int),
        "ykgpu_render_trace": ([c.c_void_p, P(RenderParams), c.c_uint32, c.c_void_p, c.c_void_p], c.c_int),
        "ykgpu_get_stats": ([c.c_void_p, P(RenderStats)], c.c_int),
        "ykgpu_math_sqrt": ([c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint64], c.c_int),
        "ykgpu_math_sqrt_f32": ([c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint64], c.c_int),
        "ykgpu_math_div": ([c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint64], c.c_int),
        "ykgpu_math_div_f32": ([c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint64], c.c_int),
        "yk_camera_reference": ([P(Camera)], c.c_int),
        "yk_camera_look": ([P(Camera), P(c.c_double), P(c.c_double), P(c.c_double), c.c_double,
                            c.c_double, c.c_double, c.c_double], c.c_int),
        "yk_scene_build": ([c.c_char_p, c.c_uint32, P(Sphere), c.c_uint32, P(c.c_uint32),
                            P(Camera)], c.c_int),
        "yk_scene_write": ([c.c_char_p, P(Sphere), c.c_uint32, P(Camera)], c.c_int),
        "yk_scene_read": ([c.c_char_p, P(Sphere), c.c_uint32, P(c.c_uint32), P(Camera)], c.c_int),
        "yk_image_height_for": ([c.c_uint32], c.c_uint32),
        "ykgpu_group_create": ([P(c.c_int), c.c_uint32, P(c.c_void_p)], c.c_int),
        "ykgpu_group_destroy": ([c.c_void_p], c.c_int),
        "ykgpu_group_size": ([c.c_void_p, P(c.c_uint32)], c.c_int),
        "ykgpu_group_set_scene": ([c.c_void_p, P(Sphere), c.c_uint32, P(Camera)], c.c_int),
        "ykgpu_group_render": ([c.c_void_p, P(RenderParams), c.c_void_p], c.c_int),
        "ykgpu_group_get_stats": ([c.c_void_p, c.c_int, P(RenderStats)], c.c_int),
        "ykgpu_render_devices": ([P(c.c_int), c.c_uint32, P(Sphere), c.c_uint32, P(Camera),
                                  P(RenderParams), c.c_void_p], c.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes, f.restype = args, res
    if lib.ykgpu_abi_version() != ABI_VERSION:
        raise YkError("ABI version mismatch")
    _lib = lib
    return lib


def _check(rc):
    if rc != 0:
        msg = load_library().ykgpu_last_error().decode(errors="replace")
        raise YkError(f"{records.ERRORS.get(rc, rc)}: {msg}")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = load_library().ykgpu_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def reference_camera() -> Camera:
    cam = Camera()
    _check(load_library().yk_camera_reference(ctypes.byref(cam)))
    return cam


def build_scene(name: str, seed: int = 0):
    """Named scenes of include/ykgpu.h (host only).  Returns (spheres ctypes array, Camera)."""
    lib = load_library()
    n, cam = ctypes.c_uint32(0), Camera()
    _check(lib.yk_scene_build(name.encode(), seed, None, 0, ctypes.byref(n), ctypes.byref(cam)))
    arr = (Sphere * n.value)()
    _check(lib.yk_scene_build(name.encode(), seed, arr, n.value, ctypes.byref(n), None))
    return arr, cam


def write_scene(path: str, spheres, camera: Camera):
    """Scene file (include/ykgpu.h yk_scene_write): tuple order, exact doubles."""
    arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
    _check(load_library().yk_scene_write(os.fsencode(path), arr, len(arr), ctypes.byref(camera)))


def read_scene(path: str):
    """Returns (spheres ctypes array, Camera) from a scene file."""
    lib = load_library()
    n, cam = ctypes.c_uint32(0), Camera()
    _check(lib.yk_scene_read(os.fsencode(path), None, 0, ctypes.byref(n), ctypes.byref(cam)))
    arr = (Sphere * n.value)()
    _check(lib.yk_scene_read(os.fsencode(path), arr, n.value, ctypes.byref(n), None))
    return arr, cam


class Renderer:
    """One device context (ykgpu_context): owns the scene in HBM, scratch and a stream."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        self._ctx = ctypes.c_void_p()
        _check(self._lib.ykgpu_context_create(device, ctypes.byref(self._ctx)))
        self.device = device

    def close(self):
        if self._ctx:
            self._lib.ykgpu_context_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_scene(self, spheres, camera: Camera):
        arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
        _check(self._lib.ykgpu_set_scene(self._ctx, arr, len(arr), ctypes.byref(camera)))

    def render(self, params: RenderParams) -> np.ndarray:
        """Host RGB8 image of the tile: uint8[row_count, W, 3] (image_t layout)."""
        out = np.empty((params.row_count, params.tile_width(), 3), np.uint8)
        _check(self._lib.ykgpu_render(self._ctx, ctypes.byref(params), out.ctypes.data))
        return out

    def render_sums(self, params: RenderParams) -> np.ndarray:
        out = np.empty((params.row_count, params.tile_width(), 3), np.float64)
        _check(self._lib.ykgpu_render_sums(self._ctx, ctypes.byref(params), out.ctypes.data))
        return out

    def render_trace(self, params: RenderParams, max_rays: int):
        """ray_color's rays (verbose level 3, raytracer.hpp:21-25) of every sample of the tile:
        (rays float64[row_count, W, spp, max_rays, 6], counts uint32[row_count, W, spp])."""
        shape = (params.row_count, params.tile_width(), params.samples_per_pixel)
        rays = np.zeros(shape + (max_rays, 6), np.float64)
        counts = np.zeros(shape, np.uint32)
        _check(self._lib.ykgpu_render_trace(self._ctx, ctypes.byref(params), max_rays, rays.ctypes.data,
                                            counts.ctypes.data))
        return rays, counts

    def render_async(self, params: RenderParams, rgb_device_ptr: int, stream_ptr: int = 0):
        """Enqueue into device memory (e.g. a torch.uint8 CUDA tensor's data_ptr())."""
        _check(self._lib.ykgpu_render_async(self._ctx, ctypes.byref(params),
                                            ctypes.c_void_p(rgb_device_ptr),
                                            ctypes.c_void_p(stream_ptr or None)))

    def math_sqrt(self, values) -> np.ndarray:
        """The device's math::sqrt (math.hpp:10-19) on a float64 array (diagnostic)."""
        a = np.ascontiguousarray(values, dtype=np.float64)
        out = np.empty_like(a)
        _check(self._lib.ykgpu_math_sqrt(self._ctx, a.ctypes.data, out.ctypes.data, a.size))
        return out

    def math_sqrt_f32(self, values) -> np.ndarray:
        """The FP32 path's math::sqrt<float> on a float32 array (diagnostic)."""
        a = np.ascontiguousarray(values, dtype=np.float32)
        out = np.empty_like(a)
        _check(self._lib.ykgpu_math_sqrt_f32(self._ctx, a.ctypes.data, out.ctypes.data, a.size))
        return out

    def math_div(self, num3, den) -> np.ndarray:
        """The renderer's vector / scalar division: num3[i, k] / den[i] (diagnostic)."""
        a = np.ascontiguousarray(num3, dtype=np.float64).reshape(-1, 3)
        b = np.ascontiguousarray(den, dtype=np.float64).reshape(-1)
        assert a.shape[0] == b.shape[0]
        out = np.empty_like(a)
        _check(self._lib.ykgpu_math_div(self._ctx, a.ctypes.data, b.ctypes.data, out.ctypes.data, b.size))
        return out

    def math_div_f32(self, num3, den) -> np.ndarray:
        """The FP32 path's vector / scalar division: num3[i, k] / den[i] in float (diagnostic)."""
        a = np.ascontiguousarray(num3, dtype=np.float32).reshape(-1, 3)
        b = np.ascontiguousarray(den, dtype=np.float32).reshape(-1)
        assert a.shape[0] == b.shape[0]
        out = np.empty_like(a)
        _check(self._lib.ykgpu_math_div_f32(self._ctx, a.ctypes.data, b.ctypes.data, out.ctypes.data, b.size))
        return out

    def stats(self) -> dict:
        st = RenderStats()
        _check(self._lib.ykgpu_get_stats(self._ctx, ctypes.byref(st)))
        return st.as_dict()


class Group:
    """Several device contexts in one process (ykgpu_group): rows dealt cyclically over the
    entries, every tile copied into its rows of one host image (include/ykgpu.h)."""

    def __init__(self, devices):
        self._lib = load_library()
        self._g = ctypes.c_void_p()
        devs = (ctypes.c_int * len(devices))(*devices)
        _check(self._lib.ykgpu_group_create(devs, len(devices), ctypes.byref(self._g)))
        self.devices = list(devices)

    def close(self):
        if self._g:
            self._lib.ykgpu_group_destroy(self._g)
            self._g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def size(self) -> int:
        n = ctypes.c_uint32(0)
        _check(self._lib.ykgpu_group_size(self._g, ctypes.byref(n)))
        return n.value

    def set_scene(self, spheres, camera: Camera):
        arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
        _check(self._lib.ykgpu_group_set_scene(self._g, arr, len(arr), ctypes.byref(camera)))

    def render(self, params: RenderParams) -> np.ndarray:
        out = np.empty((params.row_count, params.tile_width(), 3), np.uint8)
        _check(self._lib.ykgpu_group_render(self._g, ctypes.byref(params), out.ctypes.data))
        return out

    def stats(self, index: int = -1) -> dict:
        st = RenderStats()
        _check(self._lib.ykgpu_group_get_stats(self._g, index, ctypes.byref(st)))
        return st.as_dict()


def render_devices(devices, spheres, camera: Camera, params: RenderParams) -> np.ndarray:
    """ykgpu_render_devices: group, scene, render and release in one call."""
    lib = load_library()
    arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
    devs = (ctypes.c_int * len(devices))(*devices)
    out = np.empty((params.row_count, params.tile_width(), 3), np.uint8)
    _check(lib.ykgpu_render_devices(devs, len(devices), arr, len(arr), ctypes.byref(camera),
                                    ctypes.byref(params), out.ctypes.data))
    return out


__all__ = ["Renderer", "Group", "render_devices", "YkError", "build_scene", "write_scene", "read_scene", "SCENE_DIR", "reference_camera", "device_count",
           "make_params", "load_library", "records", "EXPORTS", "LIB_PATH", "CLI_PATH"]
