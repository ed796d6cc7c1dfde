"""ctypes binding to the CPU oracle (oracle/_build/libykoracle.so).  TEST INFRASTRUCTURE ONLY —
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product package."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from uecraytracing_amd.records import Camera, RenderParams, Sphere, sphere_array

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "libykoracle.so")
REF_HARNESS = os.path.join(ORACLE_DIR, "_ref", "ref_harness")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "_build/libykoracle.so"], check=True)
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    lib.yko_render.argtypes = [P(Sphere), ctypes.c_uint32, P(Camera), P(RenderParams),
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                               P(ctypes.c_uint64), P(ctypes.c_uint64)]
    lib.yko_render.restype = ctypes.c_int
    lib.yko_render_as_shipped.argtypes = lib.yko_render.argtypes
    lib.yko_render_as_shipped.restype = ctypes.c_int
    lib.yko_sample.argtypes = [P(Sphere), ctypes.c_uint32, P(Camera), P(RenderParams),
                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                               P(ctypes.c_double), P(ctypes.c_uint64)]
    lib.yko_sample.restype = ctypes.c_int
    lib.yko_mt19937.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_uint32)]
    lib.yko_mt19937.restype = None
    lib.yko_canonical_pattern.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_double)]
    lib.yko_canonical_pattern.restype = None
    lib.yko_newton_sqrt.argtypes = [ctypes.c_double]
    lib.yko_newton_sqrt.restype = ctypes.c_double
    lib.yko_newton_sqrt_n.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.yko_newton_sqrt_n.restype = None
    lib.yko_canonical_pattern_f32.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib.yko_canonical_pattern_f32.restype = None
    lib.yko_newton_sqrt_f32_n.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.yko_newton_sqrt_f32_n.restype = None
    lib.yko_xor128.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_uint32)]
    lib.yko_xor128.restype = None
    lib.yko_canonical_pattern_x128.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_double)]
    lib.yko_canonical_pattern_x128.restype = None
    lib.yko_seed_from_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    lib.yko_seed_from_key.restype = ctypes.c_uint32
    _lib = lib
    return lib


def render(spheres, camera: Camera, params: RenderParams, nthreads=None, want_rgb=True,
           want_sums=False):
    """Returns (rgb uint8[rows, W, 3] | None, sums float64[rows, W, 3] | None, segments, tests)."""
    lib = load()
    arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
    rows, W = params.row_count, params.tile_width()
    rgb = np.zeros((rows, W, 3), np.uint8) if want_rgb else None
    sums = np.zeros((rows, W, 3), np.float64) if want_sums else None
    segs, tests = ctypes.c_uint64(0), ctypes.c_uint64(0)
    nt = nthreads or max(1, min(os.cpu_count() or 1, 8))
    st = lib.yko_render(arr, len(arr), ctypes.byref(camera), ctypes.byref(params),
                        rgb.ctypes.data if rgb is not None else None,
                        sums.ctypes.data if sums is not None else None, nt,
                        ctypes.byref(segs), ctypes.byref(tests))
    if st != 0:
        raise RuntimeError(f"oracle render failed: {st}")
    return rgb, sums, segs.value, tests.value


def render_as_shipped(spheres, camera: Camera, params: RenderParams, nthreads=None):
    """The reference's as-shipped cost model (per-sample random_device seeding): timing only,
    the image is not reproducible.  Returns segments."""
    lib = load()
    arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
    rgb = np.zeros((params.row_count, params.tile_width(), 3), np.uint8)
    segs, tests = ctypes.c_uint64(0), ctypes.c_uint64(0)
    nt = nthreads or max(1, min(os.cpu_count() or 1, 8))
    st = lib.yko_render_as_shipped(arr, len(arr), ctypes.byref(camera), ctypes.byref(params),
                                   rgb.ctypes.data, None, nt, ctypes.byref(segs), ctypes.byref(tests))
    if st != 0:
        raise RuntimeError(f"oracle render failed: {st}")
    return segs.value


def sample(spheres, camera, params, y, x, s):
    lib = load()
    arr = spheres if isinstance(spheres, ctypes.Array) else sphere_array(spheres)
    out = (ctypes.c_double * 3)()
    draws = ctypes.c_uint64(0)
    st = lib.yko_sample(arr, len(arr), ctypes.byref(camera), ctypes.byref(params), y, x, s, out,
                        ctypes.byref(draws))
    if st != 0:
        raise RuntimeError(f"oracle sample failed: {st}")
    return tuple(out), draws.value


def mt19937(seed, count):
    out = (ctypes.c_uint32 * count)()
    load().yko_mt19937(seed, count, out)
    return list(out)


def xor128(seed, count):
    """yk::xor128 (random.hpp:18-41) outputs."""
    out = (ctypes.c_uint32 * count)()
    load().yko_xor128(seed, count, out)
    return list(out)


def canonical_pattern_x128(seed, count):
    out = (ctypes.c_double * count)()
    load().yko_canonical_pattern_x128(seed, count, out)
    return list(out)


def canonical_pattern(seed, count):
    out = (ctypes.c_double * count)()
    load().yko_canonical_pattern(seed, count, out)
    return list(out)


def newton_sqrt(x):
    return load().yko_newton_sqrt(x)


def newton_sqrt_array(values):
    import numpy as np
    a = np.ascontiguousarray(values, dtype=np.float64)
    out = np.empty_like(a)
    load().yko_newton_sqrt_n(a.ctypes.data, out.ctypes.data, a.size)
    return out


def canonical_pattern_f32(seed, count):
    """The KAT pattern with uniform_real_distribution<float> (render<float>)."""
    out = np.empty(count, np.float32)
    load().yko_canonical_pattern_f32(seed, count, out.ctypes.data)
    return out


def newton_sqrt_f32(values):
    """math::sqrt<float> (math.hpp:10-19 with T = float) over an array."""
    a = np.ascontiguousarray(values, dtype=np.float32)
    out = np.empty_like(a)
    load().yko_newton_sqrt_f32_n(a.ctypes.data, out.ctypes.data, a.size)
    return out


def seed_from_key(key, idx):
    """Per-sample seed of YK_SEED_RANDOM_DEVICE (include/ykgpu.h)."""
    return load().yko_seed_from_key(key, idx)
