"""ctypes mirrors of the plain-C records in include/ykgpu.h (no compute here).

These are the data that cross the C-ABI: the world tuple flattened to ``yk_sphere`` records
(hittable_list.hpp:18-30, sphere.hpp:16-23, material.hpp:37-69), the public members of
``camera<T>`` (camera.hpp:34-37) and the compile-time constants of ``source.cpp:57-66``.
"""
from __future__ import annotations

import ctypes

MATERIAL_LAMBERTIAN = 0
MATERIAL_METAL = 1
MATERIAL_DIELECTRIC = 2

PRECISION_FP64 = 0
PRECISION_FP32 = 1  # render<float> (include/ykgpu.h)
RNG_MT19937 = 0
RNG_XOR128 = 1  # yk::xor128 (random.hpp:18-41), the fast mode (include/ykgpu.h)
SEED_COUNTER = 0
SEED_RANDOM_DEVICE = 1
FLAG_COUNT_WORK = 1
FLAG_LINEAR_SCAN = 2
FLAG_ONE_LANE = 4

YK_OK = 0
ERRORS = {
    1: "YK_ERR_INVALID",
    2: "YK_ERR_DEVICE",
    3: "YK_ERR_NOMEM",
    4: "YK_ERR_UNSUPPORTED",
    5: "YK_ERR_NO_SCENE",
}

T_MIN = 0.001  # raytracer.hpp:27
SEED0_EPOCH0 = 404  # sum of the chars of __TIME__ == "00:00:00" (source.cpp:118-120)

D3 = ctypes.c_double * 3


class Sphere(ctypes.Structure):
    _fields_ = [
        ("center", D3),
        ("radius", ctypes.c_double),
        ("albedo", D3),
        ("fuzz", ctypes.c_double),
        ("ior", ctypes.c_double),
        ("material", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]

    def as_tuple(self):
        return (tuple(self.center), self.radius, tuple(self.albedo), self.fuzz, self.ior,
                self.material)


class Camera(ctypes.Structure):
    _fields_ = [
        ("origin", D3),
        ("lower_left_corner", D3),
        ("horizontal", D3),
        ("vertical", D3),
        ("lens_u", D3),
        ("lens_v", D3),
        ("lens_radius", ctypes.c_double),
    ]

    def as_tuple(self):
        return tuple(tuple(getattr(self, f)) for f, _ in self._fields_[:-1]) + (self.lens_radius,)


class RenderParams(ctypes.Structure):
    _fields_ = [
        ("image_width", ctypes.c_uint32),
        ("image_height", ctypes.c_uint32),
        ("samples_per_pixel", ctypes.c_uint32),
        ("max_depth", ctypes.c_uint32),
        ("seed0", ctypes.c_uint32),
        ("row_begin", ctypes.c_uint32),
        ("row_count", ctypes.c_uint32),
        ("row_stride", ctypes.c_uint32),
        ("precision", ctypes.c_uint32),
        ("rng", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("seed_mode", ctypes.c_uint32),
        ("t_min", ctypes.c_double),
        ("seed_key", ctypes.c_uint64),
        ("row_band_log2", ctypes.c_uint32),  # bands of 2^k rows (include/ykgpu.h)
        ("col_begin", ctypes.c_uint32),  # column set (ABI 10); col_count == 0: every column
        ("col_count", ctypes.c_uint32),
        ("col_stride", ctypes.c_uint32),
        ("col_band_log2", ctypes.c_uint32),
        ("reserved0", ctypes.c_uint32),
    ]

    def tile_width(self) -> int:
        return self.col_count or self.image_width


class RenderStats(ctypes.Structure):
    _fields_ = [
        ("kernel_ms", ctypes.c_double),
        ("resolve_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("warmup_ms", ctypes.c_double),
        ("samples", ctypes.c_uint64),
        ("segments", ctypes.c_uint64),
        ("sphere_tests", ctypes.c_uint64),
        ("sqrt_calls", ctypes.c_uint64),
        ("mt_fallbacks", ctypes.c_uint64),
        ("node_visits", ctypes.c_uint64),
        ("linear_scans", ctypes.c_uint64),
        ("newton_calls", ctypes.c_uint64),
        ("newton_iters", ctypes.c_uint64),
        ("phase_cycles", ctypes.c_uint64 * 8),
        ("timeline", ctypes.c_uint64 * 3),
        ("diag", ctypes.c_uint64 * 4),
        ("seed_key", ctypes.c_uint64),
        ("launches", ctypes.c_uint32),
        ("grid_blocks", ctypes.c_uint32),
        ("render_busy_ms", ctypes.c_double),
        ("work", ctypes.c_uint64 * 8),
        ("device_bytes", ctypes.c_uint64),
        ("call_bytes", ctypes.c_uint64),
        ("sclk_mhz", ctypes.c_double),
        ("launch_spp", ctypes.c_uint32),  # ABI 11
        ("mem_shrinks", ctypes.c_uint32),
    ]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["phase_cycles"] = list(self.phase_cycles)
        d["timeline"] = list(self.timeline)
        d["diag"] = list(self.diag)
        d["work"] = list(self.work)
        return d


assert ctypes.sizeof(Sphere) == 80
assert ctypes.sizeof(Camera) == 19 * 8
assert ctypes.sizeof(RenderParams) == 88
assert ctypes.sizeof(RenderStats) == 344


def image_height_for(width: int) -> int:
    """uint32(W / (16.0/9.0)), source.cpp:59-62."""
    return int(width / (16.0 / 9.0))


def make_params(width, height=None, spp=8, max_depth=50, seed0=SEED0_EPOCH0, rows=None,
                flags=0, t_min=T_MIN, precision=PRECISION_FP64, seed_mode=SEED_COUNTER,
                seed_key=0, rng=RNG_MT19937, cols=None) -> RenderParams:
    """rows = (row_begin, row_count, row_stride[, row_band_log2]); default: the whole image.
    cols = (col_begin, col_count, col_stride[, col_band_log2]); default: every column."""
    if height is None:
        height = image_height_for(width)
    rb, rc, rs, band = (tuple(rows) + (0,))[:4] if rows is not None else (0, height, 1, 0)
    cb, cc, cs, cband = (tuple(cols) + (0,))[:4] if cols is not None else (0, 0, 0, 0)
    return RenderParams(width, height, spp, max_depth, seed0 & 0xFFFFFFFF, rb, rc, rs,
                        precision, rng, flags, seed_mode, t_min, seed_key, band, cb, cc, cs, cband, 0)


def sphere_array(spheres) -> ctypes.Array:
    arr = (Sphere * len(spheres))()
    for i, s in enumerate(spheres):
        arr[i] = s
    return arr


def lambertian(center, radius, albedo) -> Sphere:
    return Sphere(D3(*center), radius, D3(*albedo), 0.0, 0.0, MATERIAL_LAMBERTIAN, 0)


def metal(center, radius, albedo, fuzz=0.0) -> Sphere:
    return Sphere(D3(*center), radius, D3(*albedo), fuzz, 0.0, MATERIAL_METAL, 0)


def dielectric(center, radius, ior) -> Sphere:
    return Sphere(D3(*center), radius, D3(1.0, 1.0, 1.0), 0.0, ior, MATERIAL_DIELECTRIC, 0)
