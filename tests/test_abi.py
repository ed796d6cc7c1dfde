"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every entry point
include/ykgpu.h declares, its host-side scene helpers reproduce the reference's scene values,
and the product has no CPU fallback (rendering without a GPU fails loudly)."""
import ctypes
import os
import re

import pytest

import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd import records

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "ykgpu.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(yk\w+)\s*\(", text, re.M)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert set(names) == set(yk.EXPORTS), names


def test_library_exports_every_declared_symbol():
    lib = yk.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.ykgpu_abi_version() == yk.ABI_VERSION == 11


def test_library_carries_no_diagnostic_entry_points():
    """The per-wave drain stamps (-DYK_DRAIN_DIAG, tools/drain_probe.py) are a diagnostic build's:
    the product library exports none of their accessors and holds no stamp buffer."""
    lib = yk.load_library()
    for name in ("ykgpu_diag_wave_times", "ykgpu_diag_wave_times_clear"):
        assert not hasattr(lib, name), name
    blob = open(yk.LIB_PATH, "rb").read()
    assert b"yk_wave_times" not in blob


def test_reference_camera_matches_camera_hpp():
    assert yk.reference_camera().as_tuple() == refscenes.reference_camera().as_tuple()


@pytest.mark.parametrize("name", sorted(refscenes.SCENES))
def test_scene_builder_matches_reference_values(name):
    arr, cam = yk.build_scene(name)
    want = refscenes.SCENES[name]()
    assert [s.as_tuple() for s in arr] == [s.as_tuple() for s in want]
    assert cam.as_tuple() == refscenes.reference_camera().as_tuple()


def test_extension_scenes_are_deterministic():
    a, ca = yk.build_scene("final", 42)
    b, cb = yk.build_scene("final", 42)
    c, _ = yk.build_scene("final", 43)
    assert 400 < len(a) < 490
    assert [s.as_tuple() for s in a] == [s.as_tuple() for s in b]
    assert [s.as_tuple() for s in a] != [s.as_tuple() for s in c]
    assert ca.lens_radius == 0.05 and ca.as_tuple() == cb.as_tuple()
    kinds = {s.material for s in a}
    assert kinds == {records.MATERIAL_LAMBERTIAN, records.MATERIAL_METAL, records.MATERIAL_DIELECTRIC}
    g, _ = yk.build_scene("glass", 42)
    frac = sum(s.material == records.MATERIAL_DIELECTRIC for s in g) / len(g)
    assert frac > 0.4


def test_unknown_scene_is_an_error():
    with pytest.raises(yk.YkError):
        yk.build_scene("nope")


def test_image_height_matches_source_cpp():
    lib = yk.load_library()
    for w in (16, 200, 400, 800, 1920, 3840):
        assert lib.yk_image_height_for(w) == records.image_height_for(w)
    assert records.image_height_for(200) == 112 and records.image_height_for(1920) == 1080


def test_no_cpu_fallback_without_a_gpu():
    if yk.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(yk.YkError):
        yk.Renderer(0)


def test_group_without_a_gpu_fails_loudly():
    if yk.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(yk.YkError, match="group entry 0"):
        yk.Group([0, 0])
    arr, cam = yk.build_scene("ref4")
    with pytest.raises(yk.YkError):
        yk.render_devices([0], arr, cam, records.make_params(16, 9, 2))


def test_group_invalid_arguments_are_reported():
    lib = yk.load_library()
    g = ctypes.c_void_p()
    assert lib.ykgpu_group_create(None, 0, ctypes.byref(g)) == 1
    assert b"empty device list" in lib.ykgpu_last_error()
    devs = (ctypes.c_int * 1)(0)
    assert lib.ykgpu_group_create(devs, 1, None) == 1
    assert lib.ykgpu_group_render(None, None, None) == 1
    assert lib.ykgpu_group_set_scene(None, None, 0, None) == 1
    assert lib.ykgpu_group_get_stats(None, -1, None) == 1
    n = ctypes.c_uint32(0)
    assert lib.ykgpu_group_size(None, ctypes.byref(n)) == 1


def test_render_params_layout_matches_the_header():
    """yk_render_params (include/ykgpu.h, ABI 10): the column set after row_band_log2, 88 bytes."""
    P = records.RenderParams
    assert P.t_min.offset == 48 and P.seed_key.offset == 56 and P.row_band_log2.offset == 64
    assert (P.col_begin.offset, P.col_count.offset, P.col_stride.offset, P.col_band_log2.offset,
            P.reserved0.offset) == (68, 72, 76, 80, 84)
    assert ctypes.sizeof(P) == 88
    p = records.make_params(1920, cols=(8, 240, 8, 3))
    assert (p.col_begin, p.col_count, p.col_stride, p.col_band_log2) == (8, 240, 8, 3)
    assert p.tile_width() == 240 and records.make_params(1920).tile_width() == 1920


def test_render_stats_layout_matches_the_header():
    """yk_render_stats ends with device_bytes at offset 312, call_bytes at 320, sclk_mhz at 328 and
    (ABI 11) launch_spp, mem_shrinks at 336, 340 (include/ykgpu.h)."""
    assert records.RenderStats.device_bytes.offset == 312
    assert records.RenderStats.call_bytes.offset == 320
    assert records.RenderStats.sclk_mhz.offset == 328
    assert (records.RenderStats.launch_spp.offset, records.RenderStats.mem_shrinks.offset) == (336, 340)
    assert ctypes.sizeof(records.RenderStats) == 344


def test_invalid_arguments_are_reported():
    lib = yk.load_library()
    assert lib.ykgpu_context_create(0, None) == 1
    assert b"null" in lib.ykgpu_last_error()
    assert lib.ykgpu_set_scene(None, None, 0, None) == 1


def test_fastdiv_magic_numbers_divide_exactly():
    """The kernels divide 31-bit slot and pixel indices by runtime-invariant divisors with the
    host's magic numbers (ykgpu_render.hip fastdiv / fdiv): q = (n * m) >> sh, sh = 31 + ceil(log2 d),
    m = ceil(2^sh / d).  Restated here and checked against integer division on every divisor kind
    the renderer meets (image widths, padded pixel counts) and random ones, at the numerator's
    extremes and at random numerators."""
    import random

    def magic(d):
        l = 0
        while (1 << l) < d:
            l += 1
        sh = 31 + l
        m = ((1 << sh) + d - 1) // d
        assert m < (1 << 32)
        return m, sh

    rng = random.Random(3)
    divisors = [1, 2, 3, 7, 16, 200, 400, 800, 1920, 3840, 2073600, 2078720, 8294400, (1 << 31) - 1, 1 << 30]
    divisors += [rng.randrange(1, 1 << 31) for _ in range(2000)] + [rng.randrange(1, 1 << 12) for _ in range(2000)]
    for d in divisors:
        m, sh = magic(d)
        ns = [0, 1, d - 1, d, d + 1, (1 << 31) - 1, (1 << 31) - 2] + [rng.randrange(0, 1 << 31) for _ in range(200)]
        for n in ns:
            if 0 <= n < (1 << 31):
                assert (n * m) >> sh == n // d, (n, d)
