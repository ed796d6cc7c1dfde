"""Parity of the HIP path (through the C-ABI) with the reference and the oracle — on the MI355X.

Bit-exact throughout: RGB8 bytes AND the per-pixel float64 sums before to_color3b.
  * reference-generated goldens (tests/golden, from /root/reference via oracle/_ref)
  * extension scenes (dielectric / fuzz / thin lens: parity unpinned vs the reference) against
    the oracle restatement
  * row and column tiles (the multi-GPU partitions), repeated calls, async into device memory
  * the headline configuration's geometry at full size on a strided row subset
"""
import numpy as np
import pytest

import golden_data
import oracle_lib
import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import (PRECISION_FP32, PRECISION_FP64, RNG_MT19937, RNG_XOR128,
                                       make_params)

pytestmark = pytest.mark.gpu
MAN = golden_data.manifest()


@pytest.fixture(scope="module")
def ren():
    r = yk.Renderer(0)
    yield r
    r.close()


@pytest.mark.parametrize("entry", MAN["cases"], ids=[c["name"] for c in MAN["cases"]])
def test_golden_case(ren, entry):
    sph, cam = golden_data.scene(entry)  # scene files: configs 2-5 content (gen_golden.py CASES_FILE)
    ren.set_scene(sph, cam)
    # fp32 fixtures: the reference's render<float> (YK_PRECISION_FP32); xor128 fixtures: the
    # reference's yk::xor128 as the per-sample engine (YK_RNG_XOR128)
    p = make_params(entry["W"], entry["H"], entry["spp"], entry["depth"], entry["seed0"],
                    precision=PRECISION_FP32 if entry.get("precision") == "fp32" else PRECISION_FP64,
                    rng=RNG_XOR128 if entry.get("rng") == "xor128" else RNG_MT19937)
    rgb = ren.render(p)
    np.testing.assert_array_equal(rgb, golden_data.rgb(entry))
    sums = ren.render_sums(p)
    assert golden_data.sha(sums) == entry["sums_sha256"]


def test_constexpr_build(ren):
    ren.set_scene(refscenes.ref4(), refscenes.reference_camera())
    rgb = ren.render(make_params(16, 9, 2, 50, 404))
    assert golden_data.sha(rgb) == MAN["constexpr_build"]["rgb_sha256"]


def sqrt_inputs(rng, n_random=1 << 22):
    """Doubles around every binade boundary (2^k +- m ulp) and at random exponents, all >= 0 and
    finite (the reference's loop never ends otherwise), plus zero and the smallest subnormals."""
    k = np.arange(-1074, 1024)
    base = np.ldexp(1.0, k).view(np.int64)
    m = np.arange(64)
    near = np.concatenate([(base[:, None] + m).ravel(), (base[:, None] - m).ravel()]).view(np.float64)
    near = near[np.isfinite(near) & (near >= 0)]
    wide = np.ldexp(1.0 + rng.random(n_random), rng.integers(-1022, 1023, n_random))
    unit = rng.random(n_random) * 4.0
    kat = np.array([float.fromhex(a) for a, _ in golden_data.kat()["newton_sqrt"]])
    return np.concatenate([[0.0, 5e-324, 1e-323, 2.2250738585072014e-308], near, wide, unit, kat])


def test_math_sqrt_matches_reference_loop(ren):
    """The device's math::sqrt starts at the IEEE sqrt (unique fixed point); it
    must equal the reference's loop from s/2 bit for bit."""
    x = sqrt_inputs(np.random.default_rng(11))
    got = ren.math_sqrt(x)
    want = oracle_lib.newton_sqrt_array(x)
    bad = np.flatnonzero(got.view(np.int64) != want.view(np.int64))
    assert bad.size == 0, [(x[i], got[i], want[i]) for i in bad[:5]]
    kat = golden_data.kat()["newton_sqrt"]
    got = ren.math_sqrt([float.fromhex(a) for a, _ in kat])
    assert [g.hex() for g in got] == [float.fromhex(b).hex() for _, b in kat]


def test_fast_division_is_ieee_division(ren):
    """The renderer's vector / scalar division skips div_scale / div_fixup for operands in
    [2^-400, 2^400] (yk_device.hpp); it must be IEEE division bit for bit everywhere: random
    operands of every sign and exponent, both sides of the range edges, zeros of both signs,
    subnormals and infinities (those take the full-division fallback)."""
    rng = np.random.default_rng(3)
    n = 1 << 21

    def draw(size, lo, hi):
        v = np.ldexp(1.0 + rng.random(size), rng.integers(lo, hi, size))
        return np.where(rng.random(size) < 0.5, -v, v)

    num = draw((n, 3), -420, 420)
    den = draw(n, -420, 420)
    num[: n // 8] = draw((n // 8, 3), -4, 4)          # the renderer's magnitudes
    den[: n // 8] = draw(n // 8, -2, 4)
    lo, hi = np.ldexp(1.0, -400), np.ldexp(1.0, 400)
    edges = np.array([lo, hi, np.nextafter(lo, 0), np.nextafter(hi, np.inf)])
    k = np.arange(4096)
    num[n // 8:n // 8 + 4096] = edges[k % 4, None] * np.array([1.0, -1.0, 3.0])
    den[n // 8:n // 8 + 4096] = edges[(k // 4) % 4] * np.where(k % 3 == 0, -1.0, 1.0)
    special = np.array([0.0, -0.0, 5e-324, -5e-324, np.inf, -np.inf, 1.0, -2.5])
    m = n // 4
    num[m:m + 512] = special[rng.integers(0, 8, (512, 3))]
    den[m:m + 512] = special[rng.integers(4, 8, 512)]
    got = ren.math_div(num, den)
    with np.errstate(all="ignore"):
        want = num / den[:, None]
    same = (got.view(np.int64) == want.view(np.int64)) | (np.isnan(got) & np.isnan(want))
    bad = np.argwhere(~same)
    assert bad.size == 0, [(num[i, j], den[i], got[i, j], want[i, j]) for i, j in bad[:5]]


@pytest.mark.gpu
def test_fast_float_division_is_ieee_division(ren):
    """The FP32 path's vector / scalar division skips div_scale / div_fmas / div_fixup for
    operands in [2^-40, 2^40] and shares the refined reciprocal (yk_device_f32.hpp); it must be
    IEEE float division bit for bit: every significand of the divisor in [1, 2) against random
    numerators, random operands of every sign and exponent, both sides of the range edges, zeros,
    subnormals and infinities (those take the full-division fallback)."""
    rng = np.random.default_rng(5)
    f = np.float32

    def draw(size, lo, hi):
        v = np.ldexp(1.0 + rng.random(size), rng.integers(lo, hi, size)).astype(f)
        return np.where(rng.random(size) < 0.5, -v, v).astype(f)

    # every float divisor in [1, 2) (2^23 significands), numerators in the renderer's magnitudes
    sig = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(0x3F800000)).view(f)
    num = draw((sig.size, 3), -3, 3)
    den = sig.copy()
    extra = 1 << 20
    num2 = draw((extra, 3), -60, 60)
    den2 = draw(extra, -60, 60)
    lo, hi = f(2.0 ** -40), f(2.0 ** 40)
    edges = np.array([lo, hi, np.nextafter(lo, f(0)), np.nextafter(hi, f(np.inf))], dtype=f)
    k = np.arange(4096)
    num2[:4096] = edges[k % 4, None] * np.array([1.0, -1.0, 3.0], dtype=f)
    den2[:4096] = edges[(k // 4) % 4] * np.where(k % 3 == 0, f(-1.0), f(1.0))
    special = np.array([0.0, -0.0, 1e-45, -1e-45, np.inf, -np.inf, 1.0, -2.5], dtype=f)
    num2[8192:8192 + 512] = special[rng.integers(0, 8, (512, 3))]
    den2[8192:8192 + 512] = special[rng.integers(4, 8, 512)]
    num = np.concatenate([num, num2]).astype(f)
    den = np.concatenate([den, den2]).astype(f)
    got = ren.math_div_f32(num, den)
    with np.errstate(all="ignore"):
        want = (num / den[:, None]).astype(f)
    same = (got.view(np.int32) == want.view(np.int32)) | (np.isnan(got) & np.isnan(want))
    bad = np.argwhere(~same)
    assert bad.size == 0, [(num[i, j], den[i], got[i, j], want[i, j]) for i, j in bad[:5]]


EXT = [("rtiow5", 0, 80, 45, 16, 50), ("final", 42, 64, 36, 8, 50),
       ("glass", 42, 48, 27, 8, 200), ("final", 7, 40, 22, 12, 10)]


@pytest.mark.parametrize("name,seed,W,H,spp,depth", EXT, ids=[f"{e[0]}-{e[1]}" for e in EXT])
def test_extension_scene_vs_oracle(ren, name, seed, W, H, spp, depth):
    arr, cam = yk.build_scene(name, seed)
    ren.set_scene(arr, cam)
    p = make_params(W, H, spp, depth, 404)
    _, want, _, _ = oracle_lib.render(arr, cam, p, want_rgb=False, want_sums=True)
    got = ren.render_sums(p)
    assert got.tobytes() == want.tobytes()
    rgb_o, _, _, _ = oracle_lib.render(arr, cam, p)
    np.testing.assert_array_equal(ren.render(p), rgb_o)


def test_row_tiles_reassemble(ren):
    e = next(c for c in MAN["cases"] if c["name"] == "mixed12_96x54x16_d50_s404")
    ren.set_scene(refscenes.mixed12(), refscenes.reference_camera())
    full = golden_data.rgb(e)
    for n in (2, 3, 8):
        out = np.zeros_like(full)
        for r in range(n):
            rows = len(range(r, e["H"], n))
            out[r::n] = ren.render(make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"],
                                               rows=(r, rows, n)))
        np.testing.assert_array_equal(out, full)


def test_banded_row_tiles_reassemble(ren):
    """Bands of 2^k rows dealt cyclically (bench.py --deal rows / tiles.py), including a
    partial last band: the tiles reassemble into the reference golden image bit for bit."""
    from uecraytracing_amd.tiles import tile_image_rows, tile_rows
    e = next(c for c in MAN["cases"] if c["name"] == "mixed12_96x54x16_d50_s404")
    ren.set_scene(refscenes.mixed12(), refscenes.reference_camera())
    full = golden_data.rgb(e)
    for n, L in ((2, 3), (3, 3), (8, 2), (4, 1), (3, 5)):
        out = np.zeros_like(full)
        for r in range(n):
            rows = tile_rows(r, n, e["H"], L)
            if rows[1] == 0:
                continue
            out[tile_image_rows(r, n, e["H"], L)] = ren.render(
                make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], rows=rows))
        np.testing.assert_array_equal(out, full)


def test_banded_rows_of_the_headline_config(ren):
    """Rank 5 of 8 at config 3 with bands of 8 rows (bench.py's split), first two bands vs the
    oracle, sums bit for bit."""
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    p = make_params(1920, 1080, 32, 50, 404, rows=(40, 16, 8, 3))  # rows 40-47 and 104-111
    got = ren.render_sums(p)
    _, want, _, _ = oracle_lib.render(arr, cam, p, nthreads=16, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()


def test_column_tiles_reassemble(ren):
    """Column sets (ABI 10; bench.py's N-GPU split: 8-column bands over every row), including a
    partial last band, single columns and a row set with them, in FP64, FP32 and xor128: the tiles
    reassemble into the reference golden image bit for bit."""
    from uecraytracing_amd.tiles import tile_cols, tile_image_cols
    ren.set_scene(refscenes.mixed12(), refscenes.reference_camera())
    for name, kw in (("mixed12_96x54x16_d50_s404", {}),):
        e = next(c for c in MAN["cases"] if c["name"] == name)
        full = golden_data.rgb(e)
        for n, L in ((2, 3), (3, 3), (8, 3), (5, 0), (7, 2)):
            out = np.zeros_like(full)
            for r in range(n):
                cols = tile_cols(r, n, e["W"], L)
                if cols[1] == 0:
                    continue
                out[:, tile_image_cols(r, n, e["W"], L)] = ren.render(
                    make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], cols=cols, **kw))
            np.testing.assert_array_equal(out, full)
        # a row set and a column set together
        got = ren.render(make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], rows=(1, 9, 6),
                                     cols=tile_cols(1, 3, e["W"], 3)))
        np.testing.assert_array_equal(got, full[1::6][:9][:, tile_image_cols(1, 3, e["W"], 3)])
    for prec, rng in ((PRECISION_FP32, RNG_MT19937), (PRECISION_FP64, RNG_XOR128)):
        full = ren.render(make_params(96, 54, 8, 50, 404, precision=prec, rng=rng))
        for r in range(3):
            got = ren.render(make_params(96, 54, 8, 50, 404, precision=prec, rng=rng, cols=tile_cols(r, 3, 96)))
            np.testing.assert_array_equal(got, full[:, tile_image_cols(r, 3, 96)])


def test_column_tile_of_the_headline_config(ren):
    """Rank 3 of 8 at config 3 under bench.py's column dealing (every row, 8-column bands
    24-31, 88-95, ...): two rows of the tile against the oracle's, sums bit for bit; a column set
    the image does not hold is rejected."""
    from uecraytracing_amd.tiles import tile_cols
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    p = make_params(1920, 1080, 32, 50, 404, rows=(700, 2, 1), cols=tile_cols(3, 8, 1920))
    got = ren.render_sums(p)
    assert got.shape == (2, 240, 3)
    _, want, _, _ = oracle_lib.render(arr, cam, p, nthreads=16, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()
    with pytest.raises(yk.YkError):
        ren.render(make_params(1920, 1080, 1, 50, 404, cols=(8, 240, 9, 3)))  # last band past 1920


def test_repeatable_and_counts(ren):
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    p = make_params(64, 36, 8, 50, 404, flags=1)
    a = ren.render(p)
    st = ren.stats()
    b = ren.render(p)
    np.testing.assert_array_equal(a, b)
    assert st["samples"] == 64 * 36 * 8
    assert st["segments"] >= st["samples"]
    assert 0 < st["sphere_tests"] < st["segments"] * len(arr)  # the BVH culls
    assert st["kernel_ms"] > 0
    lin = ren.render(make_params(64, 36, 8, 50, 404, flags=1 | 2))
    np.testing.assert_array_equal(lin, a)
    assert ren.stats()["sphere_tests"] == st["segments"] * len(arr)  # linear: every sphere


def test_async_into_device_memory(ren):
    torch = pytest.importorskip("torch")
    ren.set_scene(refscenes.ref4(), refscenes.reference_camera())
    e = next(c for c in MAN["cases"] if c["name"] == "ref4_32x18x6_d50_s404")
    p = make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"])
    out = torch.zeros((e["H"], e["W"], 3), dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.Stream()  # a real stream: NULL would mean the context's own stream
    ren.render_async(p, out.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), golden_data.rgb(e))


def test_back_to_back_calls_equal_a_synced_call(ren):
    """Calls enqueued while the previous one still runs overlap it (rings by global
    launch number, launches at kmax from the first) — in FP64, FP32 and xor128, with a call of
    another shape between them (which must not overlap): every output equals the synced render of
    its params, and the golden where there is one."""
    torch = pytest.importorskip("torch")
    ren.set_scene(refscenes.mixed12(), refscenes.reference_camera())
    e = next(c for c in MAN["cases"] if c["name"] == "mixed12_96x54x16_d50_s404")
    ps = [make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"]),
          make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"]),
          make_params(e["W"], e["H"], 24, e["depth"], e["seed0"], rows=(3, 20, 2)),  # another shape
          make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"]),
          make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], precision=PRECISION_FP32),
          make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], precision=PRECISION_FP32),
          make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], rng=RNG_XOR128),
          make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"], rng=RNG_XOR128)]
    want = [ren.render(p) for p in ps]
    np.testing.assert_array_equal(want[0], golden_data.rgb(e))
    outs = [torch.zeros((p.row_count, p.tile_width(), 3), dtype=torch.uint8, device="cuda:0") for p in ps]
    stream = torch.cuda.Stream()
    for rep in range(2):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()  # (the zeroing ran on torch's stream)
        for p, o in zip(ps, outs):  # no synchronisation between the calls
            ren.render_async(p, o.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        for w, o in zip(want, outs):
            np.testing.assert_array_equal(o.cpu().numpy(), w)


def test_headline_geometry_full_size_rows(ren):
    """1920x1080x512 on the ~488-sphere final scene: rows 0 and 539 bit-exact vs the oracle."""
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    p = make_params(1920, 1080, 512, 50, 404, rows=(0, 2, 539))
    got = ren.render_sums(p)
    _, want, _, _ = oracle_lib.render(arr, cam, p, nthreads=16, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()


def test_config2_full_image_vs_oracle(ren):
    """BASELINE config 2 at its own size: 800x450, 100 spp, max_depth 50, the 5-sphere
    lambertian + metal + dielectric scene, whole image, bytes and float64 sums bit-exact."""
    arr, cam = yk.build_scene("rtiow5", 0)
    ren.set_scene(arr, cam)
    p = make_params(800, 450, 100, 50, 404)
    got = ren.render_sums(p)
    rgb_o, want, _, _ = oracle_lib.render(arr, cam, p, nthreads=16, want_sums=True)
    assert got.tobytes() == want.tobytes()
    np.testing.assert_array_equal(ren.render(p), rgb_o)


def test_config4_geometry_rows_vs_oracle(ren):
    """BASELINE config 4 geometry on one GPU: 3840x2160, 1024 spp, the final scene; rows 1080
    and 2159, and the row set rank 3 of 8 renders (rows 3, 11, ...) checked on its first rows."""
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    p = make_params(3840, 2160, 1024, 50, 404, rows=(1080, 2, 1079))
    got = ren.render_sums(p)
    _, want, _, _ = oracle_lib.render(arr, cam, p, nthreads=16, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()
    tile = ren.render(make_params(3840, 2160, 64, 50, 404, rows=(3, 270, 8)))
    ref, _, _, _ = oracle_lib.render(arr, cam, make_params(3840, 2160, 64, 50, 404, rows=(3, 2, 8)),
                                     nthreads=16)
    np.testing.assert_array_equal(tile[:2], ref)


def test_config5_dielectric_rows_vs_oracle(ren):
    """BASELINE config 5: 1920x1080, 4096 spp, max_depth 200, the dielectric-heavy scene (long,
    divergent bounce chains; samples drawing past the lazy MT window); two rows bit-exact."""
    arr, cam = yk.build_scene("glass", 42)
    ren.set_scene(arr, cam)
    p = make_params(1920, 1080, 4096, 200, 404, rows=(500, 2, 40))
    got = ren.render_sums(p)
    st = ren.stats()
    _, want, _, _ = oracle_lib.render(arr, cam, p, nthreads=16, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()
    assert st["mt_fallbacks"] > 0  # the 624-word scratch engine was exercised


def test_bad_rows_rejected(ren):
    ren.set_scene(refscenes.ref4(), refscenes.reference_camera())
    with pytest.raises(yk.YkError):
        ren.render(make_params(16, 9, 2, 50, 404, rows=(8, 2, 1)))
    with pytest.raises(yk.YkError):  # banded: rows 0-3, then 8-11 (10, 11 outside)
        ren.render(make_params(16, 9, 2, 50, 404, rows=(0, 8, 2, 2)))
    with pytest.raises(yk.YkError):
        ren.render(make_params(16, 9, 2, 50, 404, rows=(0, 1, 1, 11)))


def _dupes_scene():
    """Six exactly coincident spheres (ties: the last tuple index must win) plus a ground and
    a far sphere: forces candidate-list overflow and the exact fallback."""
    from uecraytracing_amd.records import lambertian, metal
    s = [lambertian((0, -100.5, -1), 100.0, (0.8, 0.8, 0.0))]
    for k in range(6):
        s.append((lambertian if k % 2 else metal)((0, 0, -1), 0.5, (0.1 * k + 0.3, 0.5, 0.9 - 0.1 * k)))
    s.append(lambertian((3000.0, 0.0, -1.0), 2900.0, (0.2, 0.3, 0.4)))  # far: origin-bound path
    return s


@pytest.mark.parametrize("name,seed", [("final", 42), ("glass", 3), ("mixed12", 0), ("dupes", 0), ("axial", 0)])
def test_bvh_matches_linear_scan_and_oracle(ren, name, seed):
    if name == "dupes":
        arr, cam = _dupes_scene(), refscenes.reference_camera()
    elif name == "axial":  # rays within a few 2^-8 slopes of the z axis (the FP32 cone's slow axes)
        arr, cam = refscenes.axial(), refscenes.axial_camera()
    elif name == "mixed12":
        arr, cam = refscenes.mixed12(), refscenes.reference_camera()
    else:
        arr, cam = yk.build_scene(name, seed)
    ren.set_scene(arr, cam)
    p_bvh = make_params(48, 27, 8, 50, 404, flags=1)
    p_lin = make_params(48, 27, 8, 50, 404, flags=1 | 2)
    a = ren.render_sums(p_bvh)
    st = ren.stats()
    b = ren.render_sums(p_lin)
    assert a.tobytes() == b.tobytes()
    _, want, _, _ = oracle_lib.render(arr, cam, p_bvh, want_rgb=False, want_sums=True)
    assert a.tobytes() == want.tobytes()
    if name == "dupes":
        assert st["linear_scans"] > 0  # the overflow path really ran


def test_large_scene_global_memory_path(ren):
    """2600 spheres: the BVH no longer fits the LDS budget, so nodes are read from global."""
    import random
    from uecraytracing_amd.records import dielectric, lambertian, metal
    rng = random.Random(5)
    s = [lambertian((0, -1000.5, -1), 1000.0, (0.5, 0.5, 0.5))]
    for _ in range(2600):
        c = (rng.uniform(-6, 6), rng.uniform(-0.5, 3), rng.uniform(-9, -1))
        k = rng.random()
        r = rng.uniform(0.03, 0.15)
        if k < 0.6:
            s.append(lambertian(c, r, (rng.random(), rng.random(), rng.random())))
        elif k < 0.85:
            s.append(metal(c, r, (rng.random(), rng.random(), rng.random()), rng.choice([0.0, 0.2])))
        else:
            s.append(dielectric(c, r, 1.5))
    cam = refscenes.reference_camera()
    ren.set_scene(s, cam)
    p = make_params(32, 18, 4, 50, 404, flags=1)
    a = ren.render_sums(p)
    b = ren.render_sums(make_params(32, 18, 4, 50, 404, flags=3))
    assert a.tobytes() == b.tobytes()
    _, want, _, _ = oracle_lib.render(s, cam, p, want_rgb=False, want_sums=True)
    assert a.tobytes() == want.tobytes()
