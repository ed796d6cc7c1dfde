"""The non-default modes of yk_render_params on the MI355X, through the C-ABI.

  * YK_PRECISION_FP32 — the reference's render<float> (include/ykgpu.h): bit-exact against the
    reference-generated fp32 goldens (test_gpu_parity.test_golden_case) and against the oracle's
    float path on the extension scenes; math::sqrt<float> against the reference loop.
  * YK_SEED_RANDOM_DEVICE — per-sample seeds hashed from a per-call key: bit-exact against the
    oracle for a given key; a fresh key per call when none is given, reported in the stats.
  * YK_RNG_XOR128 — the reference's yk::xor128 as the per-sample engine: bit-exact against the
    reference-generated *_x128 goldens (test_gpu_parity.test_golden_case) and against the
    oracle on the extension scenes, the BVH path, row tiles and both precisions.
"""
import numpy as np
import pytest

import golden_data
import oracle_lib
import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import PRECISION_FP32, RNG_XOR128, SEED_RANDOM_DEVICE, make_params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ren():
    r = yk.Renderer(0)
    yield r
    r.close()


def f32_sqrt_inputs(rng, n_random=1 << 22):
    """Floats around every binade boundary (2^k +- m ulp, subnormals included), random
    exponents over the whole range, the KAT inputs, zero and the smallest subnormals."""
    base = np.ldexp(np.float32(1.0), np.arange(-149, 128)).astype(np.float32).view(np.int32)
    m = np.arange(64, dtype=np.int32)
    near = np.concatenate([(base[:, None] + m).ravel(), (base[:, None] - m).ravel()]).view(np.float32)
    near = near[np.isfinite(near) & (near >= 0)]
    bits = rng.integers(1, 0x7F800000, n_random, dtype=np.int64).astype(np.int32).view(np.float32)
    kat = np.array([float.fromhex(a) for a, _ in golden_data.kat()["newton_sqrt_f32"]], np.float32)
    return np.concatenate([np.array([0.0, 1e-45, 3e-45], np.float32), near, bits, kat])


def test_math_sqrt_f32_matches_reference_loop(ren):
    x = f32_sqrt_inputs(np.random.default_rng(17))
    got = ren.math_sqrt_f32(x)
    want = oracle_lib.newton_sqrt_f32(x)
    bad = np.flatnonzero(got.view(np.int32) != want.view(np.int32))
    assert bad.size == 0, [(x[i], got[i], want[i]) for i in bad[:5]]


FP32_EXT = [("rtiow5", 0, 80, 45, 16, 50), ("final", 42, 48, 27, 8, 50), ("glass", 42, 40, 22, 8, 200)]


@pytest.mark.parametrize("name,seed,W,H,spp,depth", FP32_EXT, ids=[f"{e[0]}-{e[1]}" for e in FP32_EXT])
def test_fp32_extension_scene_vs_oracle(ren, name, seed, W, H, spp, depth):
    """Dielectric, fuzzed metal and the thin-lens camera in float (parity unpinned vs the
    reference, which has none of them): GPU == oracle float path, sums and bytes."""
    arr, cam = yk.build_scene(name, seed)
    ren.set_scene(arr, cam)
    p = make_params(W, H, spp, depth, 404, precision=PRECISION_FP32)
    rgb_o, want, _, _ = oracle_lib.render(arr, cam, p, want_sums=True)
    assert ren.render_sums(p).tobytes() == want.tobytes()
    np.testing.assert_array_equal(ren.render(p), rgb_o)


def test_fp32_is_close_to_fp64(ren):
    """render<float> and render<double> are different computations of the same image — and
    they consume the RNG differently (one draw per float canonical, two per double), so their
    noise is independent.  Their difference must be noise: at 64 spp on the reference scene,
    RMSE(fp32, fp64) stays within 1.25x RMSE(fp64 seed A, fp64 seed B)."""
    ren.set_scene(refscenes.ref4(), refscenes.reference_camera())

    def img(seed0, precision=0):
        return ren.render(make_params(200, 112, 64, 50, seed0, precision=precision)).astype(np.float64)

    def rmse(a, b):
        return np.sqrt(np.mean(((a - b) / 255.0) ** 2))

    a64 = img(404)
    floor = rmse(a64, img(0x5EED))
    d = rmse(img(404, PRECISION_FP32), a64)
    assert 0 < d < 1.25 * floor, (d, floor)


def test_fp32_row_tiles_and_counts(ren):
    """Row tiles of the reference-generated fp32 golden reassemble, through the FP32 tree (it
    culls: fewer tests than 12 per segment) and through the linear scan (flag 2: every sphere)."""
    e = next(c for c in golden_data.manifest()["cases"] if c["name"] == "mixed12_96x54x16_d50_s404_f32")
    ren.set_scene(refscenes.mixed12(), refscenes.reference_camera())
    full = golden_data.rgb(e)
    for flags in (1, 3):
        out = np.zeros_like(full)
        for r in range(3):
            rows = len(range(r, e["H"], 3))
            out[r::3] = ren.render(make_params(e["W"], e["H"], e["spp"], e["depth"], e["seed0"],
                                               rows=(r, rows, 3), precision=PRECISION_FP32, flags=flags))
            st = ren.stats()
            if flags == 3:
                assert st["linear_scans"] == st["segments"] > 0
                assert st["sphere_tests"] == st["segments"] * 12
            else:
                assert st["linear_scans"] * 1000 < st["segments"]
                assert 0 < st["sphere_tests"] < st["segments"] * 12
        np.testing.assert_array_equal(out, full)


def _scene(name, seed):
    if name in refscenes.SCENES:
        return refscenes.SCENES[name](), refscenes.reference_camera()
    if name == "axial":
        return refscenes.axial(), refscenes.axial_camera()
    if name in ("dupes", "graze"):
        return getattr(refscenes, name)(), refscenes.reference_camera()
    if name == "large":
        import random
        from uecraytracing_amd.records import dielectric, lambertian, metal
        rng = random.Random(5)
        s = [lambertian((0, -1000.5, -1), 1000.0, (0.5, 0.5, 0.5))]
        for _ in range(2600):
            c = (rng.uniform(-6, 6), rng.uniform(-0.5, 3), rng.uniform(-9, -1))
            k, r = rng.random(), rng.uniform(0.03, 0.15)
            if k < 0.6:
                s.append(lambertian(c, r, (rng.random(), rng.random(), rng.random())))
            elif k < 0.85:
                s.append(metal(c, r, (rng.random(), rng.random(), rng.random()), rng.choice([0.0, 0.2])))
            else:
                s.append(dielectric(c, r, 1.5))
        return s, refscenes.reference_camera()
    return yk.build_scene(name, seed)


FP32_TREE = [("final", 42), ("glass", 3), ("rtiow5", 0), ("mixed12", 0), ("dupes", 0), ("graze", 0),
             ("axial", 0), ("large", 0)]


@pytest.mark.parametrize("name,seed", FP32_TREE, ids=[f"{n}-{s}" for n, s in FP32_TREE])
def test_fp32_tree_matches_linear_scan_and_oracle(ren, name, seed):
    """render<float> through the FP32 tree (boxes and a per-ray cone sized by the float sphere
    test's proven error) == the linear scan == the oracle's float path, float64
    sums bit for bit; the tree culls.  'large' (2600 spheres) reads its tree from global memory."""
    arr, cam = _scene(name, seed)
    ren.set_scene(arr, cam)
    W, H, spp = (32, 18, 4) if name == "large" else (96, 54, 8)
    p = make_params(W, H, spp, 50, 404, precision=PRECISION_FP32, flags=1)
    a = ren.render_sums(p)
    st = ren.stats()
    b = ren.render_sums(make_params(W, H, spp, 50, 404, precision=PRECISION_FP32, flags=3))
    assert a.tobytes() == b.tobytes()
    _, want, _, _ = oracle_lib.render(arr, cam, p, want_rgb=False, want_sums=True)
    assert a.tobytes() == want.tobytes()
    assert st["linear_scans"] < st["segments"]
    if len(arr) > 8:
        assert st["sphere_tests"] * 2 < st["segments"] * len(arr)


@pytest.mark.parametrize("name,seed,W,spp", [("final", 42, 1920, 16), ("graze", 0, 960, 32), ("axial", 0, 480, 32)])
def test_fp32_tree_whole_frame_equals_linear_scan(ren, name, seed, W, spp):
    """Whole frames in float (33 M and 17 M samples): tree == linear scan, sums bit for bit."""
    arr, cam = _scene(name, seed)
    ren.set_scene(arr, cam)
    a = ren.render_sums(make_params(W, None, spp, 50, 404, precision=PRECISION_FP32))
    b = ren.render_sums(make_params(W, None, spp, 50, 404, precision=PRECISION_FP32, flags=2))
    assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("precision", [0, PRECISION_FP32])
def test_random_device_seed_with_key_vs_oracle(ren, precision):
    arr, cam = yk.build_scene("rtiow5", 0)
    ren.set_scene(arr, cam)
    p = make_params(64, 36, 8, 50, 404, precision=precision, seed_mode=SEED_RANDOM_DEVICE,
                    seed_key=0x0123456789ABCDEF)
    got = ren.render_sums(p)
    assert ren.stats()["seed_key"] == 0x0123456789ABCDEF
    _, want, _, _ = oracle_lib.render(arr, cam, p, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()


def test_random_device_seed_fresh_key_per_call(ren):
    """Without a key every call draws one from std::random_device (like the runtime build, the
    image is not reproducible), and the reported key reproduces the call."""
    ren.set_scene(refscenes.ref4(), refscenes.reference_camera())
    p = make_params(64, 36, 4, 50, 0, seed_mode=SEED_RANDOM_DEVICE)
    a = ren.render_sums(p)
    ka = ren.stats()["seed_key"]
    b = ren.render_sums(p)
    kb = ren.stats()["seed_key"]
    assert ka != 0 and kb != 0 and ka != kb
    assert a.tobytes() != b.tobytes()
    again = ren.render_sums(make_params(64, 36, 4, 50, 0, seed_mode=SEED_RANDOM_DEVICE, seed_key=ka))
    assert again.tobytes() == a.tobytes()
    counter = ren.render(make_params(64, 36, 64, 50, 404)).astype(np.float64)
    rnd = ren.render(make_params(64, 36, 64, 50, 0, seed_mode=SEED_RANDOM_DEVICE)).astype(np.float64)
    assert np.sqrt(np.mean(((counter - rnd) / 255.0) ** 2)) < 0.05  # same image, other noise


@pytest.mark.parametrize("name,seed,W,H,spp,depth,precision", [
    ("final", 42, 96, 54, 8, 50, 0),      # 485 spheres: the BVH path with xor128
    ("glass", 7, 64, 36, 8, 200, 0),      # dielectric-heavy, depth 200 (long paths)
    ("rtiow5", 0, 80, 45, 8, 50, PRECISION_FP32),
    ("final", 42, 48, 27, 4, 50, PRECISION_FP32),
])
def test_xor128_vs_oracle(ren, name, seed, W, H, spp, depth, precision):
    arr, cam = yk.build_scene(name, seed)
    ren.set_scene(arr, cam)
    p = make_params(W, H, spp, depth, 404, precision=precision, rng=RNG_XOR128)
    got = ren.render_sums(p)
    _, want, _, _ = oracle_lib.render(arr, cam, p, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()


def test_xor128_row_tiles_random_seed_and_counts(ren):
    """Row tiles reassemble; the random-device seeding composes with xor128; no MT fallbacks."""
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    W, H = 64, 36
    full = ren.render(make_params(W, H, 8, 50, 404, rng=RNG_XOR128))
    out = np.zeros_like(full)
    for r in range(3):
        rows = len(range(r, H, 3))
        out[r::3] = ren.render(make_params(W, H, 8, 50, 404, rows=(r, rows, 3), rng=RNG_XOR128, flags=1))
        assert ren.stats()["mt_fallbacks"] == 0
    np.testing.assert_array_equal(out, full)
    p = make_params(W, H, 4, 50, 0, rng=RNG_XOR128, seed_mode=SEED_RANDOM_DEVICE, seed_key=77)
    got = ren.render_sums(p)
    _, want, _, _ = oracle_lib.render(arr, cam, p, want_rgb=False, want_sums=True)
    assert got.tobytes() == want.tobytes()

