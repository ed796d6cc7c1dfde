"""The repository's `raytrace` program, the reference's own source.cpp with the integration patch
(real cxxopts, real stb_image_write), and the reference-types drop-in.

CPU: option handling, help, bad arguments, PNG writer.  GPU: the patched reference's PNG equals
the reference's constexpr build byte for byte; its console output equals the unmodified runtime
build's (-l 2) and, at -l 3, the rays the reference's own ray_color prints (harness fixture);
the repository CLI's pixels and verbose lines match too."""
import os
import subprocess

import numpy as np
import pytest

import golden_data
import uecraytracing_amd as yk

CLI = yk.CLI_PATH
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(ROOT, "oracle", "_ref")
DROPIN = os.path.join(REF_BIN, "ref_dropin")
PATCHED = {k: os.path.join(REF_BIN, "raytrace_ykgpu" + k) for k in ("", "_16x2", "_200x8", "_3840x2")}
CX16 = os.path.join(REF_BIN, "raytrace_cx16")
RT16 = os.path.join(REF_BIN, "raytrace_rt16")
MAN = golden_data.manifest()


def need(path):
    if not os.path.exists(path):
        pytest.skip(f"{os.path.relpath(path, ROOT)} not built (needs /root/reference at build time)")


def run(*args, cwd=None):
    return subprocess.run([CLI, *args], capture_output=True, text=True, cwd=cwd, timeout=300)


def test_cli_built():
    assert os.path.exists(CLI), "build with make -C uecraytracing_amd/csrc"


@pytest.mark.parametrize("args", [[], ["-h"], ["--help"], ["-v"], ["-l", "2"]])
def test_help_when_no_output(args):
    r = run(*args)
    assert r.returncode == 0
    assert r.stdout.startswith("raytracing program\nUsage:\n  raytrace [OPTION...] positional parameters")
    for opt in ("-h, --help", "-v, --verbose", "-o, --output arg", "-l, --verbose-level arg"):
        assert opt in r.stdout


@pytest.mark.parametrize("args", [["-x", "a.png"], ["--bogus", "a.png"], ["a.png", "b.png"],
                                  ["-l", "x", "a.png"]])
def test_bad_arguments_are_reported(args):
    r = run(*args)
    assert r.returncode == 2
    assert r.stderr.startswith("raytrace: ") and "see --help" in r.stderr


def test_no_gpu_fails_loudly(tmp_path):
    if yk.device_count() > 0:
        pytest.skip("GPU present")
    r = run("--width", "16", "--spp", "1", "--seed0", "404", str(tmp_path / "o.png"))
    assert r.returncode == 1 and "no HIP device" in r.stderr
    assert not (tmp_path / "o.png").exists()


@pytest.mark.gpu
def test_cli_renders_the_constexpr_image(tmp_path):
    out = tmp_path / "image.png"
    r = run("--width", "16", "--spp", "2", "--seed0", "404", str(out))
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ["rendering...", "rendering finished",
                                     f"write to file : {out}", "success"]
    rgb, W, H = golden_data.png_rgb(str(out))
    assert (W, H) == (16, 9)
    assert golden_data.sha(np.frombuffer(rgb, np.uint8)) == golden_data.manifest()["constexpr_build"]["rgb_sha256"]


@pytest.mark.gpu
def test_cli_verbose_lines_and_options(tmp_path):
    out = tmp_path / "v.png"
    r = run("-o", str(out), "-v", "-l", "2", "-l", "1", "--width", "16", "--spp", "2", "--seed0", "404")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    px = [l for l in lines if l.startswith("(row,col) :")]
    # setw(ceil(log10(n)) - 1), source.cpp:130-133: width 0 for H = 9, 1 for W = 16
    assert len(px) == 16 * 9 and px[0] == "(row,col) : (0, 0)".replace(" 0)", "0)") and px[-1] == "(row,col) : (8,15)"
    assert not any(l.startswith("(row,col,sam)") for l in lines)  # the last -l wins


@pytest.mark.gpu
def test_cli_scene_matches_library(tmp_path):
    out = tmp_path / "f.png"
    r = run("--scene", "final", "--width", "64", "--spp", "4", "--seed0", "7", str(out))
    assert r.returncode == 0, r.stderr
    rgb, W, H = golden_data.png_rgb(str(out))
    arr, cam = yk.build_scene("final", 42)
    with yk.Renderer(0) as ren:
        ren.set_scene(arr, cam)
        want = ren.render(yk.make_params(64, None, 4, 50, 7))
    assert rgb == want.tobytes()


@pytest.mark.gpu
def test_cli_xor128_matches_reference_golden(tmp_path):
    """--rng xor128: the reference's yk::xor128 as the engine (harness render_x128 golden)."""
    out = tmp_path / "x.png"
    r = run("--width", "16", "--spp", "2", "--seed0", "404", "--rng", "xor128", str(out))
    assert r.returncode == 0, r.stderr
    rgb, W, H = golden_data.png_rgb(str(out))
    e = next(c for c in golden_data.manifest()["cases"] if c["name"] == "ref4_16x9x2_d50_s404_x128")
    assert golden_data.sha(np.frombuffer(rgb, np.uint8)) == e["rgb_sha256"]


def test_cli_rejects_unknown_rng(tmp_path):
    r = run("--width", "16", "--spp", "1", "--seed0", "1", "--rng", "pcg", str(tmp_path / "o.png"))
    assert r.returncode == 1 and "unknown rng" in r.stderr


@pytest.mark.gpu
def test_reference_types_drop_in(tmp_path):
    if not os.path.exists(DROPIN):
        pytest.skip("oracle/_ref/ref_dropin not built (needs /root/reference at build time)")
    out = tmp_path / "d.rgb"
    r = subprocess.run([DROPIN, str(out), "16", "2", "50", "404"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert golden_data.sha(np.frombuffer(out.read_bytes(), np.uint8)) == \
        golden_data.manifest()["constexpr_build"]["rgb_sha256"]
    e = next(c for c in golden_data.manifest()["cases"] if c["name"] == "ref4_200x112x8_d50_s404")
    r = subprocess.run([DROPIN, str(out), "200", "8", "50", "404"], capture_output=True, timeout=300)
    assert r.returncode == 0
    assert golden_data.sha(np.frombuffer(out.read_bytes(), np.uint8)) == e["rgb_sha256"]


def _block(stdout):
    """The render loop's console lines: between "rendering..." and "rendering finished"."""
    lines = stdout.splitlines()
    return lines[lines.index("rendering...") + 1:lines.index("rendering finished")]


@pytest.mark.gpu
def test_patched_reference_png_is_the_constexpr_builds_byte_for_byte(tmp_path):
    """source.cpp + oracle/source_cpp_ykgpu.patch (real cxxopts, real stb_image_write, render()'s
    loop on the GPU) at 16x9x2: its PNG FILE equals the unmodified constexpr build's."""
    need(PATCHED["_16x2"])
    need(CX16)
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    r = subprocess.run([PATCHED["_16x2"], "image.png"], cwd=a, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ["rendering...", "rendering finished", "write to file : image.png", "success"]
    r2 = subprocess.run([CX16, "image.png"], cwd=b, capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0
    assert (a / "image.png").read_bytes() == (b / "image.png").read_bytes()


@pytest.mark.gpu
def test_patched_reference_200x112x8_and_default_size(tmp_path):
    need(PATCHED["_200x8"])
    r = subprocess.run([PATCHED["_200x8"], "-o", "o.png"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rgb, W, H = golden_data.png_rgb(str(tmp_path / "o.png"))
    e = next(c for c in MAN["cases"] if c["name"] == "ref4_200x112x8_d50_s404")
    assert (W, H) == (200, 112) and golden_data.sha(np.frombuffer(rgb, np.uint8)) == e["rgb_sha256"]
    # the reference's default constants (source.cpp:43-53): 400x225x100, against the oracle
    need(PATCHED[""])
    r = subprocess.run([PATCHED[""], "d.png"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rgb, W, H = golden_data.png_rgb(str(tmp_path / "d.png"))
    assert (W, H) == (400, 225)
    import oracle_lib
    import refscenes
    want, _, _, _ = oracle_lib.render(refscenes.ref4(), refscenes.reference_camera(),
                                      yk.make_params(400, 225, 100, 50, 404), nthreads=16)
    assert rgb == want.tobytes()


@pytest.mark.gpu
def test_patched_reference_on_several_devices(tmp_path):
    """The patched source.cpp with YKGPU_DEVICES naming three contexts (the bridge's group: rows
    dealt over them, include/ykgpu.h): the same PNG file as one device, at 200x112x8 (the golden)
    and at 16x9x2 (the constexpr build's file), and -l 3 traces still equal the single device's."""
    need(PATCHED["_200x8"])
    need(PATCHED["_16x2"])
    env = dict(os.environ, YKGPU_DEVICES="0,0,0")
    for exe in (PATCHED["_200x8"], PATCHED["_16x2"]):
        a, b = tmp_path / ("a" + os.path.basename(exe)), tmp_path / ("b" + os.path.basename(exe))
        a.mkdir()
        b.mkdir()
        r = subprocess.run([exe, "image.png"], cwd=a, capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        r2 = subprocess.run([exe, "image.png"], cwd=b, capture_output=True, text=True, timeout=300)
        assert r2.returncode == 0, r2.stderr
        assert (a / "image.png").read_bytes() == (b / "image.png").read_bytes()
    rgb, W, H = golden_data.png_rgb(str(tmp_path / "araytrace_ykgpu_200x8" / "image.png"))
    e = next(c for c in MAN["cases"] if c["name"] == "ref4_200x112x8_d50_s404")
    assert golden_data.sha(np.frombuffer(rgb, np.uint8)) == e["rgb_sha256"]
    a = subprocess.run([PATCHED["_16x2"], "-l", "3", "o.png"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300, env=env)
    b = subprocess.run([PATCHED["_16x2"], "-l", "3", "o.png"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    assert a.returncode == b.returncode == 0 and a.stdout == b.stdout


@pytest.mark.gpu
def test_patched_reference_at_config4_geometry_on_eight_contexts(tmp_path):
    """Config 4's image size through the reference's own main, cxxopts and stb: 3840x2160 (the
    size whose 24.9 MB image_t overflows the unmodified runtime build's 8 MB stack) at
    2 spp, its rows dealt over eight contexts (YKGPU_DEVICES=0,...,0: the 8-GPU split's 270-row
    tiles), run under the default 8 MB stack; rows 0, 1079 and 2159 equal the oracle's."""
    need(PATCHED["_3840x2"])
    env = dict(os.environ, YKGPU_DEVICES=",".join(["0"] * 8))
    r = subprocess.run(["bash", "-c", 'ulimit -s 8192 && "$0" "$1"', PATCHED["_3840x2"], "c4.png"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.splitlines() == ["rendering...", "rendering finished", "write to file : c4.png", "success"]
    rgb, W, H = golden_data.png_rgb(str(tmp_path / "c4.png"))
    assert (W, H) == (3840, 2160)
    img = np.frombuffer(rgb, np.uint8).reshape(H, W, 3)
    import oracle_lib
    import refscenes
    for rows in ((0, 2, 2159), (1079, 1, 1)):
        want, _, _, _ = oracle_lib.render(refscenes.ref4(), refscenes.reference_camera(),
                                          yk.make_params(3840, 2160, 2, 50, 404, rows=rows), nthreads=16)
        ys = [rows[0] + k * rows[2] for k in range(rows[1])]
        np.testing.assert_array_equal(img[ys], want)


def test_patched_reference_rejects_a_bad_device_list(tmp_path):
    """YKGPU_DEVICES that is not a device list fails loudly before any device is touched."""
    need(PATCHED["_16x2"])
    for bad in ("x", "0,,1", "-1", "0;1", "0,", "99"):
        r = subprocess.run([PATCHED["_16x2"], "o.png"], cwd=tmp_path, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, YKGPU_DEVICES=bad))
        assert r.returncode != 0
        assert "YKGPU_DEVICES" in r.stderr, r.stderr
        assert not (tmp_path / "o.png").exists()


def test_patched_reference_rejects_unknown_render_modes(tmp_path):
    """YKGPU_SEED / YKGPU_PRECISION / YKGPU_RNG (the bridge's options_from_env) that name no mode
    fail loudly before any device is touched."""
    need(PATCHED["_16x2"])
    for var, bad in (("YKGPU_SEED", "urandom"), ("YKGPU_PRECISION", "fp16"), ("YKGPU_RNG", "pcg")):
        r = subprocess.run([PATCHED["_16x2"], "o.png"], cwd=tmp_path, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **{var: bad}))
        assert r.returncode != 0
        assert var in r.stderr and bad in r.stderr, r.stderr
        assert not (tmp_path / "o.png").exists()


@pytest.mark.gpu
def test_patched_reference_render_modes_from_the_environment(tmp_path):
    """The drop-in's other modes through the reference's own main: YKGPU_PRECISION=fp32
    (render<float>) and YKGPU_RNG=xor128 give the library's images of those modes byte for byte
    (themselves pinned to the reference by goldens); YKGPU_SEED=random_device is the runtime
    build's per-sample std::random_device seeding (source.cpp:159): two runs differ from each
    other and from the counter-seeded image."""
    need(PATCHED["_200x8"])
    from uecraytracing_amd.records import PRECISION_FP32, RNG_XOR128
    import refscenes
    with yk.Renderer(0) as r:
        r.set_scene(refscenes.ref4(), refscenes.reference_camera())
        for var, val, kw in (("YKGPU_PRECISION", "fp32", {"precision": PRECISION_FP32}),
                             ("YKGPU_RNG", "xor128", {"rng": RNG_XOR128})):
            want = r.render(yk.make_params(200, 112, 8, 50, 404, **kw))
            out = subprocess.run([PATCHED["_200x8"], f"{val}.png"], cwd=tmp_path, capture_output=True, text=True,
                                 timeout=300, env=dict(os.environ, **{var: val}))
            assert out.returncode == 0, out.stderr
            rgb, W, H = golden_data.png_rgb(str(tmp_path / f"{val}.png"))
            assert (W, H) == (200, 112) and rgb == want.tobytes()
    imgs = []
    for k in range(2):
        out = subprocess.run([PATCHED["_200x8"], f"rd{k}.png"], cwd=tmp_path, capture_output=True, text=True,
                             timeout=300, env=dict(os.environ, YKGPU_SEED="random_device"))
        assert out.returncode == 0, out.stderr
        rgb, W, H = golden_data.png_rgb(str(tmp_path / f"rd{k}.png"))
        assert (W, H) == (200, 112)
        imgs.append(rgb)
    e = next(c for c in MAN["cases"] if c["name"] == "ref4_200x112x8_d50_s404")
    assert imgs[0] != imgs[1]
    assert all(golden_data.sha(np.frombuffer(x, np.uint8)) != e["rgb_sha256"] for x in imgs)


@pytest.mark.gpu
def test_patched_reference_console_matches_runtime_build(tmp_path):
    """-v / -l 2: the unmodified runtime build's lines do not depend on its random seeds, so the
    patched build's whole stdout must equal it (cxxopts parsing, messages, setw widths)."""
    need(PATCHED["_16x2"])
    need(RT16)
    for args in (["-v", "o.png"], ["-l", "2", "o.png"], ["-l", "1", "-l", "2", "--output", "o.png"]):
        a = subprocess.run([PATCHED["_16x2"], *args], cwd=tmp_path, capture_output=True, text=True, timeout=300)
        b = subprocess.run([RT16, *args], cwd=tmp_path, capture_output=True, text=True, timeout=300)
        assert a.returncode == b.returncode == 0, a.stderr
        assert a.stdout == b.stdout, args
    # -l 3: the non-ray lines still equal the runtime build's (its rays use random seeds)
    a = subprocess.run([PATCHED["_16x2"], "-l", "3", "o.png"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    b = subprocess.run([RT16, "-l", "3", "o.png"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    keep = lambda t: [l for l in t.splitlines() if not l.startswith("ray {")]
    assert keep(a.stdout) == keep(b.stdout)


def _verbose_fixture(name):
    e = next(v for v in MAN["verbose"] if v["name"] == name)
    return e, open(os.path.join(golden_data.GOLDEN, e["file"])).read().splitlines()


@pytest.mark.gpu
def test_patched_reference_l3_rays_match_reference_ray_color(tmp_path):
    """-l 3: every ray the reference's own ray_color prints (raytracer.hpp:21-25, harness
    fixture at seed0 404), line for line, from the patched source.cpp (ykgpu_render_trace)."""
    need(PATCHED["_16x2"])
    _, want = _verbose_fixture("ref4_16x9x2_d50_s404_l3.txt")
    r = subprocess.run([PATCHED["_16x2"], "-l", "3", "o.png"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert _block(r.stdout) == want


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref4_16x9x2_d50_s404_l3.txt", "ref4_16x9x2_d50_s404_f32_l3.txt",
                                  "final48_16x9x2_d50_s404_l3.txt"])
def test_cli_l3_rays_match_reference_ray_color(tmp_path, name):
    """The repository CLI's -l 3 (FP64, FP32 and a thin-lens scene file with fuzzed metal and glass)."""
    e, want = _verbose_fixture(name)
    args = ["-l", "3", "--width", "16", "--spp", "2", "--seed0", "404"]
    if e["precision"] == "fp32":
        args += ["--precision", "fp32"]
    if "scene_file" in e:
        args += ["--scene-file", os.path.join(golden_data.GOLDEN, e["scene_file"])]
    r = run(*args, str(tmp_path / "o.png"))
    assert r.returncode == 0, r.stderr
    assert _block(r.stdout) == want
