"""The drop-in `raytrace` program (source.cpp main) and the reference-types drop-in.

CPU: option handling, help, abort on unknown options (the reference's uncaught cxxopts
exception), PNG writer.  GPU: the rendered PNG's pixels equal the reference's constexpr build,
and the reference's own scene types rendered through the bridge equal it too."""
import os
import subprocess

import numpy as np
import pytest

import golden_data
import uecraytracing_amd as yk

CLI = yk.CLI_PATH
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ref_dropin")


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
def test_bad_arguments_abort_like_uncaught_cxxopts(args):
    r = run(*args)
    assert r.returncode in (-6, 134)
    assert "what():" in r.stderr


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
