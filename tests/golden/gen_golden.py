#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container (needs /root/reference):  python tests/golden/gen_golden.py

Sources of truth, all compiled from /root/reference by oracle/Makefile into oracle/_ref/:
  * oracle/_ref/raytrace_cx16 — the reference's unmodified source.cpp, constexpr build
    (Makefile:11-12,20-21) at YK_IMAGE_WIDTH=16, YK_SPP=2, __TIME__ pinned to 00:00:00
    (SOURCE_DATE_EPOCH=0 → seed0 = 404).  Its PNG is decoded to raw RGB → cx16_ref4.rgb.
  * oracle/_ref/ref_harness — our driver over the reference headers (oracle/ref_harness.cpp):
    the same loop with the constexpr seed formula at runtime, any size; RNG / sqrt KATs; and
    scene files with the extension materials (dielectric, fuzzed metal, thin-lens camera) plugged
    into the reference's integrator (BASELINE configs 2-5 content: CASES_FILE).
The oracle restatement (oracle/yk_oracle.c) is used here ONLY to choose which samples are
interesting (long paths); every stored value comes from the reference.

Fixtures are data (inputs named by scene/size/seed, outputs as raw bytes or hashes).  Large
per-pixel sums are stored as sha256 only (a bit-exact check without the bytes).
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
CX16 = os.path.join(ROOT, "oracle", "_ref", "raytrace_cx16")

# (scene, W, H, spp, depth, seed0, store_sums_bytes)
CASES = [
    ("ref4", 16, 9, 2, 50, 404, True),          # == the constexpr build of source.cpp
    ("ref4", 200, 112, 8, 50, 404, False),      # BASELINE config 1 shape
    ("ref4", 200, 112, 64, 50, 404, False),     # 64 spp (the FP32 RMSE gate size in SURVEY)
    ("lambert3", 200, 112, 8, 50, 404, False),  # config 1 wording: 3-sphere lambertian
    ("mixed12", 96, 54, 16, 50, 404, True),     # 12 spheres, exact-duplicate tie-break
    ("walls2", 64, 36, 8, 200, 404, True),      # long paths: draws past 227 and 624
    ("ref4", 32, 18, 6, 50, 404, True),         # spp % 4 != 0: sequential tail of the sum
    ("ref4", 40, 22, 4, 1, 404, True),          # depth 1: every hit is black
    ("ref4", 40, 22, 4, 2, 404, True),          # depth 2
    ("ref4", 48, 27, 4, 50, 4294967000, True),  # seed wraps mod 2^32 inside the image
    ("ref4", 33, 17, 5, 50, 7, True),           # odd, non-16:9 size, spp 5
]
# render<float> (YK_PRECISION_FP32): the harness's render32 mode, same loop with T = float
CASES_F32 = [
    ("ref4", 16, 9, 2, 50, 404, True),
    ("ref4", 200, 112, 8, 50, 404, False),      # config 1 shape
    ("ref4", 200, 112, 64, 50, 404, False),
    ("mixed12", 96, 54, 16, 50, 404, True),
    ("walls2", 64, 36, 8, 200, 404, True),      # long paths (one draw per canonical in float)
    ("ref4", 32, 18, 6, 50, 404, True),
    ("ref4", 48, 27, 4, 50, 4294967000, True),
    ("ref4", 33, 17, 5, 50, 7, True),
]

# yk::xor128 as the per-sample engine (YK_RNG_XOR128): the harness's render_x128 / render32_x128
CASES_X128 = [
    ("ref4", 16, 9, 2, 50, 404, True),
    ("ref4", 200, 112, 8, 50, 404, False),      # config 1 shape
    ("mixed12", 96, 54, 16, 50, 404, True),
    ("walls2", 64, 36, 8, 200, 404, True),      # long paths
    ("ref4", 32, 18, 6, 50, 404, True),
    ("ref4", 48, 27, 4, 50, 4294967000, True),
    ("ref4", 33, 17, 5, 50, 7, True),
]
CASES_X128_F32 = [
    ("ref4", 16, 9, 2, 50, 404, True),
    ("mixed12", 96, 54, 16, 50, 404, True),
    ("walls2", 64, 36, 8, 200, 404, True),
]

# BASELINE configs 2-5 content (dielectric, fuzzed metal, positionable thin-lens camera): scene
# files rendered by the harness's *_file modes, i.e. through the reference's own ray_color,
# hittable_list, sphere, mt19937 and math::sqrt with the extension materials plugged in
# (oracle/ref_harness.cpp).  (scene-file fixture, W, H, spp, depth, seed0, keep_sums, fp32, x128)
SCENE_FILES = {
    # config 2's whole scene: lambertian, glass + hollow glass (negative radius), metal; lookat camera
    "rtiow5.yks": ("uecraytracing_amd/scenes/rtiow5.yks", None),
    # 48-sphere slices of the config 3/4 final scene and the config 5 glass scene (ground, the big
    # spheres and the small spheres nearest the view centre, in tuple order; thin-lens camera)
    "final48.yks": ("uecraytracing_amd/scenes/final_seed42.yks", 48),
    "glass48.yks": ("uecraytracing_amd/scenes/glass_seed42.yks", 48),
}
CASES_FILE = [
    ("rtiow5.yks", 96, 54, 16, 50, 404, True, False, False),
    ("rtiow5.yks", 200, 112, 8, 50, 404, False, False, False),   # config 1 shape on config 2's scene
    ("rtiow5.yks", 96, 54, 16, 50, 404, True, True, False),
    ("final48.yks", 96, 54, 8, 50, 404, True, False, False),
    ("final48.yks", 96, 54, 8, 50, 404, True, True, False),
    ("final48.yks", 96, 54, 8, 50, 404, True, False, True),
    ("glass48.yks", 64, 36, 8, 200, 404, True, False, False),     # config 5: depth 200, glass-heavy
    ("glass48.yks", 64, 36, 8, 200, 404, True, True, False),
]

# verbose level 3 (-l 3): the loop's console lines with every ray printed by the reference's own
# ray_color (raytracer.hpp:21-25); (scene or scene file, W, H, spp, depth, seed0, level, fp32)
VERBOSE = [
    ("ref4", 16, 9, 2, 50, 404, 3, False),
    ("ref4", 16, 9, 2, 50, 404, 3, True),
    ("final48.yks", 16, 9, 2, 50, 404, 3, False),
]


def write_scene_file(path, spheres, cam):
    """include/ykgpu.h yk_scene_write's format (%.17g round-trips every double)."""
    kinds = {0: "lambertian", 1: "metal", 2: "dielectric"}
    g = lambda v: "%.17g" % v
    with open(path, "w") as f:
        f.write(f"yk-scene 1\n# {len(spheres)} spheres; tuple order\ncamera")
        for v in (cam.origin, cam.lower_left_corner, cam.horizontal, cam.vertical, cam.lens_u, cam.lens_v):
            f.write(" " + " ".join(g(c) for c in (v[0], v[1], v[2])))
        f.write(" " + g(cam.lens_radius) + "\n")
        for sp in spheres:
            f.write("sphere %s %s\n" % (kinds[sp.material], " ".join(g(v) for v in (
                sp.center[0], sp.center[1], sp.center[2], sp.radius, sp.albedo[0], sp.albedo[1], sp.albedo[2],
                sp.fuzz, sp.ior))))


def make_scene_fixture(name, src, n, focus=(2.0, 0.2, 1.0)):
    """Copies a committed scene, or slices it to n spheres: the big ones (|r| >= 0.9, incl. the
    ground) and the small spheres nearest `focus`, kept in tuple order (ids and ties unchanged)."""
    import golden_data
    sph, cam = golden_data.read_scene_file(os.path.join(ROOT, src))
    if n is not None:
        big = [i for i, x in enumerate(sph) if abs(x.radius) >= 0.9]
        small = sorted((i for i, x in enumerate(sph) if abs(x.radius) < 0.9),
                       key=lambda i: sum((sph[i].center[k] - focus[k]) ** 2 for k in range(3)))
        sph = [sph[i] for i in sorted(big + small[:n - len(big)])]
    write_scene_file(os.path.join(HERE, name), sph, cam)
    return len(sph)


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def png_rgb(path):
    """Minimal PNG decoder (8-bit RGB, non-interlaced) for the stb output."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, W = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            W, H, bd, ct, _, _, il = struct.unpack(">IIBBBBB", body)
            assert (bd, ct, il) == (8, 2, 0)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    stride, out, prev = 3 * W, bytearray(), bytearray(3 * W)
    for y in range(H):
        f = raw[y * (stride + 1)]
        line = bytearray(raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)])
        for i in range(stride):
            a = line[i - 3] if i >= 3 else 0
            b = prev[i]
            c = prev[i - 3] if i >= 3 else 0
            if f == 1:
                line[i] = (line[i] + a) & 255
            elif f == 2:
                line[i] = (line[i] + b) & 255
            elif f == 3:
                line[i] = (line[i] + (a + b) // 2) & 255
            elif f == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                line[i] = (line[i] + pr) & 255
        out += line
        prev = line
    return bytes(out), W, H


def case_name(scene, W, H, spp, depth, seed0, f32=False, x128=False):
    return (f"{scene}_{W}x{H}x{spp}_d{depth}_s{seed0}" + ("_f32" if f32 else "")
            + ("_x128" if x128 else ""))


def main():
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    manifest = {"generator": "tests/golden/gen_golden.py", "cases": [], "samples": {}}

    # 1. the unmodified reference, constexpr build
    with tempfile.TemporaryDirectory() as td:
        subprocess.run([CX16, "image.png"], cwd=td, check=True, stdout=subprocess.DEVNULL)
        rgb, W, H = png_rgb(os.path.join(td, "image.png"))
    assert (W, H) == (16, 9)
    open(os.path.join(HERE, "cx16_ref4.rgb"), "wb").write(rgb)
    manifest["constexpr_build"] = {"file": "cx16_ref4.rgb", "scene": "ref4", "W": 16, "H": 9,
                                   "spp": 2, "depth": 50, "seed0": 404, "rgb_sha256": sha(rgb)}

    # 2. harness renders (FP64 = render() as shipped, then FP32 = render<float>; each with
    #    yk::mt19937 and with yk::xor128 as the engine)
    for f32, x128, cases in ((False, False, CASES), (True, False, CASES_F32),
                             (False, True, CASES_X128), (True, True, CASES_X128_F32)):
      for scene, W, H, spp, depth, seed0, keep_sums in cases:
        name = case_name(scene, W, H, spp, depth, seed0, f32, x128)
        mode = ("render32" if f32 else "render") + ("_x128" if x128 else "")
        with tempfile.TemporaryDirectory() as td:
            f_rgb, f_sums = os.path.join(td, "o.rgb"), os.path.join(td, "o.sums")
            subprocess.run([HARNESS, mode, scene, str(W), str(H),
                            str(spp), str(depth), str(seed0), f_rgb, f_sums], check=True)
            rgb, sums = open(f_rgb, "rb").read(), open(f_sums, "rb").read()
        entry = {"name": name, "scene": scene, "W": W, "H": H, "spp": spp, "depth": depth,
                 "seed0": seed0, "precision": "fp32" if f32 else "fp64",
                 "rng": "xor128" if x128 else "mt19937",
                 "rgb_file": name + ".rgb", "rgb_sha256": sha(rgb),
                 "sums_sha256": sha(sums)}
        open(os.path.join(HERE, name + ".rgb"), "wb").write(rgb)
        if keep_sums:
            entry["sums_file"] = name + ".sums"
            open(os.path.join(HERE, name + ".sums"), "wb").write(sums)
        manifest["cases"].append(entry)
        print("case", name, entry["rgb_sha256"][:16])
    # 2b. configs 2-5 content through the reference's integrator (scene files, *_file modes)
    for fname, (src, n) in SCENE_FILES.items():
        print("scene file", fname, make_scene_fixture(fname, src, n), "spheres")
    for fname, W, H, spp, depth, seed0, keep_sums, f32, x128 in CASES_FILE:
        scene = fname[:-4]
        name = case_name(scene, W, H, spp, depth, seed0, f32, x128)
        mode = ("render32" if f32 else "render") + ("_x128" if x128 else "") + "_file"
        with tempfile.TemporaryDirectory() as td:
            f_rgb, f_sums = os.path.join(td, "o.rgb"), os.path.join(td, "o.sums")
            subprocess.run([HARNESS, mode, os.path.join(HERE, fname), str(W), str(H),
                            str(spp), str(depth), str(seed0), f_rgb, f_sums], check=True)
            rgb, sums = open(f_rgb, "rb").read(), open(f_sums, "rb").read()
        entry = {"name": name, "scene": scene, "scene_file": fname, "W": W, "H": H, "spp": spp,
                 "depth": depth, "seed0": seed0, "precision": "fp32" if f32 else "fp64",
                 "rng": "xor128" if x128 else "mt19937",
                 "rgb_file": name + ".rgb", "rgb_sha256": sha(rgb), "sums_sha256": sha(sums)}
        open(os.path.join(HERE, name + ".rgb"), "wb").write(rgb)
        if keep_sums:
            entry["sums_file"] = name + ".sums"
            open(os.path.join(HERE, name + ".sums"), "wb").write(sums)
        manifest["cases"].append(entry)
        print("case", name, entry["rgb_sha256"][:16])
    manifest["verbose"] = []
    for scene, W, H, spp, depth, seed0, lv, f32 in VERBOSE:
        is_file = scene.endswith(".yks")
        mode = "verbose" + ("32" if f32 else "") + ("_file" if is_file else "")
        out = subprocess.run([HARNESS, mode, os.path.join(HERE, scene) if is_file else scene, str(W), str(H),
                              str(spp), str(depth), str(seed0), str(lv)], check=True, capture_output=True).stdout
        name = case_name(scene[:-4] if is_file else scene, W, H, spp, depth, seed0, f32) + f"_l{lv}.txt"
        open(os.path.join(HERE, name), "wb").write(out)
        manifest["verbose"].append({"name": name, "scene": scene[:-4] if is_file else scene,
                                    **({"scene_file": scene} if is_file else {}), "W": W, "H": H, "spp": spp,
                                    "depth": depth, "seed0": seed0, "level": lv,
                                    "precision": "fp32" if f32 else "fp64", "file": name})
        print("verbose", name, out.count(b"\n"), "lines")
    cx = manifest["constexpr_build"]["rgb_sha256"]
    assert manifest["cases"][0]["rgb_sha256"] == cx, "harness disagrees with the constexpr build"

    # 3. per-sample colours + draw counts (long paths chosen with the oracle, values from the
    #    reference harness)
    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.records import PRECISION_FP32, PRECISION_FP64, RNG_MT19937, RNG_XOR128
    import golden_data
    for scene, W, H, spp, depth, f32, x128 in [("final48", 96, 54, 8, 50, False, False),
                                               ("glass48", 64, 36, 8, 200, False, False),
                                               ("ref4", 200, 112, 8, 50, False, False),
                                               ("mixed12", 96, 54, 16, 50, False, False),
                                               ("walls2", 64, 36, 8, 200, False, False),
                                               ("ref4", 200, 112, 8, 50, True, False),
                                               ("walls2", 64, 36, 8, 200, True, False),
                                               ("mixed12", 96, 54, 16, 50, False, True),
                                               ("walls2", 64, 36, 8, 200, False, True)]:
        is_file = scene in ("final48", "glass48")
        if is_file:
            sph, cam = golden_data.read_scene_file(os.path.join(HERE, scene + ".yks"))
        else:
            sph, cam = refscenes.SCENES[scene](), refscenes.reference_camera()
        p = make_params(W, H, spp, depth, 404,
                        precision=PRECISION_FP32 if f32 else PRECISION_FP64,
                        rng=RNG_XOR128 if x128 else RNG_MT19937)
        cand = []
        for y in range(0, H, 3):
            for x in range(0, W, 5):
                for s in range(0, spp, 3):
                    _, d = oracle_lib.sample(sph, cam, p, y, x, s)
                    cand.append((d, y, x, s))
        cand.sort(reverse=True)
        pick = cand[:12] + cand[len(cand) // 2:len(cand) // 2 + 6] + cand[-4:]
        pick += [(0, 0, 0, 0), (0, H - 1, W - 1, spp - 1)]
        args = [str(v) for _, y, x, s in pick for v in (y, x, s)]
        mode = ("samples32" if f32 else "samples") + ("_x128" if x128 else "") + ("_file" if is_file else "")
        out = subprocess.run([HARNESS, mode, os.path.join(HERE, scene + ".yks") if is_file else scene, str(W), str(H),
                              str(spp), str(depth), "404"] + args,
                             check=True, capture_output=True, text=True).stdout
        manifest["samples"][scene + ("_f32" if f32 else "") + ("_x128" if x128 else "")] = {
            **({"scene": scene, "scene_file": scene + ".yks"} if is_file else {}),
            "W": W, "H": H, "spp": spp, "depth": depth, "seed0": 404,
            "precision": "fp32" if f32 else "fp64", "rng": "xor128" if x128 else "mt19937",
            "points": json.loads(out)}
        print("samples", scene, "max draws", max(e["draws"] for e in json.loads(out)))

    # 4. KATs
    kat = subprocess.run([HARNESS, "kat"], check=True, capture_output=True, text=True).stdout
    json.loads(kat)
    open(os.path.join(HERE, "kat.json"), "w").write(kat)

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("ok")


if __name__ == "__main__":
    main()
