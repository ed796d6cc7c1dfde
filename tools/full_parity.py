"""Whole-image parity of the headline workload (and config 4's rank-0 tile) against the CPU oracle.

bench.py compares 24 rows of the timed image with the oracle every run; this renders the WHOLE
1920x1080x512 frame of BASELINE config 3 (1.06e9 samples) on the GPU through the C-ABI — RGB8 and
the float64 per-pixel sums — and on the host with oracle/yk_oracle.c on every usable core, and
compares every byte and every sum bit; likewise rank 0's row tile of config 4's 8-GPU split
(3840x2160x1024, every 8th row: 1.06e9 samples).  Prints one JSON line (bytes differing, sums
differing, RMSE and max |diff| in levels, CPU time).  ~4 minutes of CPU per workload on 16 cores.
usage: python tools/full_parity.py [config3] [config4]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import oracle_lib  # noqa: E402
import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import image_height_for, make_params  # noqa: E402
from uecraytracing_amd.tiles import rank_tile  # noqa: E402

which = sys.argv[1:] or ["config3", "config4"]
nthreads = bench.usable_cpus()[0]
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
out = {"threads": nthreads}
with yk.Renderer(0) as ren:
    ren.set_scene(arr, cam)
    for name in which:
        if name == "config3":
            W, spp, tk = 1920, 512, {}
        else:
            W, spp = 3840, 1024
            tk = rank_tile(0, 8, image_height_for(W), W, "rows")
        H = image_height_for(W)
        p = make_params(W, H, spp, 50, 404, **tk)
        t = time.perf_counter()
        g_rgb = ren.render(p)
        g_sums = ren.render_sums(p)
        tg = time.perf_counter() - t
        # the CPU image in blocks of tile rows, a progress line after each (a silent multi-minute
        # call would look hung to the GPU box's watchdog)
        t = time.perf_counter()
        rb, rc, rs = p.row_begin, p.row_count, p.row_stride
        c_rgb = np.zeros_like(g_rgb)
        c_sums = np.zeros_like(g_sums)
        step = max(1, rc // 12)
        for t0 in range(0, rc, step):
            n = min(step, rc - t0)
            q = make_params(W, H, spp, 50, 404, rows=(rb + t0 * rs, n, rs))
            c_rgb[t0:t0 + n], c_sums[t0:t0 + n], _, _ = oracle_lib.render(arr, cam, q, nthreads=nthreads,
                                                                           want_rgb=True, want_sums=True)
            print(f"{name}: CPU rows {t0 + n}/{rc} ({time.perf_counter() - t:.0f} s)", flush=True)
        tc = time.perf_counter() - t
        d = g_rgb.astype(np.int64) - c_rgb.astype(np.int64)
        out[name] = {
            "workload": f"{W}x{H}x{spp}, depth 50, final_seed42.yks, seed0 404, mt19937 + FP64"
                        + (f", rows {tk['rows']}" if tk else ", whole frame"),
            "samples": int(p.row_count) * int(p.tile_width()) * spp,
            "pixels": int(p.row_count) * int(p.tile_width()),
            "bytes_differing": int((d != 0).sum()),
            "max_abs_levels": int(np.abs(d).max()),
            "rmse": float(np.sqrt(np.mean((d / 255.0) ** 2))),
            "sums_bitwise_equal": bool(g_sums.tobytes() == c_sums.tobytes()),
            "gpu_s_two_calls": round(tg, 2), "cpu_s": round(tc, 1),
        }
        print(json.dumps({name: out[name]}), flush=True)
print(json.dumps(out), flush=True)
