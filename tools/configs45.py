"""Throughput of BASELINE configs 4 and 5 on one GPU (diagnostic probe; bench.py carries the
judged figures): config 5 = 1920x1080x4096, depth 200, the dielectric-heavy glass scene, whole
frame; config 4 = 3840x2160x1024 on the final scene, rank 0's tile of the 8-way split (tiles.DEAL;
YK_DEAL=rows: the row split).
usage: python tools/configs45.py [c4] [c5]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import image_height_for, make_params  # noqa: E402
from uecraytracing_amd.tiles import DEAL, rank_tile  # noqa: E402

which = sys.argv[1:] or ["c4", "c5"]
cases = {"c5": ("glass", 1920, 4096, 200, None), "c4": ("final", 3840, 1024, 50, (0, 8))}
with yk.Renderer(0) as r:
    for name in which:
        scene, W, spp, depth, split = cases[name]
        arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, f"{scene}_seed42.yks"))
        r.set_scene(arr, cam)
        H = image_height_for(W)
        tk = rank_tile(split[0], split[1], H, W, os.environ.get("YK_DEAL", DEAL)) if split else {}
        rows = tk.get("rows")
        p = make_params(W, H, spp, depth, 404, flags=0, **tk)
        r.render(p)
        t = time.perf_counter()
        r.render(p)
        dt = time.perf_counter() - t
        st = r.stats()
        pc = make_params(W, H, spp, depth, 404, flags=1, **tk)
        r.render(pc)
        sc = r.stats()
        n = st["samples"]
        print(f"{name}: {scene} {W}x{H}x{spp} d{depth} tile={tk}: {dt * 1e3:.1f} ms, "
              f"{n / dt / 1e6:.1f} Msamples/s, launches {st['launches']}, busy {st['render_busy_ms']:.1f} ms, "
              f"segs/sample {sc['segments'] / n:.3f}, fallbacks {sc['mt_fallbacks']}, "
              f"linear {sc['linear_scans']}", flush=True)
