"""Render time against path length on the headline scene (diagnostic): max_depth 1, 2, 3, 50 at
1920x1080 and a few spp — per-segment cost of primary-heavy vs mixed trips.
usage: python tools/depth_probe.py [spp]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import make_params  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for depth in (1, 2, 3, 50):
        p = make_params(1920, 1080, spp, depth, 404, flags=0)
        r.render(p)
        ts = []
        for _ in range(2):
            t = time.perf_counter()
            r.render(p)
            ts.append(time.perf_counter() - t)
        busy = r.stats()["render_busy_ms"]
        r.render(make_params(1920, 1080, spp, depth, 404, flags=1))
        st = r.stats()
        print(f"depth {depth}: {min(ts) * 1e3:.1f} ms call, render busy {busy:.1f} ms, segments/sample "
              f"{st['segments'] / st['samples']:.3f}, busy ns per segment x1e3 "
              f"{busy * 1e6 / st['segments'] * 1e3:.2f}, node visits/segment {st['node_visits'] / st['segments']:.2f}",
              flush=True)
