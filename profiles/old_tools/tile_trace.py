"""One row-tile render (the rank-0 tile of an N-way split) for a kernel-trace timeline.
usage: python tools/tile_trace.py <N> [spp]"""
import sys
import time
sys.path.insert(0, '.')
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
n = int(sys.argv[1]); spp = int(sys.argv[2]) if len(sys.argv) > 2 else 512
arr, cam = yk.build_scene("final", 42)
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    p = make_params(1920, None, spp, 50, 404, rows=(0, len(range(0, 1080, n)), n))
    r.render(p)
    t = time.perf_counter(); r.render(p); print(f"N={n}: {1e3*(time.perf_counter()-t):.1f} ms", r.stats()["launches"], "launches")
