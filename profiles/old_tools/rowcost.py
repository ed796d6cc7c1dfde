"""Work per row band of the headline image (counting instance): segments and node visits per
pixel, to study the pixel processing order.  usage: python tools/rowcost.py [spp] [band]"""
import json
import sys

sys.path.insert(0, '.')
import torch  # noqa: F401  (one HIP runtime: torch's)
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
band = int(sys.argv[2]) if len(sys.argv) > 2 else 27
arr, cam = yk.build_scene("final", 42)
out = []
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for r0 in range(0, 1080, band):
        p = make_params(1920, 1080, spp, 50, 404, rows=(r0, min(band, 1080 - r0), 1), flags=1)
        r.render(p)
        st = r.stats()
        n = st["samples"]
        out.append({"row": r0, "segs": st["segments"] / n, "nodes": st["node_visits"] / n,
                    "tests": st["sphere_tests"] / n, "ms": st["kernel_ms"]})
        print(json.dumps(out[-1]), flush=True)
