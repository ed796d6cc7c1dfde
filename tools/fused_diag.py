"""Diagnostic counters of a fused first-segment render build (-DYK_PRIMARY_SPLIT=2 -DYK_FUSED_DIAG,
DESIGN.md §9): one warm and one timed call of the headline workload at the given spp; prints the
call's time and ykgpu_get_stats diag[0..3] (producer pauses, idle waits, consumer trips with free
lanes and no chunk, regions rendered by non-producer waves) per million samples.
usage: YKGPU_LIB_OVERRIDE=... python tools/fused_diag.py [spp]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import make_params  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 512
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    p = make_params(1920, 1080, spp, 50, 404)
    r.render(p)
    t = time.perf_counter()
    r.render(p)
    ms = (time.perf_counter() - t) * 1e3
    st = r.stats()
    n = st["samples"] / 1e6
    print(json.dumps({"spp": spp, "ms": round(ms, 3), "samples": st["samples"],
                      "diag_per_msample": [round(v / n, 3) for v in st["diag"]], "diag": list(st["diag"])}))
