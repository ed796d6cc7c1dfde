"""One render of the headline workload with YKGPU_TIMELINE=1 (per-launch event times on stderr)
and the call's stats (diagnostic).  usage: YKGPU_LIB_OVERRIDE=... python tools/timeline_once.py [spp [precision]]"""
import os
import sys

os.environ["YKGPU_TIMELINE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import make_params  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 512
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 0
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    p = make_params(1920, 1080, spp, 50, 404, precision=prec)
    r.render(p)
    print("---- timed call", file=sys.stderr, flush=True)
    r.render(p)
    st = r.stats()
    print({k: st[k] for k in ("total_ms", "kernel_ms", "render_busy_ms", "warmup_ms", "resolve_ms",
                              "launches")}, flush=True)
