"""Per-launch timelines (YKGPU_TIMELINE=1) of several consecutive headline calls (diagnostic)."""
import os, sys
os.environ["YKGPU_TIMELINE"] = "1"
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    p = make_params(1920, 1080, 512, 50, 404)
    for i in range(7):
        print(f"---- call {i}", file=sys.stderr, flush=True)
        r.render(p)
