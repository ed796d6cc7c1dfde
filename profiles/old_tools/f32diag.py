"""Work counters of the FP32 tree vs the FP64 tree (diagnostic).
usage: python tools/f32diag.py [W H SPP [scene ...]]   (default 96 54 16 mixed12 final graze)"""
import sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import PRECISION_FP32, make_params

W, H, SPP = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (96, 54, 16)
names = sys.argv[4:] or ["mixed12", "final", "graze"]
with yk.Renderer(0) as r:
    for name in names:
        if name == "final":
            arr, cam = yk.build_scene("final", 42)
        else:
            arr, cam = getattr(refscenes, name)(), refscenes.reference_camera()
        r.set_scene(arr, cam)
        for prec in (0, PRECISION_FP32):
            r.render(make_params(W, H, SPP, 50, 404, precision=prec, flags=1))
            st = r.stats()
            sg = max(1, st["segments"])
            per = {k: round(st[k] / sg, 4) for k in ("linear_scans", "node_visits", "sphere_tests", "sqrt_calls")}
            print(name, "fp32" if prec else "fp64", {"segments": st["segments"], **per,
                                                     "linear_scans_total": st["linear_scans"]}, flush=True)
