"""Work counters of the FP32 tree vs the FP64 tree on a few scenes (diagnostic)."""
import sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import PRECISION_FP32, make_params

with yk.Renderer(0) as r:
    for name in ("mixed12", "final", "graze"):
        if name == "final":
            arr, cam = yk.build_scene("final", 42)
        else:
            arr, cam = getattr(refscenes, name)(), refscenes.reference_camera()
        r.set_scene(arr, cam)
        for prec in (0, PRECISION_FP32):
            r.render(make_params(96, 54, 16, 50, 404, precision=prec, flags=1))
            st = r.stats()
            print(name, "fp32" if prec else "fp64", {k: st[k] for k in ("segments", "linear_scans", "node_visits", "sphere_tests", "sqrt_calls", "diag", "phase_cycles")}, flush=True)
