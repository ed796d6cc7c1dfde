"""Quick throughput/work-count probe (not the contract bench): final scene at a few sizes."""
import sys
import time

sys.path.insert(0, '.')
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params

scene = sys.argv[1] if len(sys.argv) > 1 else "final"
arr, cam = yk.build_scene(scene, 42)
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for (W, spp) in [tuple(map(int, a.split("x"))) for a in (sys.argv[2:] or ["192x16", "480x32", "1920x16"])]:
        p = make_params(W, None, spp, 50, 404, flags=1)
        r.render(p)
        t = time.time()
        r.render(p)
        dt = time.time() - t
        st = r.stats()
        n, sg = st["samples"], max(1, st["segments"])
        print(f"W={W} spp={spp}: {dt*1e3:.1f} ms wall, kernels {st['kernel_ms']:.1f} ms, "
              f"{n/st['kernel_ms']/1e3:.1f} Msamples/s | segs/sample {sg/n:.3f} nodes/seg "
              f"{st['node_visits']/sg:.2f} tests/seg {st['sphere_tests']/sg:.2f} sqrt/seg "
              f"{st['sqrt_calls']/sg:.3f} linear {st['linear_scans']} fb {st['mt_fallbacks']} "
              f"grid {st['grid_blocks']}", flush=True)
