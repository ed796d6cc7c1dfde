import sys, time
sys.path.insert(0, '.')
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
arr, cam = yk.build_scene("final", 42)
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for (W, spp) in ((192, 16), (480, 32), (1920, 16)):
        p = make_params(W, None, spp, 50, 404, flags=1)
        r.render(p)
        t = time.time(); r.render(p); dt = time.time() - t
        st = r.stats()
        n = st["samples"]
        print(f"W={W} spp={spp}: {dt*1e3:.1f} ms wall, kernel {st['kernel_ms']:.1f} ms, "
              f"{n/st['kernel_ms']/1e3:.1f} Msamples/s, segs/sample {st['segments']/n:.2f}, "
              f"sqrt/seg {st['sqrt_calls']/max(1,st['segments']):.2f}, fb {st['mt_fallbacks']}, grid {st['grid_blocks']}", flush=True)
