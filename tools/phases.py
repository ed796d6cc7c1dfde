"""Per-phase wave-cycle shares from the YK_ABLATE=8 stamp build (diagnostic only)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
scene = sys.argv[1] if len(sys.argv) > 1 else "final"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 32
arr, cam = yk.build_scene(scene, 42)
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    p = make_params(1920, None, spp, 50, 404, flags=1)
    r.render(p); r.render(p)
    st = r.stats()
    pc = st["phase_cycles"]; tot = sum(pc) or 1
    names = ["refill", "start", "traversal", "candidates", "shade", "path_end"]
    print(scene, f"kernels {st['kernel_ms']:.1f} ms", " ".join(f"{n}={c/tot*100:.1f}%" for n, c in zip(names, pc)))
