"""Per-phase wave-cycle shares from the stamp build (yk_stamps.hpp, -DYK_STAMPS=1; diagnostic only).
usage: [PREC=1] [ROWS=b:c:s] [DEPTH=n] python tools/phases.py [scene [spp]]   (PREC=1: render<float>; DEPTH: max_depth, 50)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
scene = sys.argv[1] if len(sys.argv) > 1 else "final"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 32
arr, cam = yk.build_scene(scene, 42)
prec = int(os.environ.get("PREC", "0"))
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    rows = tuple(int(v) for v in os.environ["ROWS"].split(":")) if os.environ.get("ROWS") else None
    p = make_params(1920, None, spp, int(os.environ.get("DEPTH", "50")), 404, rows=rows, flags=1, precision=prec)
    r.render(p); r.render(p)
    st = r.stats()
    pc = st["phase_cycles"]
    node_iters = pc[7]
    pc = pc[:7]; tot = sum(pc) or 1
    names = ["refill", "start", "trav_nodes", "candidates", "shade", "path_end", "trav_leaves", "-"]
    print(scene, "fp32" if prec else "fp64", f"kernels {st['kernel_ms']:.1f} ms", " ".join(f"{n}={c/tot*100:.1f}%" for n, c in zip(names, pc)))
    seg = max(1, st["segments"])
    print("wave-cycles per lane-segment:", " ".join(f"{n}={c/seg:.0f}" for n, c in zip(names, pc)), f"total={tot/seg:.0f}")
    tl = st["timeline"]
    if tl[0] and tl[2] > tl[0]:
        span = tl[2] - tl[0]
        print(f"timeline: pixels exhausted at {(tl[1] - tl[0]) / span * 100:.1f}% of the launch "
              f"({span / 1e5:.1f} ms), tail {(tl[2] - tl[1]) / span * 100:.1f}%")
    diag = st["diag"]
    r.render(make_params(1920, None, spp, 50, 404, rows=rows, flags=1, precision=prec))
    st2 = r.stats()
    print(f"leaf tests {st2['sphere_tests']}, with disc >= 0 {diag[0]} ({diag[0] / max(1, st2['sphere_tests']):.3f})")
    print(f"node visits (lanes) {st2['node_visits']}, wave-level node-loop iterations {node_iters} -> "
          f"lane utilisation in the node loop {st2['node_visits'] / max(1, node_iters * 64):.3f}; "
          f"wave-cycles per node iteration {pc[2] / max(1, node_iters):.0f}")
