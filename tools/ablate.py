"""Timing of ablation builds (YK_ABLATE masks) against the real library, interleaved in one
process per variant run (subprocess per variant: one library per process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, time, json
sys.path.insert(0, %r)
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
arr, cam = yk.build_scene("final", 42)
r = yk.Renderer(0); r.set_scene(arr, cam)
p = make_params(1920, None, int(sys.argv[1]), 50, 404, flags=0)  # production instance
r.render(p); ts = []
for _ in range(3):
    r.render(p); ts.append(r.stats()["kernel_ms"])
r.render(make_params(1920, None, int(sys.argv[1]), 50, 404, flags=1))  # work counters
st = r.stats()
sg = st["segments"]
print(json.dumps({"ms": round(min(ts), 3), "segs": round(sg / st["samples"], 4),
                  "nodes/seg": round(st["node_visits"] / sg, 3), "tests/seg": round(st["sphere_tests"] / sg, 3)}))
''' % ROOT
variants = [("base", os.path.join(ROOT, "uecraytracing_amd/lib/libykgpu.so"))]
for m in sys.argv[2:] or ["1", "2", "3"]:
    variants.append((f"v_{m}", os.path.join(ROOT, f"uecraytracing_amd/lib/abl/libykgpu_{m}.so")))
spp = sys.argv[1] if len(sys.argv) > 1 else "64"
for rnd in range(2):
    for name, lib in variants:
        env = dict(os.environ, YKGPU_LIB_OVERRIDE=lib)
        out = subprocess.run([sys.executable, "-c", CODE, spp], env=env, capture_output=True, text=True)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(rnd, name, line[-1] if line else out.stderr[-400:], flush=True)
