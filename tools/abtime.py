"""A/B wall time of library variants on the headline workload at a chosen spp (production
instance, flags=0): one subprocess per variant run (one library per process), interleaved.
usage: python tools/abtime.py <spp> <variant> [<variant> ...]   (variant 'base' = lib/libykgpu.so,
otherwise lib/abl/libykgpu_<variant>.so; "<variant>@VAR=value[@VAR2=value2...]" also sets
environment variables of that run, e.g. base@YKGPU_BVH_BINS=32); AB_ROWS="begin:count:stride" renders a row tile only
(e.g. "0:135:8" = rank 0 of 8); AB_W sets the image width (default 1920; the height is 16:9);
AB_PREC=1 times the FP32 mode"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, time, json
sys.path.insert(0, %r)
import torch
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
arr, cam = yk.build_scene("final", 42)
r = yk.Renderer(0); r.set_scene(arr, cam)
rows = tuple(int(v) for v in sys.argv[3].split(":")) if len(sys.argv) > 3 and sys.argv[3] else None
p = make_params(int(sys.argv[5]), None, int(sys.argv[1]), 50, 404, rows=rows, flags=0, precision=int(sys.argv[4]))
img = r.render(p); ts = []
for _ in range(int(sys.argv[2])):
    t = time.perf_counter(); r.render(p); ts.append(time.perf_counter() - t)
import hashlib
st = r.stats()
print(json.dumps({"ms": round(min(ts) * 1e3, 3), "kernel_ms": round(st["kernel_ms"], 3),
                  "render_busy_ms": round(st["render_busy_ms"], 3), "call_gb": round(st["call_bytes"] / 1e9, 2),
                  "sha": hashlib.sha256(img.tobytes()).hexdigest()[:12]}))
''' % ROOT
spp = sys.argv[1]
reps = os.environ.get("AB_REPS", "3")
names = sys.argv[2:] or ["base"]
for rnd in range(2):
    for name in names:
        lname, *envspecs = name.split("@")
        lib = os.path.join(ROOT, "uecraytracing_amd/lib/libykgpu.so") if lname == "base" else \
            os.path.join(ROOT, f"uecraytracing_amd/lib/abl/libykgpu_{lname}.so")
        env = dict(os.environ, YKGPU_LIB_OVERRIDE=lib)
        for envspec in envspecs:
            k, _, v = envspec.partition("=")
            env[k] = v
        out = subprocess.run([sys.executable, "-c", CODE, spp, reps, os.environ.get("AB_ROWS", ""),
                              os.environ.get("AB_PREC", "0"), os.environ.get("AB_W", "1920")],
                             env=env, capture_output=True, text=True)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(rnd, name, line[-1] if line else out.stderr[-400:], flush=True)
