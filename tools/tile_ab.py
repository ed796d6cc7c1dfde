"""A/B of one rank's tile of the N-GPU split timed as the N-GPU bench's steps run it: one warm
call, then `calls` back-to-back render_async calls, ms per call (HIP events), two interleaved
rounds, one subprocess per variant run (variants as tools/abtime.py: base or
lib/abl/libykgpu_<name>.so, "@VAR=value" settings).  TILE="W:spp:N:rank:deal" (default the
config-3 8-way tile "1920:512:8:0:cols"; N = 1 times the whole frame; deal "rows3": rows in
bands of 8).
usage: [TILE=...] python tools/tile_ab.py <variant> [<variant> ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, json, os
sys.path.insert(0, %r)
import torch
import uecraytracing_amd as yk
from uecraytracing_amd.records import image_height_for, make_params
from uecraytracing_amd.tiles import rank_tile
W, spp, n, rank, deal = sys.argv[1].split(":")
W, spp, n, rank = int(W), int(spp), int(n), int(rank)
band = int(deal[4:]) if deal.startswith("rows") and len(deal) > 4 else None  # "rows3": 8-row bands
deal = deal[:4]
H = image_height_for(W)
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
ren = yk.Renderer(0); ren.set_scene(arr, cam)
p = make_params(W, H, spp, 50, 404, flags=0, **(rank_tile(rank, n, H, W, deal, band) if n > 1 else {}))
buf = torch.empty((p.row_count, p.tile_width(), 3), dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()
calls = int(sys.argv[2])
with torch.cuda.stream(s):
    ren.render_async(p, buf.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
res = []
for rep in range(2):
    with torch.cuda.stream(s):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(calls):
            ren.render_async(p, buf.data_ptr(), s.cuda_stream)
        e1.record(s)
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / calls)
st = ren.stats()
print(json.dumps({"ms_per_call": round(min(res), 3), "launches": st["launches"],
                  "call_gb": round(st["call_bytes"] / 1e9, 2)}))
''' % ROOT
tile = os.environ.get("TILE", "1920:512:8:0:cols")
calls = os.environ.get("CALLS", "6")
for rnd in range(2):
    for name in sys.argv[1:] or ["base"]:
        lname, *envspecs = name.split("@")
        lib = os.path.join(ROOT, "uecraytracing_amd/lib/libykgpu.so") if lname == "base" else \
            os.path.join(ROOT, f"uecraytracing_amd/lib/abl/libykgpu_{lname}.so")
        env = dict(os.environ, YKGPU_LIB_OVERRIDE=lib)
        for envspec in envspecs:
            k, _, v = envspec.partition("=")
            env[k] = v
        out = subprocess.run([sys.executable, "-c", CODE, tile, calls], env=env, capture_output=True, text=True)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(rnd, tile, name, line[-1] if line else out.stderr[-400:], flush=True)
