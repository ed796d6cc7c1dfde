"""Step-to-step spread of the headline render: N back-to-back synced calls
of the bench's workload, each with its HIP-event time, the library's render_busy_ms and the
shader clock its launches ran at (sclk_mhz, the YK_CLOCK probe); YKGPU_TIMELINE=1 adds every
launch's event times and clock on stderr.  usage: python tools/variance_probe.py [calls]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import make_params  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
ren = yk.Renderer(0)
ren.set_scene(arr, cam)
p = make_params(1920, 1080, 512, 50, 404)
tile = torch.empty((1080, 1920, 3), dtype=torch.uint8, device="cuda:0")
stream = torch.cuda.Stream()
rows = []
for k in range(calls + 1):
    with torch.cuda.stream(stream):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        ren.render_async(p, tile.data_ptr(), stream.cuda_stream)
        b.record(stream)
    torch.cuda.synchronize()
    st = ren.stats()
    print(f"---- call {k}", file=sys.stderr, flush=True)
    if k:  # (call 0 warms the allocations)
        rows.append({"ms": round(a.elapsed_time(b), 3), "render_busy_ms": round(st["render_busy_ms"], 3),
                     "sclk_mhz": round(st["sclk_mhz"], 1)})
ms = [r["ms"] for r in rows]
mhz = [r["sclk_mhz"] for r in rows]
n = len(rows)
mx, my = sum(mhz) / n, sum(ms) / n
cov = sum((x - mx) * (y - my) for x, y in zip(mhz, ms)) / n
vx = sum((x - mx) ** 2 for x in mhz) / n
vy = sum((y - my) ** 2 for y in ms) / n
print(json.dumps({"calls": rows, "ms_min": min(ms), "ms_max": max(ms), "max_over_min": round(max(ms) / min(ms), 4),
                  "ms_mean": round(my, 3), "sclk_min": min(mhz), "sclk_max": max(mhz),
                  "corr_ms_sclk": round(cov / (vx * vy) ** 0.5, 3) if vx > 0 and vy > 0 else None}))
