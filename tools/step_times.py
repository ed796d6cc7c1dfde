"""Per-step event times of the bench's back-to-back render_async steps (diagnostic: the bench line
averages them).  usage: YKGPU_LIB_OVERRIDE=... python tools/step_times.py [steps] [sync_each]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import make_params  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
sync_each = len(sys.argv) > 2 and sys.argv[2] == "1"
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
ren = yk.Renderer(0)
ren.set_scene(arr, cam)
p = make_params(1920, 1080, 512, 50, 404)
tile = torch.empty((1080, 1920, 3), dtype=torch.uint8, device="cuda:0")
stream = torch.cuda.Stream()
with torch.cuda.stream(stream):
    ren.render_async(p, tile.data_ptr(), stream.cuda_stream)
torch.cuda.synchronize()
import time  # noqa: E402
ev, host, lib = [], [], []
for _ in range(steps):
    with torch.cuda.stream(stream):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        t = time.perf_counter()
        ren.render_async(p, tile.data_ptr(), stream.cuda_stream)
        host.append(round((time.perf_counter() - t) * 1e3, 2))
        b.record(stream)
        ev.append((a, b))
    if sync_each:
        torch.cuda.synchronize()
        st = ren.stats()
        lib.append((round(st["kernel_ms"], 1), round(st["render_busy_ms"], 1)))
torch.cuda.synchronize()
ts = [round(a.elapsed_time(b), 2) for a, b in ev]
print("sync_each" if sync_each else "async", ts, "mean", round(sum(ts) / len(ts), 2), "min", min(ts))
print("  host enqueue ms", host)
if lib:
    print("  library (kernel_ms, render_busy_ms)", lib)
