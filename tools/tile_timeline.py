"""Per-launch timeline (YKGPU_TIMELINE=1, stderr) of one rank's tile of the N-GPU split, as a
synced call and as the last of `calls` back-to-back calls (the N-GPU bench's steps), with the
HIP-event time per call (diagnostic: where a small tile's per-call cost goes).
usage: python tools/tile_timeline.py [W] [spp] [N] [rank] [deal] [calls]"""
import json
import os
import sys

os.environ["YKGPU_TIMELINE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import image_height_for, make_params  # noqa: E402
from uecraytracing_amd.tiles import rank_tile  # noqa: E402

a = sys.argv[1:]
W = int(a[0]) if len(a) > 0 else 1920
spp = int(a[1]) if len(a) > 1 else 512
n = int(a[2]) if len(a) > 2 else 8
rank = int(a[3]) if len(a) > 3 else 0
deal = a[4] if len(a) > 4 else "cols"
calls = int(a[5]) if len(a) > 5 else 4
H = image_height_for(W)
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
ren = yk.Renderer(0)
ren.set_scene(arr, cam)
p = make_params(W, H, spp, 50, 404, flags=0, **(rank_tile(rank, n, H, W, deal) if n > 1 else {}))
buf = torch.empty((p.row_count, p.tile_width(), 3), dtype=torch.uint8, device="cuda:0")
stream = torch.cuda.Stream()
out = {"W": W, "spp": spp, "N": n, "rank": rank, "deal": deal}
for mode, k in (("warm", 1), ("synced", 1), ("back_to_back", calls)):
    print(f"---- {mode} x{k}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            ren.render_async(p, buf.data_ptr(), stream.cuda_stream)
        e1.record(stream)
    torch.cuda.synchronize()
    st = ren.stats()  # the last call's (prints its timeline)
    out[mode] = {"ms_per_call": round(e0.elapsed_time(e1) / k, 3), "last_call_ms": round(st["total_ms"], 3),
                 "render_busy_ms": round(st["render_busy_ms"], 3), "launches": st["launches"]}
print(json.dumps(out), flush=True)
