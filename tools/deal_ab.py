"""Every rank's tile of an N-way split under several dealings, timed as the contract loop times a
step (warm-up calls, a sync, K back-to-back calls; HIP events), two interleaved rounds: which
partition the N-GPU bench and the drop-in should deal.
deal: "cols" (8-column bands), "rows" (single rows), "rowsB" (rows in bands of 2^B).
usage: [K=8] [N=8] [W=1920] [SPP=512] python tools/deal_ab.py cols rows rows3"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import image_height_for, make_params  # noqa: E402
from uecraytracing_amd.tiles import rank_tile  # noqa: E402

K = int(os.environ.get("K", "8"))
N = int(os.environ.get("N", "8"))
W = int(os.environ.get("W", "1920"))
SPP = int(os.environ.get("SPP", "512"))
H = image_height_for(W)
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
ren = yk.Renderer(0)
ren.set_scene(arr, cam)
buf = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()


def call_ms(p):
    with torch.cuda.stream(s):
        for _ in range(2):
            ren.render_async(p, buf.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    with torch.cuda.stream(s):
        ev[0].record(s)
        for k in range(K):
            ren.render_async(p, buf.data_ptr(), s.cuda_stream)
            ev[k + 1].record(s)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[K]) / K, ev[1].elapsed_time(ev[K]) / max(1, K - 1)


for rnd in range(2):
    frame = call_ms(make_params(W, H, SPP, 50, 404, flags=0))
    print(json.dumps({"round": rnd, "deal": "frame", "ms": round(frame[0], 3), "in_flight_ms": round(frame[1], 3)}),
          flush=True)
    for deal in sys.argv[1:] or ["cols", "rows"]:
        band = int(deal[4:]) if deal.startswith("rows") and len(deal) > 4 else None
        ms = [call_ms(make_params(W, H, SPP, 50, 404, flags=0, **rank_tile(r, N, H, W, deal[:4], band)))
              for r in range(N)]
        tot, inf = [m[0] for m in ms], [m[1] for m in ms]
        print(json.dumps({"round": rnd, "deal": deal, "tile_ms": [round(x, 3) for x in tot],
                          "slowest_over_ideal": round(max(tot) / (frame[0] / N), 4),
                          "in_flight_ms": [round(x, 3) for x in inf],
                          "in_flight_slowest_over_ideal": round(max(inf) / (frame[1] / N), 4)}), flush=True)
