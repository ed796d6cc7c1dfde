"""Does the N-GPU step's RCCL gather get CUs while the next step's renders hold them?  

One process, a world of 1 over 'nccl' (RCCL), on the one-GPU box: rank 0's tile of the 8-way split
of config 3 rendered back to back K times, each step followed (as in bench.py) by a collective on
the bench stream — dist.gather of the tile, or all_gather — and the same loop without it.  The
renders' workgroups take one CU each with ~158 KB of LDS, and a back-to-back step's launches start
while the previous step's collective waits for its image, so a collective kernel that needs LDS or
registers the renders hold would wait for a CU to drain.  Prints ms per step for each variant,
and with the NCCL stream at high priority (ProcessGroupNCCL.Options.is_high_priority_stream).
usage: [K=20] [DEAL=rows] python tools/gather_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import image_height_for, make_params  # noqa: E402
from uecraytracing_amd.tiles import rank_tile  # noqa: E402

K = int(os.environ.get("K", "20"))
DEAL = os.environ.get("DEAL", "rows")
HIPRIO = os.environ.get("HIPRIO", "0") == "1"
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
torch.cuda.set_device(0)
opts = None
if HIPRIO:
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0), pg_options=opts)
W, spp = 1920, 512
H = image_height_for(W)
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
ren = yk.Renderer(0)
ren.set_scene(arr, cam)
p = make_params(W, H, spp, 50, 404, flags=0, **rank_tile(0, 8, H, W, DEAL))
tile = torch.zeros((p.row_count, p.tile_width(), 3), dtype=torch.uint8, device="cuda:0")
gathered = torch.zeros((1,) + tuple(tile.shape), dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()


def run(mode):
    def step():
        with torch.cuda.stream(s):
            ren.render_async(p, tile.data_ptr(), s.cuda_stream)
            if mode == "gather":
                dist.gather(tile, [gathered[0]], dst=0)
            elif mode == "all_gather":
                dist.all_gather_into_tensor(gathered, tile)
            elif mode == "copy":
                gathered[0].copy_(tile)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / K * 1e3


out = {"K": K, "deal": DEAL, "nccl_high_priority_stream": HIPRIO, "tile": list(tile.shape)}
for rnd in range(2):
    for mode in ("none", "copy", "gather", "all_gather"):
        out[f"{mode}_{rnd}"] = round(run(mode), 3)
print(json.dumps(out), flush=True)
dist.destroy_process_group()
