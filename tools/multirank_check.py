"""Rehearsal of the N-rank render + gather on whatever GPUs the box has (ranks may share one):
each rank renders its tile (tiles.DEAL: single rows; YK_DEAL=cols: 8-column bands) into device memory through the C-ABI, the tiles go to
rank 0 through uecraytracing_amd.tiles.TileGather, and rank 0 compares the assembled image with
a single-process render of the whole image.  Launch with torchrun; YK_BENCH_BACKEND=gloo when
ranks share a GPU (RCCL needs one GPU per rank).
usage: torchrun --nproc-per-node N tools/multirank_check.py [W] [spp]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import image_height_for, make_params  # noqa: E402
from uecraytracing_amd.tiles import DEAL, TileGather, rank_tile  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 320
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    H = image_height_for(W)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ.get("YK_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    arr, cam = yk.build_scene("final", 42)
    with yk.Renderer(local) as r:
        r.set_scene(arr, cam)
        deal = os.environ.get("YK_DEAL", DEAL)
        tg = TileGather(rank, world, H, W, dev, deal=deal)
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            r.render_async(make_params(W, H, spp, 50, 404, **rank_tile(rank, world, H, W, deal)),
                           tg.tile.data_ptr(), s.cuda_stream)
        s.synchronize()
        img = tg.gather()
        torch.cuda.synchronize()
        if rank == 0:
            full = r.render(make_params(W, H, spp, 50, 404))
            same = bool((img.cpu().numpy() == full).all())
            print(json.dumps({"world": world, "backend": backend, "deal": deal, "W": W, "H": H, "spp": spp,
                              "identical_to_single_render": same}), flush=True)
            if not same:
                sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
