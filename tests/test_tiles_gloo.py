"""N>1 path on CPU: world_size-2 (and 3) gloo processes each render their cyclic row tile (the
oracle stands in for the GPU here), gather to rank 0 through uecraytracing_amd.tiles — the same
code bench.py runs over RCCL — and rank 0's image must equal the single-process image."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, spp, out_path):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist

    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.tiles import TileGather, tile_rows

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rows = tile_rows(rank, world, H)
    rgb, _, _, _ = oracle_lib.render(refscenes.mixed12(), refscenes.reference_camera(),
                                     make_params(W, H, spp, 50, 404, rows=rows), nthreads=2)
    tg = TileGather(rank, world, H, W, "cpu")
    tg.tile[: rows[1]] = torch.from_numpy(rgb)
    img = tg.gather()
    if rank == 0:
        np.save(out_path, img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_cyclic_tiles_gather_to_the_full_image(tmp_path, world):
    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    W, H, spp = 40, 23, 4
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, spp, out), nprocs=world, join=True)
    full, _, _, _ = oracle_lib.render(refscenes.mixed12(), refscenes.reference_camera(),
                                      make_params(W, H, spp, 50, 404))
    np.testing.assert_array_equal(np.load(out), full)


def test_tile_rows_partition():
    from uecraytracing_amd.tiles import assembly_index, rows_max, tile_rows
    for world in (1, 2, 3, 8):
        for H in (1, 9, 112, 1080, 2160):
            rows = [r for k in range(world) for r in range(*[tile_rows(k, world, H)[0], H, world])]
            assert sorted(rows) == list(range(H))
            assert sum(tile_rows(k, world, H)[1] for k in range(world)) == H
            idx = assembly_index(world, H).tolist()
            assert len(set(idx)) == H and max(idx) < world * rows_max(world, H)
