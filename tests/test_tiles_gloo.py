"""N>1 path on CPU: world_size-2 (and 3) gloo processes each render their row tile — bands of
rows dealt cyclically, and single rows — (the oracle stands in for the GPU here), gather to rank 0
through uecraytracing_amd.tiles — the same code bench.py runs over RCCL — and rank 0's image must
equal the single-process image.  The tiles are CPU tensors, so TileGather.gather takes its RCCL
branch's exact call — dist.gather(tile, list(gathered.unbind(0)), dst=0) then index_select — on
gloo; only the device of the buffers differs from bench.py's N-GPU run."""
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


def _worker(rank, world, port, W, H, spp, out_path, band_log2):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist

    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.tiles import TileGather, tile_rows

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rows = tile_rows(rank, world, H, band_log2)
    rgb, _, _, _ = oracle_lib.render(refscenes.mixed12(), refscenes.reference_camera(),
                                     make_params(W, H, spp, 50, 404, rows=rows), nthreads=2)
    tg = TileGather(rank, world, H, W, "cpu", band_log2)
    tg.tile[: rows[1]] = torch.from_numpy(rgb)
    img = tg.gather()
    if rank == 0:
        np.save(out_path, img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band_log2,W,H,spp", [(2, 3, 40, 23, 4), (3, 3, 40, 23, 4), (3, 1, 40, 23, 4),
                                                    (2, 0, 40, 23, 4),
                                                    # the driver's 8-GPU split of config 3's 1080 rows:
                                                    # 135-row tiles, assembly over 8 ranks
                                                    (8, 0, 12, 1080, 1)])
def test_cyclic_tiles_gather_to_the_full_image(tmp_path, world, band_log2, W, H, spp):
    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.tiles import rows_max
    if world == 8:
        assert rows_max(8, H, band_log2) == 135
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, spp, out, band_log2), nprocs=world, join=True)
    full, _, _, _ = oracle_lib.render(refscenes.mixed12(), refscenes.reference_camera(),
                                      make_params(W, H, spp, 50, 404))
    np.testing.assert_array_equal(np.load(out), full)


def _row_y(rb, rs, L, t):
    """include/ykgpu.h: tile row t of (row_begin, row_stride, row_band_log2)"""
    return rb + (((t >> L) * rs) << L) + (t & ((1 << L) - 1))


@pytest.mark.parametrize("band_log2", [0, 1, 3, 5])
def test_tile_rows_partition(band_log2):
    from uecraytracing_amd.tiles import assembly_index, rows_max, tile_image_rows, tile_rows
    for world in (1, 2, 3, 8):
        for H in (1, 9, 112, 450, 1080, 2160):
            rows = []
            for k in range(world):
                rb, rc, rs, L = tile_rows(k, world, H, band_log2)
                mine = [_row_y(rb, rs, L, t) for t in range(rc)]
                assert mine == tile_image_rows(k, world, H, band_log2)
                assert all(y < H for y in mine)
                rows += mine
            assert sorted(rows) == list(range(H))
            idx = assembly_index(world, H, band_log2=band_log2).tolist()
            assert len(set(idx)) == H and max(idx) < world * rows_max(world, H, band_log2)


def test_banded_tiles_are_balanced():
    """Bands of 8 rows dealt cyclically: every rank of an 8-GPU split of 1080 rows gets 16 or
    17 bands (max / mean rows <= 1.01)."""
    from uecraytracing_amd.tiles import tile_rows
    for world, H in ((2, 1080), (4, 1080), (8, 1080), (8, 2160)):
        counts = [tile_rows(k, world, H)[1] for k in range(world)]
        assert max(counts) / (H / world) <= 1.01, counts
