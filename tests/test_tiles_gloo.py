"""N>1 path on CPU: world_size-2 (and 3, 8) gloo processes each render their tile — bands of
columns dealt cyclically over every row (the bench's default), bands of rows, single rows — (the
oracle stands in for the GPU here), gather to rank 0
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


def _worker(rank, world, port, W, H, spp, out_path, band_log2, deal):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist

    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.tiles import TileGather, tile_cols, tile_rows

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    kw = ({"rows": tile_rows(rank, world, H, band_log2)} if deal == "rows" else
          {"rows": (0, H, 1, 0), "cols": tile_cols(rank, world, W, band_log2)})
    rgb, _, _, _ = oracle_lib.render(refscenes.mixed12(), refscenes.reference_camera(),
                                     make_params(W, H, spp, 50, 404, **kw), nthreads=2)
    tg = TileGather(rank, world, H, W, "cpu", band_log2, deal=deal)
    # as the C-ABI writes it: the tile's rows x its own width, contiguous from the buffer's start
    tg.tile.view(-1)[: rgb.size] = torch.from_numpy(rgb).reshape(-1)
    img = tg.gather()
    if rank == 0:
        np.save(out_path, img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band_log2,W,H,spp,deal", [
    (2, 3, 40, 23, 4, "rows"), (3, 3, 40, 23, 4, "rows"), (3, 1, 40, 23, 4, "rows"), (2, 0, 40, 23, 4, "rows"),
    # the driver's 8-GPU split of config 3's 1080 rows: 135-row tiles, assembly over 8 ranks
    (8, 0, 12, 1080, 1, "rows"),
    # column dealing (bench.py's default): 8-column bands, ragged widths (44 = 5.5 bands; 2 ranks
    # of 3 get 2 bands, one gets 1.5), single columns
    (2, 3, 40, 23, 4, "cols"), (3, 3, 44, 9, 2, "cols"), (3, 0, 40, 23, 4, "cols"),
    # the driver's 8-GPU split of config 3's 1920 columns: 240 columns (30 bands) per rank
    (8, 3, 1920, 3, 1, "cols")])
def test_cyclic_tiles_gather_to_the_full_image(tmp_path, world, band_log2, W, H, spp, deal):
    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.tiles import rows_max
    if world == 8:
        assert rows_max(8, H if deal == "rows" else W, band_log2) == (135 if deal == "rows" else 240)
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, spp, out, band_log2, deal), nprocs=world, join=True)
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


@pytest.mark.parametrize("band_log2", [0, 3])
def test_tile_cols_partition_and_pixel_assembly(band_log2):
    """Column sets (include/ykgpu.h ABI 10: tile column j → image column col_begin +
    (j / C) * col_stride * C + j % C) partition the width, and the pixel assembly index of the
    column dealing sends every image pixel to one distinct tile pixel."""
    from uecraytracing_amd.tiles import pixel_assembly_index, rows_max, tile_cols, tile_image_cols
    for world in (1, 2, 3, 8):
        for W in (1, 9, 44, 1920, 3840):
            cols = []
            for k in range(world):
                cb, cc, cs, L = tile_cols(k, world, W, band_log2)
                mine = [_row_y(cb, cs, L, j) for j in range(cc)]
                assert mine == tile_image_cols(k, world, W, band_log2)
                cols += mine
            assert sorted(cols) == list(range(W))
        H, W = 5, 44
        idx = pixel_assembly_index(world, H, W, band_log2=band_log2).tolist()
        cm = rows_max(world, W, band_log2)
        assert len(idx) == H * W and len(set(idx)) == H * W and max(idx) < world * H * cm
        for k in range(world):  # pixel (y, j) of rank k's tile (row pitch: its own width) lands at x
            mine = tile_image_cols(k, world, W, band_log2)
            for j, x in enumerate(mine):
                for y in range(H):
                    assert idx[y * W + x] == k * H * cm + y * len(mine) + j


def test_column_tiles_render_the_image_columns():
    """The oracle's column sets (the C-ABI's, include/ykgpu.h ABI 10) render the full image's own
    pixels: each rank's tile equals the full render's columns, for bands of 8 and single columns,
    and an invalid column set is rejected."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import make_params
    from uecraytracing_amd.tiles import tile_cols, tile_image_cols
    W, H, spp = 44, 9, 2
    sc, cam = refscenes.mixed12(), refscenes.reference_camera()
    full, _, _, _ = oracle_lib.render(sc, cam, make_params(W, H, spp, 50, 404), nthreads=4)
    for world, L in ((3, 3), (2, 0), (5, 1)):
        for k in range(world):
            rgb, _, _, _ = oracle_lib.render(sc, cam, make_params(W, H, spp, 50, 404, rows=(2, 3, 3),
                                                                  cols=tile_cols(k, world, W, L)), nthreads=4)
            np.testing.assert_array_equal(rgb, full[2::3][:, tile_image_cols(k, world, W, L)])
    for bad in ((40, 8, 1, 0), (0, 3, 0, 0), (0, 3, 1, 11)):
        with pytest.raises(RuntimeError):
            oracle_lib.render(sc, cam, make_params(W, H, spp, 50, 404, cols=bad))
    p = make_params(W, H, spp, 50, 404)
    p.col_stride = 1  # col_count == 0 (every column) with a stride set
    with pytest.raises(RuntimeError):
        oracle_lib.render(sc, cam, p)


def test_rank_tile_refuses_an_empty_tile():
    """with fewer than 8 x world columns (8-column bands) a rank would get an empty
    column set, which the C-ABI reads as 'every column' (col_count 0) and rejects; rank_tile says
    so up front, naming the row dealing, which still works for such an image."""
    from uecraytracing_amd.tiles import rank_tile
    with pytest.raises(ValueError, match="deal rows") as e:
        rank_tile(7, 8, 40, 56, "cols")
    assert "width > 56 needed" in str(e.value)  # the real bound, one band per rank
    # 57 columns over 8 ranks: the last rank's band is one column wide, every rank gets pixels
    assert rank_tile(7, 8, 40, 57, "cols")["cols"] == (56, 1, 8, 3)
    assert rank_tile(6, 8, 40, 56, "cols")["cols"] == (48, 8, 8, 3)
    assert rank_tile(7, 8, 40, 56, "rows")["rows"] == (7, 5, 8, 0)
    with pytest.raises(ValueError, match="rank 5 would get none"):
        rank_tile(5, 8, 5, 1920, "rows")
    assert rank_tile(0, 1, 9, 4, "cols") == {"rows": (0, 9, 1, 0), "cols": None}
