"""Tiling of one image across ranks (one process per GPU) and the gather to rank 0.

Every sample's random stream depends only on (y, x, s) (source.cpp:154-158) and every pixel is
independent, so any partition of the rows renders byte-identical pixels.  Rows are dealt in
BANDS of 2^band_log2 consecutive rows, band b → rank b mod N: cyclic dealing spreads cheap sky
rows and expensive ground rows evenly.  The default is single rows (band_log2 = 0): with 8-row
bands rank r's rows sit 8r rows lower in every period, and on the final round-2 kernel the
slowest of 8 ranks took 29.2 ms against 27.5 ms with single rows, 101.2 against 97.6 ms at
2 ranks (profiles/r02bq_rank_tiles, profiles/r02br_rank_tiles; the per-sample cost of single
rows, 9-17% at round 1, no longer shows).  Each rank's tile is a
contiguous uint8[rows_max, W, 3] buffer in HBM (padded to the largest tile so the collective
moves equal-sized buffers), the tiles are gathered to rank 0 with one collective (RCCL over xGMI
with backend 'nccl'; 'gloo' on CPU tensors in the tests), and rank 0 de-interleaves them with one
index_select.

Single rows are the N-rank bench's default (DEAL = "rows", round 6: north_star's "row-tiled"),
and the drop-in's device group deals them too (ykgpu_group_render), so one partition ships.
Column dealing (rounds 4-5's default, `bench.py --deal cols`): every rank renders every row, and
the columns are dealt in bands of 2^COL_BAND_LOG2 = 8, band b → rank b mod N, so a rank's 8x8
processing blocks are 8x8 blocks of the image, where a row-dealt tile's blocks span every N-th
row.  Measured like the contract loop (profiles/r06_ab/tiles/r06e_deal8.txt), the
two are equal at 8 ranks within 0.4% (slowest tile 1.048-1.053 x frame/8 either way at K = 8);
8-row bands balance worse (1.083).  A column tile is uint8[H, cols_max, 3]; rank 0
de-interleaves the gathered tiles with one index_select over pixels.
"""
from __future__ import annotations

BAND_LOG2 = 0
COL_BAND_LOG2 = 3
DEAL = "rows"


def tile_rows(rank: int, world: int, height: int, band_log2: int = BAND_LOG2):
    """(row_begin, row_count, row_stride, row_band_log2) of rank's tile — the C-ABI's row set
    (include/ykgpu.h yk_render_params)."""
    B = 1 << band_log2
    count = sum(min(B, height - b * B) for b in range(rank, -(-height // B), world))
    return rank * B, count, world, band_log2


def tile_image_rows(rank: int, world: int, height: int, band_log2: int = BAND_LOG2):
    """Image row of each of rank's tile rows, in tile order."""
    B = 1 << band_log2
    return [y for b in range(rank, -(-height // B), world) for y in range(b * B, min((b + 1) * B, height))]


def rows_max(world: int, height: int, band_log2: int = BAND_LOG2) -> int:
    return max(tile_rows(r, world, height, band_log2)[1] for r in range(world))


def assembly_index(world: int, height: int, device=None, band_log2: int = BAND_LOG2):
    """Image row y is tile row (y's position in its rank's tile) of rank (y // B) % world's
    padded tile, stacked rank after rank."""
    import torch
    rm = rows_max(world, height, band_log2)
    idx = [0] * height
    for r in range(world):
        for t, y in enumerate(tile_image_rows(r, world, height, band_log2)):
            idx[y] = r * rm + t
    return torch.tensor(idx, device=device)


def tile_cols(rank: int, world: int, width: int, band_log2: int = COL_BAND_LOG2):
    """(col_begin, col_count, col_stride, col_band_log2) of rank's column set — the C-ABI's
    column set (include/ykgpu.h yk_render_params, ABI 10)."""
    return tile_rows(rank, world, width, band_log2)


def tile_image_cols(rank: int, world: int, width: int, band_log2: int = COL_BAND_LOG2):
    """Image column of each of rank's tile columns, in tile order."""
    return tile_image_rows(rank, world, width, band_log2)


def rank_tile(rank: int, world: int, height: int, width: int, deal: str = DEAL, band_log2: int | None = None) -> dict:
    """make_params keyword arguments (rows=, cols=) of rank's tile under `deal` ("rows" or
    "cols").  Every rank must get pixels: the C-ABI takes no empty row or column set (col_count
    0 means every column), so an image too small for the split — fewer than 8 x world columns
    dealt in 8-column bands, i.e. width <= 8 (world - 1), fewer than world rows — is refused here, naming the other dealing."""
    if deal == "rows":
        rows = tile_rows(rank, world, height, BAND_LOG2 if band_log2 is None else band_log2)
        if rows[1] == 0:
            raise ValueError(f"{height} rows cannot be dealt over {world} ranks (rank {rank} would get none)")
        return {"rows": rows}
    if deal == "cols":
        cols = tile_cols(rank, world, width, COL_BAND_LOG2 if band_log2 is None else band_log2) if world > 1 else None
        if cols is not None and cols[1] == 0:
            raise ValueError(f"{width} columns in {1 << COL_BAND_LOG2}-column bands cannot be dealt over {world} "
                             f"ranks (rank {rank} would get none; every rank needs at least one band: width > "
                             f"{(world - 1) << COL_BAND_LOG2} needed): deal rows instead")
        return {"rows": (0, height, 1, 0), "cols": cols}
    raise ValueError(f"deal must be 'rows' or 'cols', not {deal!r}")


def pixel_assembly_index(world: int, height: int, width: int, device=None,
                         band_log2: int = COL_BAND_LOG2):
    """Column dealing: image pixel (y, x) is pixel (y, j) of rank r = (x // C) % world's tile.  A
    rank's tile is height x its own width w_r, written contiguously (row pitch w_r, as the C-ABI
    writes it) at the start of its height x cols_max slot; the slots are stacked rank after rank.
    Flattened pixel indices."""
    import torch
    cm = rows_max(world, width, band_log2)
    rank_of, j_of, w_of = [0] * width, [0] * width, [0] * width
    for r in range(world):
        cols = tile_image_cols(r, world, width, band_log2)
        for j, x in enumerate(cols):
            rank_of[x], j_of[x], w_of[x] = r, j, len(cols)
    rank_of, j_of, w_of = (torch.tensor(v, dtype=torch.int64) for v in (rank_of, j_of, w_of))
    y = torch.arange(height, dtype=torch.int64)[:, None]
    idx = rank_of[None, :] * (height * cm) + y * w_of[None, :] + j_of[None, :]
    return idx.reshape(-1).to(device)


class TileGather:
    """Gather of the per-rank tiles into the whole image on rank 0 (pre-allocated buffers, so
    the timed loop allocates nothing)."""

    def __init__(self, rank: int, world: int, height: int, width: int, device, band_log2: int | None = None,
                 deal: str = "rows", collective: bool | None = None):
        """collective: run the collective and the de-interleave (default: world > 1; True at
        world 1 exercises the N-rank branch on one device, tests/test_gpu_tiles_rccl.py)."""
        import torch
        if deal not in ("rows", "cols"):
            raise ValueError(f"deal must be 'rows' or 'cols', not {deal!r}")
        if band_log2 is None:
            band_log2 = COL_BAND_LOG2 if deal == "cols" else BAND_LOG2
        self.rank, self.world, self.height, self.width = rank, world, height, width
        self.collective = world > 1 if collective is None else bool(collective)
        self.deal = deal if self.collective else "rows"
        if self.deal == "cols":  # tile: every row, cols_max columns (band_log2: the column bands);
            # the render writes its height x (own width) pixels contiguously from the start
            self.rm, self.cm = height, rows_max(world, width, band_log2)
        else:
            self.rm, self.cm = rows_max(world, height, band_log2), width
        self.tile = torch.zeros((self.rm, self.cm, 3), dtype=torch.uint8, device=device)
        self.image = torch.empty((height, width, 3), dtype=torch.uint8, device=device)
        self.gathered = (torch.empty((world, self.rm, self.cm, 3), dtype=torch.uint8, device=device)
                         if rank == 0 and self.collective else None)
        self.index = (pixel_assembly_index(world, height, width, device, band_log2) if self.deal == "cols"
                      else assembly_index(world, height, device, band_log2))

    def gather(self):
        """Collective + de-interleave; after it, rank 0's self.image holds the whole image."""
        import torch
        import torch.distributed as dist
        if not self.collective:
            self.image.copy_(self.tile[: self.height])
            return self.image
        if self.tile.is_cuda and dist.get_backend() == "gloo":
            # gloo gathers host tensors (test rehearsals of the N-rank path on one GPU)
            cpu = self.tile.cpu()
            outs = [torch.empty_like(cpu) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(cpu, outs, dst=0)
            if self.rank == 0:
                self.gathered.copy_(torch.stack(outs))
        else:
            dist.gather(self.tile, list(self.gathered.unbind(0)) if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            if self.deal == "cols":
                torch.index_select(self.gathered.reshape(-1, 3), 0, self.index,
                                   out=self.image.view(self.height * self.width, 3))
            else:
                torch.index_select(self.gathered.reshape(self.world * self.rm, self.width, 3), 0,
                                   self.index, out=self.image)
        return self.image
