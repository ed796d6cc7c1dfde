"""Row tiling of one image across ranks (one process per GPU) and the gather to rank 0.

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
"""
from __future__ import annotations

BAND_LOG2 = 0


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


class TileGather:
    """Gather of the per-rank tiles into the whole image on rank 0 (pre-allocated buffers, so
    the timed loop allocates nothing)."""

    def __init__(self, rank: int, world: int, height: int, width: int, device, band_log2: int = BAND_LOG2):
        import torch
        self.rank, self.world, self.height, self.width = rank, world, height, width
        self.rm = rows_max(world, height, band_log2)
        self.tile = torch.zeros((self.rm, width, 3), dtype=torch.uint8, device=device)
        self.image = torch.empty((height, width, 3), dtype=torch.uint8, device=device)
        self.gathered = (torch.empty((world, self.rm, width, 3), dtype=torch.uint8, device=device)
                         if rank == 0 and world > 1 else None)
        self.index = assembly_index(world, height, device, band_log2)

    def gather(self):
        """Collective + de-interleave; after it, rank 0's self.image holds the whole image."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
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
            torch.index_select(self.gathered.reshape(self.world * self.rm, self.width, 3), 0,
                               self.index, out=self.image)
        return self.image
