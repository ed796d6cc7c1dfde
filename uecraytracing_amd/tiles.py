"""Row tiling of one image across ranks (one process per GPU) and the gather to rank 0.

Every sample's random stream depends only on (y, x, s) (source.cpp:154-158) and every pixel is
independent, so any partition of the rows renders byte-identical pixels.  Rows are dealt
CYCLICALLY (row r → rank r mod N) so that cheap sky rows and expensive ground rows are spread
evenly; each rank's tile is a contiguous uint8[rows_max, W, 3] buffer in HBM (padded to the
largest tile so the collective moves equal-sized buffers), the tiles are gathered to rank 0
with one collective (RCCL over xGMI with backend 'nccl'; 'gloo' on CPU tensors in the tests),
and rank 0 de-interleaves them with one index_select.
"""
from __future__ import annotations


def tile_rows(rank: int, world: int, height: int):
    """(row_begin, row_count, row_stride) of rank's cyclic tile — the C-ABI's row set."""
    return rank, len(range(rank, height, world)), world


def rows_max(world: int, height: int) -> int:
    return -(-height // world)


def assembly_index(world: int, height: int, device=None):
    """Row r of the image is row r // world of rank r % world's (padded) tile."""
    import torch
    rm = rows_max(world, height)
    return torch.tensor([(r % world) * rm + r // world for r in range(height)], device=device)


class TileGather:
    """Gather of the per-rank tiles into the whole image on rank 0 (pre-allocated buffers, so
    the timed loop allocates nothing)."""

    def __init__(self, rank: int, world: int, height: int, width: int, device):
        import torch
        self.rank, self.world, self.height, self.width = rank, world, height, width
        self.rm = rows_max(world, height)
        self.tile = torch.zeros((self.rm, width, 3), dtype=torch.uint8, device=device)
        self.image = torch.empty((height, width, 3), dtype=torch.uint8, device=device)
        self.gathered = (torch.empty((world, self.rm, width, 3), dtype=torch.uint8, device=device)
                         if rank == 0 and world > 1 else None)
        self.index = assembly_index(world, height, device)

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
