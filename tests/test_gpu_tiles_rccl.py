"""The N-rank gather's device branch (uecraytracing_amd/tiles.py TileGather.gather: the RCCL
`dist.gather` of device tensors, then the de-interleave on the device) on the one-GPU box: a
world of one over the 'nccl' backend (RCCL; several ranks would need a GPU each), the tile
rendered by the C-ABI into the gather's own buffer under both dealings, with the collective
forced on.  The image must equal a direct render byte for byte.  (The N-rank logic itself —
several ranks, ragged tiles — is covered over gloo in tests/test_tiles_gloo.py.)"""
import socket

import numpy as np
import pytest

import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_gather_branch_on_the_device():
    torch = pytest.importorskip("torch")
    import torch.distributed as dist

    from uecraytracing_amd.tiles import TileGather, tile_cols
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        W, H = 200, 112
        with yk.Renderer(0) as r:
            r.set_scene(refscenes.mixed12(), refscenes.reference_camera())
            want = r.render(make_params(W, H, 8, 50, 404))
            stream = torch.cuda.Stream()
            for deal, kw in (("cols", {"cols": tile_cols(0, 1, W)}), ("rows", {"rows": (0, H, 1, 0)})):
                tg = TileGather(0, 1, H, W, torch.device("cuda", 0), deal=deal, collective=True)
                assert tg.gathered is not None and tg.gathered.is_cuda
                with torch.cuda.stream(stream):
                    r.render_async(make_params(W, H, 8, 50, 404, **kw), tg.tile.data_ptr(), stream.cuda_stream)
                    img = tg.gather()
                torch.cuda.synchronize()
                np.testing.assert_array_equal(img.cpu().numpy(), want)
    finally:
        dist.destroy_process_group()
