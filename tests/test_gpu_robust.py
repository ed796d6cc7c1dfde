"""Robustness of the C-ABI's call scheduling on the MI355X.

* Calls that overlap (cross-call pipelining) only when their rings and scratch have the
  same geometry: an FP64 call whose largest launch is 24 spp and an FP32 call whose largest is 32
  spp on the same tile have equal start-record buffers (24 x 64 B = 32 x 48 B per pixel slot) but
  different colour and scratch offsets, so they must not overlap; alternated back to back without
  synchronisation, every image equals its synced render.
* A call on another stream than the previous call's: the xor128 call's slot-counter and
  work-counter clears wait for the previous (mt19937) call's renders.
* A device short of memory makes a call slower, not fatal: with all but ~16 GB of HBM held by
  another allocation, BASELINE config 5's whole frame (1920x1080x4096, depth 200, ~69 GB of rings
  at full launch size) renders with smaller launches, bit-exact against the CPU oracle.
"""
import numpy as np
import pytest

import oracle_lib
import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import PRECISION_FP32, RNG_XOR128, make_params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ren():
    r = yk.Renderer(0)
    yield r
    r.close()


def test_alternating_precisions_with_colliding_start_buffers(ren):
    torch = pytest.importorskip("torch")
    ren.set_scene(refscenes.mixed12(), refscenes.reference_camera())
    # synced schedules 4, 8, 16, 24 (K = 24, FP64: 64-B records) and 4, 8, 16, 32 (K = 32, FP32:
    # 48-B records): 1536 bytes of start records per pixel slot and launch buffer in both
    ps = [make_params(96, 54, 52, 50, 404), make_params(96, 54, 60, 50, 404, precision=PRECISION_FP32)] * 3
    want = [ren.render(p) for p in ps[:2]] * 3
    st = ren.stats()
    assert st["launch_spp"] == 32 and st["launches"] == 4
    outs = [torch.zeros((p.row_count, p.tile_width(), 3), dtype=torch.uint8, device="cuda:0") for p in ps]
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    for p, o in zip(ps, outs):  # back to back, no synchronisation
        ren.render_async(p, o.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    for w, o in zip(want, outs):
        np.testing.assert_array_equal(o.cpu().numpy(), w)


def test_xor128_call_on_another_stream_after_an_mt19937_call(ren):
    torch = pytest.importorskip("torch")
    arr, cam = yk.build_scene("final", 42)
    ren.set_scene(arr, cam)
    pa = make_params(320, 180, 64, 50, 404)
    pb = make_params(320, 180, 16, 50, 404, rng=RNG_XOR128)
    wa, wb = ren.render(pa), ren.render(pb)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        a = torch.zeros((180, 320, 3), dtype=torch.uint8, device="cuda:0")
        b = torch.zeros_like(a)
        torch.cuda.synchronize()
        ren.render_async(pa, a.data_ptr(), s1.cuda_stream)  # still running when the next is enqueued
        ren.render_async(pb, b.data_ptr(), s2.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.cpu().numpy(), wa)
        np.testing.assert_array_equal(b.cpu().numpy(), wb)


def test_config5_frame_on_a_device_short_of_memory():
    torch = pytest.importorskip("torch")
    arr, cam = yk.build_scene("glass", 42)
    p = make_params(1920, 1080, 4096, 200, 404)
    free, _ = torch.cuda.mem_get_info(0)
    keep = 16 << 30
    if free < keep + (8 << 30):
        pytest.skip("device already short of memory")
    hog = torch.empty(free - keep, dtype=torch.uint8, device="cuda:0")
    try:
        with yk.Renderer(0) as r:
            r.set_scene(arr, cam)
            got = r.render_sums(p)
            st = r.stats()
    finally:
        del hog
        torch.cuda.empty_cache()
    assert st["mem_shrinks"] > 0 and st["launch_spp"] < 121  # 121: the unconstrained launch
    assert st["call_bytes"] < keep
    assert st["mt_fallbacks"] > 0
    rows = (500, 540)
    q = make_params(1920, 1080, 4096, 200, 404, rows=(rows[0], 2, rows[1] - rows[0]))
    _, want, _, _ = oracle_lib.render(arr, cam, q, nthreads=16, want_rgb=False, want_sums=True)
    assert got[list(rows)].tobytes() == want.tobytes()
