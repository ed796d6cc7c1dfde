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
import os

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
    # launch buffers of kmax samples per pixel: 48 (FP64, 64-B records; synced schedule 4, 8, 16,
    # 20) and 64 (FP32, 48-B records; 4, 8, 16, 36): 3072 bytes of start records per pixel slot and
    # launch buffer in both, while the colour buffers' offsets differ
    ps = [make_params(96, 54, 48, 50, 404), make_params(96, 54, 64, 50, 404, precision=PRECISION_FP32)] * 3
    want = [ren.render(p) for p in ps[:2]] * 3
    st = ren.stats()
    assert st["launch_spp"] == 64 and st["launches"] == 4
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


_RETRY_CODE = r'''
import hashlib, json, os, sys
sys.path.insert(0, os.environ["YK_ROOT"])
import torch
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
out = {}
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for spp in (32, 40):  # synced 4, 8, 20 and 4, 8, 16, 12: launches up to 2048 slots per warm-up wave
        img = r.render(make_params(1920, 1080, spp, 50, 404))
        st = r.stats()
        out[str(spp)] = {"sha": hashlib.sha256(img.tobytes()).hexdigest(), "rows": img[[7, 1071]].tolist(),
                         "call_bytes": st["call_bytes"], "launches": st["launches"]}
print(json.dumps(out))
'''


def test_lens_retry_ring_fallbacks_are_bit_exact():
    """the deferred lens-retry warm-up's two fallbacks, forced by test builds of the
    library (uecraytracing_amd/csrc/Makefile TESTVARIANTS, -DYK_RETRY_CAP_FORCE): a ring of 64
    records per wave against ~440 expected rejections per wave at the frame's 2048 slots per
    warm-up wave, so it fills and the samples that find it full reach the render as kNoStart starts
    the render makes itself; and no ring (0), the in-line rejection loop a failed ring allocation
    falls back to.  The thin-lens final scene at 1920x1080: both images equal the product
    library's byte for byte and two rows equal the CPU oracle's; the ring's bytes show in
    call_bytes (product > 64-record ring > none)."""
    import json
    import os
    import subprocess
    import sys
    root = yk.LIB_DIR  # uecraytracing_amd/lib
    repo = os.path.dirname(os.path.dirname(root))
    res = {}
    for name, lib in (("product", os.path.join(root, "libykgpu.so")), ("retry64", os.path.join(root, "abl", "libykgpu_retry64.so")),
                      ("retry0", os.path.join(root, "abl", "libykgpu_retry0.so"))):
        assert os.path.exists(lib), f"{lib}: built by uecraytracing_amd/csrc/Makefile (all)"
        env = dict(os.environ, YKGPU_LIB_OVERRIDE=lib, YK_ROOT=repo)
        pr = subprocess.run([sys.executable, "-c", _RETRY_CODE], env=env, capture_output=True, text=True,
                            timeout=240)
        assert pr.returncode == 0, pr.stderr[-2000:]
        res[name] = json.loads([ln for ln in pr.stdout.splitlines() if ln.startswith("{")][-1])
    arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
    for spp in ("32", "40"):
        assert res["retry64"][spp]["sha"] == res["product"][spp]["sha"]
        assert res["retry0"][spp]["sha"] == res["product"][spp]["sha"]
        assert res["product"][spp]["call_bytes"] > res["retry64"][spp]["call_bytes"] > res["retry0"][spp]["call_bytes"]
    want, _, _, _ = oracle_lib.render(arr, cam, make_params(1920, 1080, 32, 50, 404, rows=(7, 2, 1064)))
    np.testing.assert_array_equal(np.array(res["retry64"]["32"]["rows"], dtype=np.uint8), want)


_STACK_CODE = r'''
import hashlib, json, os, sys
sys.path.insert(0, os.environ["YK_ROOT"])
import torch
import uecraytracing_amd as yk
from uecraytracing_amd.records import PRECISION_FP32, make_params
arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
out = {}
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for name, prec in (("fp64", 0), ("fp32", PRECISION_FP32)):
        p = make_params(192, 108, 16, 50, 404, flags=1, precision=prec)  # counting instance
        sums = r.render_sums(p)
        st = r.stats()
        out[name] = {"sha": hashlib.sha256(sums.tobytes()).hexdigest(), "linear_scans": st["linear_scans"],
                     "segments": st["segments"]}
print(json.dumps(out))
'''


def test_shallow_checked_stack_overflows_to_the_linear_scan():
    """The FP64 branch-free visit skips its stack check where the plan gives the stack its proven
    depth (3 x wide depth + 1 entries, KernelArgs::stack_check = 0: every headline launch).  The
    checked path — a scene whose LDS copy leaves less room — is forced by a test build
    (Makefile TESTVARIANTS, -DYK_STACK_CAP_FORCE=5: five checked entries for both trees): lanes
    whose traversal overflows the stack take the exact linear scan, so the float64 per-pixel sums
    equal the product library's bit for bit in FP64 and FP32, with linear scans counted only in
    the shallow build."""
    import json
    import subprocess
    import sys
    root = yk.LIB_DIR
    repo = os.path.dirname(os.path.dirname(root))
    res = {}
    for name, lib in (("product", os.path.join(root, "libykgpu.so")), ("stack5", os.path.join(root, "abl", "libykgpu_stack5.so"))):
        assert os.path.exists(lib), f"{lib}: built by uecraytracing_amd/csrc/Makefile (all)"
        env = dict(os.environ, YKGPU_LIB_OVERRIDE=lib, YK_ROOT=repo)
        pr = subprocess.run([sys.executable, "-c", _STACK_CODE], env=env, capture_output=True, text=True,
                            timeout=240)
        assert pr.returncode == 0, pr.stderr[-2000:]
        res[name] = json.loads([ln for ln in pr.stdout.splitlines() if ln.startswith("{")][-1])
    for prec in ("fp64", "fp32"):
        assert res["stack5"][prec]["sha"] == res["product"][prec]["sha"]
        assert res["stack5"][prec]["segments"] == res["product"][prec]["segments"]
        assert res["stack5"][prec]["linear_scans"] > res["product"][prec]["linear_scans"]
    assert res["product"]["fp64"]["linear_scans"] == 0


def test_two_and_three_launch_calls_back_to_back():
    """Calls of an 8-way column tile of 1920x1080 (259,200 pixels): in flight, 1024 spp is two
    launches of 512 spp and 1536 spp three (launches of ~2^27 slots), so both calls have
    rings of kmax = 512 — three start-record buffers and two colour buffers, deeper than a
    two-launch call — and every call reuses buffers of the calls before it (ctx->gev, run_len); a
    synced call spreads its samples over launches of ~2^26 slots inside the same rings.  Enqueued
    back to back in a mixed order, every image equals the synced render of its params, and two rows
    equal the CPU oracle's."""
    torch = pytest.importorskip("torch")
    from uecraytracing_amd.tiles import rank_tile
    arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
    with yk.Renderer(0) as r:
        r.set_scene(arr, cam)
        tk = rank_tile(3, 8, 1080, 1920, "cols")
        p2 = make_params(1920, 1080, 1024, 50, 404, **tk)
        p3 = make_params(1920, 1080, 1536, 50, 404, **tk)
        want = {1024: r.render(p2), 1536: r.render(p3)}
        st = r.stats()
        assert st["launch_spp"] == 512 and st["launches"] > 3  # synced: ~2^26-slot launches in rings of 512
        seq = [p2, p2, p3, p2, p3, p2, p3]
        outs = [torch.zeros((1080, p2.tile_width(), 3), dtype=torch.uint8, device="cuda:0") for _ in seq]
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        for p, o in zip(seq, outs):  # no synchronisation between the calls
            r.render_async(p, o.data_ptr(), s.cuda_stream)
        s.synchronize()
        st = r.stats()  # the last call's: in flight, three launches at kmax
        assert st["launches"] == 3 and st["launch_spp"] == 512
        for p, o in zip(seq, outs):
            np.testing.assert_array_equal(o.cpu().numpy(), want[p.samples_per_pixel])
    xs = [x for x in range(1920) if (x >> 3) % 8 == 3]
    cpu, _, _, _ = oracle_lib.render(arr, cam, make_params(1920, 1080, 1024, 50, 404, rows=(5, 2, 1070)), nthreads=16)
    np.testing.assert_array_equal(want[1024][[5, 1075]], cpu[:, xs])


def test_random_back_to_back_sequence_of_mixed_calls():
    """A seeded random sequence of calls enqueued back to back without synchronisation — whole
    frames and row / column tiles of 1920x1080 whose launches are 1, 2 or 3 per call
    (~2^26 slots synced, ~2^27 in flight), small single-launch calls, FP32 and xor128 calls between them — so
    calls of equal ring geometry overlap across calls of other geometries, of other launch counts
    and of other modes (launch(): ctx->gev, run_len).  Every output equals the synced render of its
    params."""
    torch = pytest.importorskip("torch")
    import random

    from uecraytracing_amd.tiles import rank_tile
    arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
    shapes = [
        make_params(1920, 1080, 64, 50, 404),                                   # 2 launches of 32
        make_params(1920, 1080, 96, 50, 404),                                   # 3 of 32 synced, 2 of 48 in flight
        make_params(1920, 1080, 512, 50, 404, **rank_tile(2, 8, 1080, 1920, "rows")),   # 2 of 256
        make_params(1920, 1080, 768, 50, 404, **rank_tile(2, 8, 1080, 1920, "rows")),   # 3 of 256 synced, 2 of 384 in flight
        make_params(1920, 1080, 256, 50, 404, **rank_tile(1, 4, 1080, 1920, "cols")),   # 2 of 128
        make_params(320, 180, 16, 50, 404),                                     # 1 launch
        make_params(320, 180, 16, 50, 404, precision=PRECISION_FP32),
        make_params(320, 180, 16, 50, 404, rng=RNG_XOR128),
    ]
    rnd = random.Random(6)
    seq = [rnd.randrange(len(shapes)) for _ in range(18)]
    with yk.Renderer(0) as r:
        r.set_scene(arr, cam)
        want = {k: r.render(shapes[k]) for k in sorted(set(seq))}
        outs = [torch.zeros((shapes[k].row_count, shapes[k].tile_width(), 3), dtype=torch.uint8, device="cuda:0")
                for k in seq]
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        for k, o in zip(seq, outs):
            r.render_async(shapes[k], o.data_ptr(), s.cuda_stream)
        s.synchronize()
        for k, o in zip(seq, outs):
            np.testing.assert_array_equal(o.cpu().numpy(), want[k])
