"""Several devices in one process (include/ykgpu.h ykgpu_group_*, ykgpu_render_devices) — on the
MI355X.  The one-GPU box runs the multi-device path with repeated entries ({0, 0, 0}: three
contexts on device 0, each rendering its dealt rows concurrently); the image must equal one
context's byte for byte (every row is independent, source.cpp:154-158), and the row dealing is
tiles.py's (tile row t → entry t mod k), checked per entry against the single render's rows.
"""
import numpy as np
import pytest

import golden_data
import refscenes
import uecraytracing_amd as yk
from uecraytracing_amd.records import make_params
from uecraytracing_amd.tiles import tile_image_rows

pytestmark = pytest.mark.gpu
MAN = golden_data.manifest()


@pytest.fixture(scope="module")
def single():
    r = yk.Renderer(0)
    yield r
    r.close()


def golden(name):
    return next(c for c in MAN["cases"] if c["name"] == name)


@pytest.mark.parametrize("entries", [1, 2, 3, 8])
def test_group_equals_the_reference_golden(entries):
    """ref4 200x112x8 (reference-generated golden) dealt over 1, 2, 3 and 8 contexts."""
    entry = golden("ref4_200x112x8_d50_s404")
    with yk.Group([0] * entries) as g:
        assert g.size() == entries
        g.set_scene(refscenes.ref4(), refscenes.reference_camera())
        rgb = g.render(make_params(200, 112, 8, 50, 404))
        np.testing.assert_array_equal(rgb, golden_data.rgb(entry))
        tot = g.stats(-1)
        assert tot["samples"] == 200 * 112 * 8
        per = [g.stats(e) for e in range(entries)]
        assert sum(s["samples"] for s in per) == tot["samples"]
        # entry e rendered tiles.py's rows of rank e of `entries`
        for e, s in enumerate(per):
            assert s["samples"] == len(tile_image_rows(e, entries, 112)) * 200 * 8
        assert tot["device_bytes"] >= sum(s["device_bytes"] for s in per) > 0
        assert tot["call_bytes"] >= sum(s["call_bytes"] for s in per) > 0


def test_group_final_scene_strided_rows_equal_single(single):
    """The headline scene at width 384, a strided row set (every 3rd row from 1) over 4 entries:
    the dealing composes with the caller's row set."""
    arr, cam = yk.read_scene(f"{yk.SCENE_DIR}/final_seed42.yks")
    single.set_scene(arr, cam)
    p = make_params(384, 216, 16, 50, 404, rows=(1, 70, 3))
    want = single.render(p)
    with yk.Group([0, 0, 0, 0]) as g:
        g.set_scene(arr, cam)
        got = g.render(p)
        np.testing.assert_array_equal(got, want)
        assert g.stats(-1)["launches"] >= 4


def test_group_keeps_the_column_set(single):
    """A column set (ABI 10) passes through the group: the entries deal its rows and render the
    same columns; the tile is row_count x col_count."""
    from uecraytracing_amd.tiles import tile_cols
    arr, cam = yk.read_scene(f"{yk.SCENE_DIR}/final_seed42.yks")
    single.set_scene(arr, cam)
    p = make_params(384, 216, 8, 50, 404, rows=(3, 60, 2), cols=tile_cols(2, 3, 384))
    want = single.render(p)
    assert want.shape == (60, 128, 3)
    with yk.Group([0, 0, 0]) as g:
        g.set_scene(arr, cam)
        np.testing.assert_array_equal(g.render(p), want)


def test_group_more_entries_than_rows(single):
    """Entries with no row (k > row_count) are skipped."""
    single.set_scene(refscenes.ref4(), refscenes.reference_camera())
    p = make_params(64, 36, 4, 50, 404, rows=(10, 3, 1))
    want = single.render(p)
    with yk.Group([0] * 5) as g:
        g.set_scene(refscenes.ref4(), refscenes.reference_camera())
        np.testing.assert_array_equal(g.render(p), want)
        assert g.stats(3)["samples"] == 0 and g.stats(4)["samples"] == 0


def test_group_rejects_banded_row_sets():
    with yk.Group([0, 0]) as g:
        g.set_scene(refscenes.ref4(), refscenes.reference_camera())
        with pytest.raises(yk.YkError, match="UNSUPPORTED"):
            g.render(make_params(64, 36, 2, 50, 404, rows=(0, 16, 2, 3)))
        with pytest.raises(yk.YkError, match="out of range"):
            g.stats(2)


def test_render_devices_one_call_equals_golden():
    entry = golden("ref4_32x18x6_d50_s404")
    sph, cam = golden_data.scene(entry)
    rgb = yk.render_devices([0, 0, 0], sph, cam, make_params(32, 18, 6, 50, 404))
    np.testing.assert_array_equal(rgb, golden_data.rgb(entry))


def test_group_repeated_calls_and_new_scene(single):
    """A group keeps its contexts: two scenes, two calls each, the same bytes as one context."""
    arr, cam = yk.build_scene("rtiow5", 0)
    single.set_scene(arr, cam)
    p = make_params(96, 54, 8, 50, 404)
    want = single.render(p)
    with yk.Group([0, 0, 0]) as g:
        g.set_scene(refscenes.ref4(), refscenes.reference_camera())
        g.render(p)
        g.set_scene(arr, cam)
        np.testing.assert_array_equal(g.render(p), want)
        np.testing.assert_array_equal(g.render(p), want)
