"""The documents a binder reads agree with the boundary: INTEGRATION.md's ABI
version and record sizes, and include/ykgpu.h's ABI version, against the ctypes mirrors
(uecraytracing_amd/records.py, whose sizes test_abi.py pins to the header's field layout) and the
library itself.  A drift of either document fails here."""
import ctypes
import os
import re

import uecraytracing_amd as yk
from uecraytracing_amd import records

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = open(os.path.join(ROOT, "INTEGRATION.md")).read()
HEADER = open(os.path.join(ROOT, "include", "ykgpu.h")).read()


def test_integration_abi_version_matches_the_library():
    versions = {int(v) for v in re.findall(r"ABI version (\d+)", DOC)}
    asserted = {int(v) for v in re.findall(r"ykgpu_abi_version\(\) == (\d+)", DOC)}
    (hdr,) = re.findall(r"#define YKGPU_ABI_VERSION (\d+)u", HEADER)
    lib = yk.load_library().ykgpu_abi_version()
    assert versions == asserted == {int(hdr)} == {lib} == {yk.ABI_VERSION}


def test_integration_record_sizes_match_the_ctypes_mirrors():
    table = dict((name, int(b)) for name, b in re.findall(r"^\| `(yk_\w+)` \| (\d+) \|$", DOC, re.M))
    mirrors = {"yk_sphere": records.Sphere, "yk_camera": records.Camera,
               "yk_render_params": records.RenderParams, "yk_render_stats": records.RenderStats}
    assert set(table) == set(mirrors)
    for name, cls in mirrors.items():
        assert table[name] == ctypes.sizeof(cls), name
        # and the header declares the record
        assert re.search(r"typedef struct %s \{" % name, HEADER), name


def test_integration_names_only_the_variables_the_library_reads():
    """The product library's getenv names (its .rodata) are exactly the two INTEGRATION §4
    documents for it: the A/B knobs exist only in -DYK_AB_KNOBS variant builds."""
    data = open(yk.LIB_PATH, "rb").read()
    names = {m.decode() for m in re.findall(rb"YKGPU_[A-Z0-9_]+", data)}
    assert names == {"YKGPU_OVERLAP", "YKGPU_TIMELINE"}, names
    rows = re.findall(r"^\| `(YKGPU_\w+)` \| the library \|", DOC, re.M)
    assert set(rows) == names
