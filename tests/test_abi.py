"""The C ABIs load and export every function their headers declare."""
from __future__ import annotations

import ctypes as C
import os
import re

import pytest

import rtamd
from conftest import ROOT, PKG


def declared(header: str) -> list[str]:
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rth?_\w+)\s*\(", src, flags=re.M)))


@pytest.mark.parametrize("header,lib", [("rt_hip.h", "librt_hip.so"), ("rt_host.h", "librt_host.so")])
def test_exports(header, lib):
    names = declared(header)
    assert len(names) >= 8
    L = C.CDLL(os.path.join(PKG, "lib", lib))
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_bindings_cover_headers():
    assert set(declared("rt_hip.h")) == set(rtamd.HIP_SYMBOLS)
    assert set(declared("rt_host.h")) == set(rtamd.HOST_SYMBOLS)


def test_struct_sizes_match_c():
    # sizes from the C definitions in include/rt_hip.h
    assert C.sizeof(rtamd.rt_material) == 12 * 4
    assert C.sizeof(rtamd.rt_sphere_desc) == 4 * 4 + 48 + 4
    assert C.sizeof(rtamd.rt_face_desc) == (9 + 9 + 6) * 4 + 4 + 48 + 4
    assert C.sizeof(rtamd.rt_camera) == 48
    assert C.sizeof(rtamd.rt_stats) == 6 * 8 + 8 + 3 * 8 + 3 * 8 + 8


def test_strerror_without_device():
    L = rtamd.hip_lib()
    assert L.rt_strerror(0) == b"ok"
    assert L.rt_strerror(-2) == b"no such HIP device"
