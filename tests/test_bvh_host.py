"""Structural invariants of the host BVH builder (csrc/rt_bvh.h) -- CPU only.
A malformed tree would send the GPU traversal out of bounds, so the builder
is checked before any kernel sees it."""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bvh") / "bvh_check")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tools", "bvh_check.cpp"), "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("n,seed,mode", [(1, 1, 0), (2, 1, 0), (3, 2, 0), (17, 3, 0), (1000, 4, 0),
                                         (2000, 5, 0), (100000, 6, 0), (500, 7, 1), (5000, 8, 2)])
def test_bvh_structure(checker, n, seed, mode):
    r = subprocess.run([checker, str(n), str(seed), str(mode)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
