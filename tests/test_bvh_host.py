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
                                         (2000, 5, 0), (100000, 6, 0), (500, 7, 1), (5000, 8, 2), (900, 9, 3)])
def test_bvh_structure(checker, n, seed, mode):
    """Greedy and SAH-optimal collapses, binary16 node bounds (containment and
    one-step tightness), leaf records -- on random, coincident, collinear and
    geometrically spaced (deep) primitive sets."""
    r = subprocess.run([checker, str(n), str(seed), str(mode)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


def test_bvh_device_padding_stack(checker):
    """Mode 4 builds the device's tree (sphere padding of build_bvh, SAH
    collapse) from sphere centres on stdin and reports its worst-case stack:
    the deep-stack GPU test's scene gives a skewed tree."""
    import math
    lines = []
    for i in range(800):
        k, arm = i % 200, i // 200
        d, ang = 1.08 ** k, arm * math.pi / 2
        lines.append(f"{math.cos(ang) * d * 0.3} {math.sin(ang) * d * 0.3} {-(5 + d)} 0.4")
    r = subprocess.run([checker, "0", "0", "4"], input="\n".join(lines), capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.startswith("spheres=800"), r.stdout + r.stderr
    stack = int(r.stdout.split("stack=")[1].split()[0])
    assert stack >= 24, r.stdout


# Tree hashes (tools/bvh_bench.cpp: FNV-1a over the uploaded node, record,
# object-leaf and cone-tree arrays) of the seeded benchmark scenes with the
# 104-B binary16 device nodes: the round-3 builder's trees; the round-4
# builder (primitive array reordered in place, one-pass range statistics,
# sparse bins for small ranges, subtrees on threads, bitwise binary16
# rounding) builds the same trees.
BENCH_TREE_HASH = {104: {"C3": "d0d4c36f4057bc62", "C4": "5023c92e900cccd1", "C5": "0fa041b2ecb60269"}}


@pytest.fixture(scope="module")
def bvh_bench():
    pkg = os.path.join(ROOT, "simple-raytracer_amd")
    subprocess.run(["make", "-C", pkg, "bvh_bench"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(pkg, "lib", "bvh_bench")


@pytest.mark.parametrize("cfg", ["C3", "C4", "C5"])
def test_bvh_build_threads_identical(bvh_bench, tmp_path, cfg):
    """The host build on 4 threads gives the serial build's trees bit for bit,
    and both are the pinned trees of the seeded scene (no GPU)."""
    import json
    from rtamd import scenes as gen
    path = gen.write_scene(str(tmp_path), cfg)
    r = subprocess.run([bvh_bench, path, "4", "1"], capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    j = json.loads(r.stdout)
    assert j["identical"] and j["ok"] == 1, j
    assert j["hash"] == BENCH_TREE_HASH[j["node_bytes"]][cfg], j
