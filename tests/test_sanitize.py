"""SURVEY.md §5's sanitizer runs, on the CPU (no GPU): the host code that runs
threads -- the parser and the parallel P3 writers of librt_host
(tools/host_stress.cpp: an image of ~65 chunks of 32 768 pixels with every
kind of value the writer formats, written whole, in ragged row blocks and as
bytes, compared byte for byte), the threaded BVH build (tools/bvh_bench.cpp on
the 100 000-sphere C5 scene: the threaded tree must equal the serial one) and
the OpenMP oracle (oracle/rt_oracle.c, C3 and C5 at depth 8) -- built by
`make -C simple-raytracer_amd sanitize` with -fsanitize=thread (lib_tsan/) and
with -fsanitize=address,undefined (lib_asan/).  A report fails the test.
(The reference's own hot path is not thread-safe, main.cpp:1372-1376; these
builds check that this repo's threaded host code is.)"""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT, SCENES

PKG = os.path.join(ROOT, "simple-raytracer_amd")
ENV = {
    # archer (libomp's TSan tool) annotates the OpenMP synchronisation; the
    # runtime's own uninstrumented internals are ignored
    "tsan": {"TSAN_OPTIONS": "ignore_noninstrumented_modules=1 halt_on_error=1 exitcode=66"},
    # the OpenMP runtime keeps its per-thread state until exit (tools/lsan.supp)
    "asan": {"ASAN_OPTIONS": "detect_leaks=1 halt_on_error=1",
             "LSAN_OPTIONS": "suppressions=" + os.path.join(ROOT, "tools", "lsan.supp"),
             "UBSAN_OPTIONS": "print_stacktrace=1 halt_on_error=1"},
}


@pytest.fixture(scope="module")
def scenes(tmp_path_factory):
    from rtamd import scenes as gen
    d = tmp_path_factory.mktemp("san")
    return str(d), {c: gen.write_scene(str(d), c) for c in ("C3", "C5")}


@pytest.fixture(scope="module", params=["tsan", "asan"])
def san(request):
    subprocess.run(["make", "-C", PKG, f"san-{request.param}"], check=True, stdout=subprocess.DEVNULL,
                   timeout=600)
    return request.param, os.path.join(PKG, f"lib_{request.param}")


def _run(san, args, cwd):
    kind, _ = san
    env = dict(os.environ, **ENV[kind])
    r = subprocess.run(args, cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        (args, r.returncode, r.stdout[-2000:], r.stderr[-6000:])
    return r


def test_host_writers_and_parser(san, scenes, tmp_path):
    d, sc = scenes
    r = _run(san, [os.path.join(san[1], "host_stress"), sc["C3"], str(tmp_path), "8", "1536", "1400"], d)
    assert '"identical": true' in r.stdout


def test_threaded_bvh_build(san, scenes):
    import json
    d, sc = scenes
    r = _run(san, [os.path.join(san[1], "bvh_bench"), sc["C5"], "8", "1"], d)
    j = json.loads(r.stdout)
    assert j["identical"] and j["ok"] == 1 and j["threads"] > 1, j


@pytest.mark.parametrize("case", ["C3", "C5", "test7"])
def test_openmp_oracle(san, scenes, tmp_path, case):
    d, sc = scenes
    exe = os.path.join(san[1], "rt_oracle")
    if case == "test7":
        args, cwd = [exe, os.path.join(SCENES, "test7_s.txt"), "--threads", "8"], str(tmp_path)
        import shutil
        shutil.copy(os.path.join(SCENES, "test7_s.txt"), tmp_path)
        args[1] = str(tmp_path / "test7_s.txt")
    elif case == "C3":
        args, cwd = [exe, sc["C3"], "--imsize", "96", "96", "--threads", "8"], d
    else:
        args, cwd = [exe, sc["C5"], "--imsize", "16", "16", "--depth", "8", "--threads", "8"], d
    r = _run(san, args, cwd)
    assert "rays prim=" in r.stderr
