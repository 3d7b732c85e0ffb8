"""The reference-side binding (integration/rt_hip_binding.cpp): what a
maintainer adds to the reference so that its own main (main.cpp:607) calls
this repo's C ABI.

  CPU: it compiles against the reference's own headers, read in place
       (-I/root/reference: src/definitions.h's Vector3 / Color / Mat3D /
       Globals), and INTEGRATION.md shows that file, not an excerpt;
  GPU: oracle/_ref/SimpleRayTracer_hip -- the reference's main.cpp with its
       seam replaced by the binding (oracle/Makefile ref-hip) -- writes the
       reference's PPMs (tests/test_gpu_parity.py::test_reference_main_with_hip_seam).
"""
from __future__ import annotations

import os
import re
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"
BINDING = os.path.join(ROOT, "integration", "rt_hip_binding.cpp")

needs_ref = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "main.cpp")),
                               reason="the reference's sources are not on this machine")


@needs_ref
def test_binding_compiles_against_reference_headers():
    r = subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", f"-I{REF}",
                        "-I" + os.path.join(ROOT, "include"), BINDING], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@needs_ref
def test_binding_replaces_the_seam(tmp_path):
    """Linked with the reference's own main.cpp (its definition weakened), the
    binary's create_view_window_and_ray_trace is the binding's: the strong
    symbol comes from rt_hip_binding.o and the reference's main calls it."""
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref-hip"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    exe = os.path.join(ROOT, "oracle", "_ref", "SimpleRayTracer_hip")
    nm = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    seam = [l for l in nm.splitlines() if l.endswith("_Z32create_view_window_and_ray_trace7Vector3S_S_fff5Color")]
    assert len(seam) == 1 and " T " in seam[0], seam
    binding = subprocess.run(["nm", os.path.join(ROOT, "oracle", "_ref", "rt_hip_binding.o")], capture_output=True,
                             text=True, check=True).stdout
    addr = seam[0].split()[0]
    assert "_Z32create_view_window_and_ray_trace7Vector3S_S_fff5Color" in binding
    dyn = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for sym in ("rt_scene_create", "rt_render_rows", "rt_scene_destroy", "rth_quantize"):
        assert sym in dyn, sym
    assert int(addr, 16) > 0


def test_integration_md_shows_the_binding_file():
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```cpp\n(.*?)```", md, flags=re.S)
    src = open(BINDING).read()
    assert any(b == src for b in blocks), "INTEGRATION.md's binding listing differs from integration/rt_hip_binding.cpp"
