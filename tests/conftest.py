"""Shared fixtures.  `-m "not gpu"` runs on CPU only; `-m gpu` needs an MI355X."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD_DIR = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLD_DIR, "scenes")
PKG = os.path.join(ROOT, "simple-raytracer_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _ensure_built():
    libs = [os.path.join(PKG, "lib", n) for n in ("librt_host.so", "librt_hip.so", "rt")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.run(["make", "-C", PKG, "-j4"], check=True, stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True,
                       stdout=subprocess.DEVNULL)


def _ensure_generated_scenes():
    """Seeded synthetic fixture scenes are regenerated (not committed: C5's
    is 10 MB) and must reproduce the exact text the goldens were made from."""
    import hashlib
    from rtamd import scenes as gen
    with open(os.path.join(GOLD_DIR, "golden.json")) as f:
        g = json.load(f)
    for name, ent in g.items():
        spec = ent.get("generated")
        if not spec:
            continue
        path = os.path.join(SCENES, name)
        if not os.path.exists(path):
            txt = gen.scene_text(spec["config"], w=spec["w"], h=spec["h"])
            with open(path, "w") as f:
                f.write(txt)
        with open(path, "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == spec["sha256"], f"generator drift: {name}"


def pytest_sessionstart(session):
    _ensure_built()
    _ensure_generated_scenes()


@pytest.fixture(scope="session")
def golden() -> dict:
    with open(os.path.join(GOLD_DIR, "golden.json")) as f:
        return json.load(f)


def golden_names(pred=None) -> list[str]:
    with open(os.path.join(GOLD_DIR, "golden.json")) as f:
        g = json.load(f)
    return sorted(k for k, v in g.items() if pred is None or pred(v))
