"""The oracle is pinned to the REAL reference: byte-identical PPMs and the
exact TraceRay/ShadeRay call counts of the reference's gprof build, for every
fixture scene (tests/golden/golden.json, made by tools/make_goldens.py)."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from conftest import GOLD_DIR, SCENES, golden_names
from oracle_py import OracleScene, ppm_bytes, quantize

SMALL = golden_names(lambda v: v["width"] * v["height"] <= 300 * 300)
LARGE = golden_names(lambda v: v["width"] * v["height"] > 300 * 300)


def _check(name, golden):
    g = golden[name]
    sc = OracleScene(name, cwd=SCENES)
    assert sc.rc == 0, sc.msg
    assert (sc.width, sc.height) == (g["width"], g["height"])
    img, cnt = sc.render(threads=0)
    # byte-identical P3 output
    assert hashlib.md5(ppm_bytes(img)).hexdigest() == g["md5"]
    # one ray = one TraceRay call; shadow rays = lights x ShadeRay calls
    _, _, nl = sc.counts()
    rays = cnt["primary"] + cnt["shadow"] + cnt["refraction"] + cnt["reflection"]
    assert rays == g["trace_calls"]
    assert cnt["shadow"] == nl * g["shade_calls"]
    assert cnt["primary"] == g["width"] * g["height"]
    if "npz" in g:
        q = np.load(os.path.join(GOLD_DIR, g["npz"]))["q"]
        assert np.array_equal(quantize(img), q)


@pytest.mark.parametrize("name", SMALL)
def test_oracle_matches_reference_small(name, golden):
    _check(name, golden)


@pytest.mark.slow
@pytest.mark.parametrize("name", LARGE)
def test_oracle_matches_reference_full_size(name, golden):
    _check(name, golden)


def test_oracle_rows_subset_consistent():
    """Rendering a row subset gives exactly the same rows as a full render."""
    sc = OracleScene("test7_s.txt", cwd=SCENES)
    full, _ = sc.render()
    rows = [0, 5, 31, 63]
    part, cnt = sc.render(rows=rows)
    assert np.array_equal(np.nan_to_num(part, nan=-7), np.nan_to_num(full[rows], nan=-7))
    assert cnt["primary"] == len(rows) * sc.width
