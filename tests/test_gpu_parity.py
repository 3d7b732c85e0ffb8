"""HIP path vs the CPU oracle (and the reference's golden fixtures) on the
same scene files.  Needs an MI355X: `pytest -m gpu`."""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import rtamd
from conftest import GOLD_DIR, PKG, SCENES, golden_names
from oracle_py import OracleScene
from parity import assert_parity, compare, quantized_flips
from rtamd import scenes as gen

pytestmark = pytest.mark.gpu

RAYS = ("primary", "shadow", "refraction", "reflection")
_summary = {}


def _counts(st) -> dict:
    return {k: int(getattr(st, k)) for k in RAYS + ("skip_trans", "ub_back")}


@pytest.fixture(scope="module", autouse=True)
def _report():
    yield
    out = os.path.join(os.path.dirname(GOLD_DIR), "..", "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity_summary.json"), "w") as f:
        json.dump(_summary, f, indent=1, sort_keys=True)


@pytest.mark.parametrize("name", golden_names())
def test_scene_parity(name, golden):
    g = golden[name]
    img, st = rtamd.render_scene(name, cwd=SCENES)
    ref, cnt = OracleScene(name, cwd=SCENES).render()
    c = compare(img, ref)
    mine = _counts(st)
    _summary[name] = dict(c, gpu_counts=mine, oracle_counts=cnt)
    assert_parity(img, ref, name)
    # ray counts: exact against the oracle, whose total is pinned to the
    # reference's TraceRay call count (gprof)
    assert mine == cnt, (mine, cnt)
    assert sum(mine[k] for k in RAYS) == g["trace_calls"]
    if "npz" in g:
        # the reference's own 8-bit output: every differing value is a
        # rounding flip of a float within the tolerance of a level boundary
        q = np.load(os.path.join(GOLD_DIR, g["npz"]))["q"]
        _summary[name]["quantized"] = quantized_flips(img, rtamd.quantize(img), q, name)


@pytest.mark.parametrize("accel", [0, 1])
@pytest.mark.parametrize("name", golden_names(lambda v: v["width"] * v["height"] <= 300 * 300))
def test_scene_parity_forced_path(name, accel, golden):
    """Both search strategies on every small fixture: the brute-force scan
    (accel=0) and the BVH (accel=1, with its exact fallbacks), each against
    the oracle, with identical ray counts."""
    img, st = rtamd.render_scene(name, cwd=SCENES, options={"accel": accel})
    ref, cnt = OracleScene(name, cwd=SCENES).render()
    c = compare(img, ref)
    tag = "accel%d" % accel
    _summary[f"{name}@{tag}"] = dict(c, tests=dict(box=st.box_tests, face=st.face_tests,
                                                   sphere=st.sphere_tests))
    assert_parity(img, ref, f"{name} {tag}")
    assert _counts(st) == cnt


@pytest.mark.parametrize("accel", [0, 1])
@pytest.mark.parametrize("name", golden_names(lambda v: v["width"] * v["height"] <= 300 * 300))
def test_benched_instantiation_bit_identical(name, accel):
    """The kernel instantiation bench.py times (option counters = 0) renders
    every small fixture bit for bit like the counting one the parity tests pin
    to the oracle, on both search paths -- including the shortcuts only it
    takes (a known shadow ray's light step in the same shading step, round 6)."""
    a, st_a = rtamd.render_scene(name, cwd=SCENES, options={"accel": accel})
    b, st_b = rtamd.render_scene(name, cwd=SCENES, options={"accel": accel, "counters": 0})
    assert np.array_equal(np.nan_to_num(a, nan=-9), np.nan_to_num(b, nan=-9)), name
    assert st_b.rays() == 0 and st_a.rays() > 0


def test_strips_and_determinism():
    """Rendering rows in strips reproduces the full image bit for bit, and two
    renders are identical (no order dependence in the persistent scheduler)."""
    hs = rtamd.HostScene("test7_s.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    full, st = gs.render_rows(cam, W, H, 0, H)
    full2, st2 = gs.render_rows(cam, W, H, 0, H)
    parts = []
    tot = 0
    for y0, y1 in [(0, 7), (7, 40), (40, H)]:
        part, s = gs.render_rows(cam, W, H, y0, y1)
        parts.append(part)
        tot += s.rays()
    strip = np.concatenate(parts)
    eq = lambda a, b: np.array_equal(np.nan_to_num(a, nan=-9), np.nan_to_num(b, nan=-9))
    assert eq(full, full2) and st.rays() == st2.rays()
    assert eq(full, strip) and tot == st.rays()


@pytest.mark.parametrize("depth", [0, 1, 2, 6, 8])
def test_depth_knob(depth):
    """The reference hard-codes depth 4 (main.cpp:100); other depths are
    checked against the oracle at the same depth, which is pinned bit for bit
    to an instrumented reference build at these depths on these scenes
    (tests/test_float_goldens.py, tests/golden/ref_f/*@d<depth>)."""
    for name in ("test7_s.txt", "edge_nested_nobkgeta.txt", "C5_8x8.txt"):
        img, st = rtamd.render_scene(name, cwd=SCENES, depth=depth)
        o = OracleScene(name, cwd=SCENES)
        o.set_depth(depth)
        ref, cnt = o.render()
        assert_parity(img, ref, f"{name}@depth{depth}")
        assert _counts(st) == cnt


def test_c5_depth8_mini():
    """C5 (BASELINE depth 8) at 12x12 against the oracle; the same miniature
    is pinned to the instrumented reference (ref_f/C5_12x12@d8)."""
    txt = gen.scene_text("C5", w=12, h=12)
    p = os.path.join(SCENES, "_c5_d8.txt")
    open(p, "w").write(txt)
    try:
        img, st = rtamd.render_scene("_c5_d8.txt", cwd=SCENES, depth=8)
        o = OracleScene("_c5_d8.txt", cwd=SCENES)
        o.set_depth(8)
        ref, cnt = o.render()
    finally:
        os.remove(p)
    assert_parity(img, ref, "C5@12x12 depth 8")
    assert _counts(st) == cnt


def _benched_rows_vs_oracle(tmp_path, config: str, nrows: int, depth: int = 4, key: str | None = None,
                            dense_row: bool = False):
    """A BASELINE config at its full size, rendered whole into HBM by the
    kernel instantiation bench.py times (option counters = 0), compared on
    `nrows` rows spread over the image with the oracle; the same rows'
    pixels rendered again by the counting instantiation (rt_render_pixels)
    are bit for bit the timed image's, with exactly the oracle's per-type ray
    counts (main.cpp:718-764)."""
    torch = pytest.importorskip("torch")
    d = str(tmp_path)
    path = gen.write_scene(d, config)
    hs = rtamd.HostScene(path, cwd=d)
    hs.set_depth(depth)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    gs.set_option("counters", 0)
    img = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    gs.render_rows_async(cam, W, H, 0, H, img.data_ptr(), torch.cuda.current_stream().cuda_stream)
    gs.last_stats()
    torch.cuda.synchronize()
    assert gs.debug_counters()[48] == 0          # the uncounted (benched) instantiation ran
    rows = np.unique(np.linspace(0, H - 1, nrows).astype(np.int32))
    if dense_row:
        rows[0] = H // 3                     # the image's top rows are mostly sky: take a dense one too
        rows = np.unique(rows)
    got = img[rows.tolist()].cpu().numpy()
    del img
    o = OracleScene(path, cwd=d)
    o.set_depth(depth)
    ref, cnt = o.render(rows=rows)
    c = assert_parity(got, ref, f"{config} rows (counters=0)")
    gs.set_option("counters", 1)
    xs, ys = np.meshgrid(np.arange(W, dtype=np.int32), rows)
    xy = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)
    alone, st_px = gs.render_pixels(cam, W, H, xy)
    assert np.array_equal(np.nan_to_num(alone.reshape(got.shape), nan=-9), np.nan_to_num(got, nan=-9))
    assert _counts(st_px) == cnt, (_counts(st_px), cnt)
    gs.close()
    _summary[key or f"{config}_full_rows_counters0"] = dict(c, rows=len(rows), pixels=int(len(xy)), sample=cnt)
    return c, cnt


def test_c3_full_size_row_sample(tmp_path):
    """BASELINE config C3 at its full 4096x4096 (the bench's workload), by the
    benched instantiation: 256 rows (1 M pixels, ~7 M rays) against the
    oracle, exact per-type counts of those rows."""
    _, cnt = _benched_rows_vs_oracle(tmp_path, "C3", 256, key="C3_full_rows")
    assert cnt["refraction"] > 0 and cnt["reflection"] > 0


@pytest.mark.parametrize("config", ["C3G", "C3D"])
def test_c3_variants_full_size_row_sample(tmp_path, config):
    """C3G (glass triangles: SKIP_TRANS, main.cpp:1000-1002) and C3D (an
    unnormalised directional light against spheres, main.cpp:895) at
    4096x4096 by the benched instantiation: 64 rows against the oracle."""
    _, cnt = _benched_rows_vs_oracle(tmp_path, config, 64, key=f"{config}_full_rows")
    if config == "C3G":
        assert cnt["skip_trans"] > 0


def _render_on_device(path: str, cwd: str, depth: int):
    """Whole image rendered into HBM (torch buffer); -> (device image, stats,
    host scene, GPU scene, camera)."""
    torch = pytest.importorskip("torch")
    hs = rtamd.HostScene(path, cwd=cwd)
    hs.set_depth(depth)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    img = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    gs.render_rows_async(cam, W, H, 0, H, img.data_ptr(), torch.cuda.current_stream().cuda_stream)
    st = gs.last_stats()
    torch.cuda.synchronize()
    return img, st, hs, gs, cam


C4_ROWS, C4_PARTS = 64, 4             # C4's full-size sample: 64 rows, the oracle's work in 4 parts


@pytest.fixture(scope="module")
def c4_full(tmp_path_factory):
    """BASELINE config C4 at its full 8192x8192 rendered whole into HBM by the
    benched instantiation (counters = 0); C4_ROWS rows spread over the image
    (one of them dense) read out for the parts below."""
    torch = pytest.importorskip("torch")
    d = str(tmp_path_factory.mktemp("c4"))
    path = gen.write_scene(d, "C4")
    hs = rtamd.HostScene(path, cwd=d)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    gs.set_option("counters", 0)
    img = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    gs.render_rows_async(cam, W, H, 0, H, img.data_ptr(), torch.cuda.current_stream().cuda_stream)
    gs.last_stats()
    torch.cuda.synchronize()
    assert gs.debug_counters()[48] == 0          # the uncounted (benched) instantiation ran
    # the top rows are mostly sky: one dense row besides (H // 3 + 1: no
    # linspace row, so C4_ROWS + 1 rows in all)
    rows = np.unique(np.append(np.linspace(0, H - 1, C4_ROWS).astype(np.int32), H // 3 + 1)).astype(np.int32)
    assert len(rows) == C4_ROWS + 1
    got = img[rows.tolist()].cpu().numpy()
    del img
    gs.set_option("counters", 1)
    ctx = dict(W=W, H=H, gs=gs, cam=cam, rows=rows, got=got, o=OracleScene(path, cwd=d), parts={})
    yield ctx
    parts = ctx["parts"].values()
    _summary["C4_full_rows"] = dict(rows=int(sum(p["rows"] for p in parts)), pixels=int(sum(p["pixels"] for p in parts)),
                                    max_abs=max((p["max_abs"] for p in parts), default=None), parts=len(parts),
                                    sample={k: sum(p["sample"][k] for p in parts) for k in RAYS} if parts else {})
    gs.close()


@pytest.mark.parametrize("part", range(C4_PARTS))
def test_c4_full_size_row_sample(c4_full, part):
    """BASELINE config C4 at its full 8192x8192: 10 000 textured triangles with
    the real-size 2048x1024 synthetic texture, a directional and a point light
    (hard shadows), rendered by the benched instantiation (fixture c4_full).
    Part `part` of its 65 sample rows (532 480 pixels in all) against the
    oracle (on every CPU the lease grants: OMP_NUM_THREADS), and the same
    rows' pixels rendered again by the counting instantiation
    (rt_render_pixels): bit for bit the timed image's, with exactly the
    oracle's per-type ray counts (main.cpp:718-764)."""
    c = c4_full
    n = (len(c["rows"]) + C4_PARTS - 1) // C4_PARTS
    rows, got = c["rows"][part * n:(part + 1) * n], c["got"][part * n:(part + 1) * n]
    ref, cnt = c["o"].render(rows=rows)
    r = assert_parity(got, ref, f"C4 rows part {part} (counters=0)")
    xs, ys = np.meshgrid(np.arange(c["W"], dtype=np.int32), rows)
    xy = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)
    alone, st_px = c["gs"].render_pixels(c["cam"], c["W"], c["H"], xy)
    assert np.array_equal(np.nan_to_num(alone.reshape(got.shape), nan=-9), np.nan_to_num(got, nan=-9))
    assert _counts(st_px) == cnt, (_counts(st_px), cnt)
    assert cnt["shadow"] > 0
    c["parts"][part] = dict(r, rows=int(len(rows)), pixels=int(len(xy)), sample=cnt)


def test_c5_full_size_span_sample(tmp_path):
    """BASELINE config C5 at its full 16384x16384 with 100 000 spheres (depth 4,
    the reference's): 256-pixel spans on 64 rows spread over the image (16 384
    pixels) against the oracle (a full C5 row costs the oracle minutes).  The
    whole image is rendered on the GPU first; the spans are read out of HBM."""
    d = str(tmp_path)
    path = gen.write_scene(d, "C5")
    img, st, hs, gs, cam = _render_on_device(path, d, 4)
    W, H = hs.width, hs.height
    assert (W, H) == (16384, 16384) and st.primary == W * H
    xy = _span_sample(W, H, rows=64, span=256)
    got = img[xy[:, 1].tolist(), xy[:, 0].tolist()].cpu().numpy()
    del img
    ref, cnt = OracleScene(path, cwd=d).render_pixels(W, H, xy)
    c = assert_parity(got, ref, "C5 span sample")
    assert cnt["refraction"] + cnt["reflection"] > 0
    alone, st_px = gs.render_pixels(cam, W, H, xy)
    assert np.array_equal(np.nan_to_num(alone, nan=-9), np.nan_to_num(got, nan=-9))
    assert _counts(st_px) == cnt
    _summary["C5_full_spans"] = dict(c, pixels=len(xy), gpu_total=_counts(st), sample=cnt)
    gs.close()


def _span_sample(W: int, H: int, rows: int = 16, span: int = 64) -> np.ndarray:
    """`rows` rows spread over the image, a `span`-pixel run on each."""
    xy = []
    for k, r in enumerate(np.unique(np.linspace(0, H - 1, rows).astype(np.int64))):
        x0 = (k * 1637) % (W - span)
        xy += [(x0 + i, int(r)) for i in range(span)]
    return np.array(xy, dtype=np.int32)


def _ub_pixels(o: OracleScene, W: int, H: int, xy: np.ndarray) -> list:
    """Sample pixels whose shade tree takes back() on an empty medium stack
    (main.cpp:1028, undefined in the reference), one oracle call per pixel."""
    out = []
    for x, y in xy:
        _, c = o.render_pixels(W, H, np.array([[x, y]], dtype=np.int32), threads=1)
        if c["ub_back"]:
            out.append([int(x), int(y), c["ub_back"]])
    return out


C5D8_PARTS = 8                      # the depth-8 sample's oracle work in parts of 16 384 pixels


@pytest.fixture(scope="module")
def c5_depth8(tmp_path_factory):
    """BASELINE config C5 at its own setting: 16384x16384, 100 000 spheres,
    reflection + refraction at DEPTH 8 (3.8 G rays), rendered whole on the GPU
    into HBM once; the 131 072 sample pixels (512-pixel spans on 256 rows)
    and the pixels the kernel lists for back() of an empty medium stack are
    read out for the tests below."""
    d = str(tmp_path_factory.mktemp("c5d8"))
    path = gen.write_scene(d, "C5")
    img, st, hs, gs, cam = _render_on_device(path, d, 8)
    W, H = hs.width, hs.height
    assert (W, H) == (16384, 16384) and st.primary == W * H
    events, ubxy = gs.debug_ub_pixels()
    assert events == st.ub_back
    ub_px = np.unique(ubxy, axis=0).astype(np.int32) if len(ubxy) else np.zeros((0, 2), np.int32)
    xy = _span_sample(W, H, rows=256, span=512)
    got = img[xy[:, 1].tolist(), xy[:, 0].tolist()].cpu().numpy()
    got_ub = img[ub_px[:, 1].tolist(), ub_px[:, 0].tolist()].cpu().numpy() if len(ub_px) else None
    del img
    o = OracleScene(path, cwd=d)
    o.set_depth(8)
    ctx = dict(W=W, H=H, gs=gs, cam=cam, st=st, xy=xy, got=got, ub_px=ub_px, got_ub=got_ub, events=int(events),
               o=o, parts={})
    yield ctx
    tot = {k: sum(p["sample"][k] for p in ctx["parts"].values()) for k in RAYS + ("skip_trans", "ub_back")} \
        if ctx["parts"] else {}
    worst = max((p["max_abs"] for p in ctx["parts"].values()), default=None)
    _summary["C5_full_d8_spans"] = dict(pixels=int(sum(p["pixels"] for p in ctx["parts"].values())),
                                        parts=len(ctx["parts"]), max_abs=worst, gpu_total=_counts(st), sample=tot,
                                        ub_back=ctx.get("ub"))
    gs.close()


@pytest.mark.parametrize("part", range(C5D8_PARTS))
def test_c5_full_size_depth8_span_sample(c5_depth8, part):
    """C5 at depth 8, full size (fixture c5_depth8): part `part` of the
    131 072 sample pixels (16 384 each, so that no single test runs the
    oracle for minutes) against the oracle at depth 8 (pinned to the
    reference's own depth-8 floats by ref_f/C5_32x32@d8 and C5_12x12@d8).
    The same pixels rendered alone (rt_render_pixels) give bit for bit the
    whole image's colours and exactly the oracle's per-type ray counts."""
    c = c5_depth8
    n = len(c["xy"]) // C5D8_PARTS
    xy, got = c["xy"][part * n:(part + 1) * n], c["got"][part * n:(part + 1) * n]
    ref, cnt = c["o"].render_pixels(c["W"], c["H"], xy)
    r = assert_parity(got, ref, f"C5 depth 8 span sample part {part}")
    alone, st_px = c["gs"].render_pixels(c["cam"], c["W"], c["H"], xy)
    assert np.array_equal(np.nan_to_num(alone, nan=-9), np.nan_to_num(got, nan=-9))
    assert _counts(st_px) == cnt, (_counts(st_px), cnt)
    assert cnt["refraction"] > 0 and cnt["reflection"] > 0
    c["parts"][part] = dict(r, pixels=int(len(xy)), sample=cnt)


def test_c5_full_size_depth8_ub_pixels(c5_depth8):
    """Every pixel of the depth-8 C5 frame whose shade tree reads back() of an
    empty medium stack (main.cpp:1028: UB in the reference, defined here as
    eta_bkg like the oracle) is listed by the kernel
    (rt_scene_debug_ub_pixels) and compared with the oracle: agreement of two
    restatements, parity-unpinned against the reference itself."""
    c = c5_depth8
    ub = dict(events=c["events"], pixels=int(len(c["ub_px"])))
    if len(c["ub_px"]):
        ref_ub, cnt_ub = c["o"].render_pixels(c["W"], c["H"], c["ub_px"])
        ub["parity"] = assert_parity(c["got_ub"], ref_ub, "C5 depth 8 ub_back pixels")
        alone_ub, st_ub = c["gs"].render_pixels(c["cam"], c["W"], c["H"], c["ub_px"])
        assert np.array_equal(np.nan_to_num(alone_ub, nan=-9), np.nan_to_num(c["got_ub"], nan=-9))
        assert _counts(st_ub) == cnt_ub
        if c["events"] <= 4096:              # every event's pixel listed
            assert cnt_ub["ub_back"] == c["events"]
        ub["xy"] = c["ub_px"].tolist()
    c["ub"] = ub


def test_c2_full_size_whole_image(tmp_path):
    """BASELINE config C2 at its full 1024x1024 (100 spheres, 2 point lights,
    no reflection / refraction): every pixel against the oracle, exact
    per-type ray counts."""
    d = str(tmp_path)
    path = gen.write_scene(d, "C2")
    img, st = rtamd.render_scene(path, cwd=d)
    assert img.shape == (1024, 1024, 3)
    ref, cnt = OracleScene(path, cwd=d).render()
    c = assert_parity(img, ref, "C2 1024x1024")
    assert _counts(st) == cnt
    _summary["C2_full"] = dict(c, rays=cnt)


def test_render_pixels_bit_identical():
    """rt_render_pixels: listed pixels (any order, repeats, the image corners)
    get bit for bit the whole-image render's colours, and the rays of the
    list alone -- equal to the oracle's on the same pixels."""
    for name, depth in (("test7_s.txt", 4), ("C3_64x64.txt", 4), ("C5_8x8.txt", 8)):
        hs = rtamd.HostScene(name, cwd=SCENES)
        hs.set_depth(depth)
        W, H = hs.width, hs.height
        cam = hs.camera()
        gs = rtamd.GpuScene(hs)
        full, _ = gs.render_rows(cam, W, H, 0, H)
        rng = np.random.default_rng(5)
        xy = np.stack([rng.integers(0, W, 300), rng.integers(0, H, 300)], axis=1).astype(np.int32)
        xy = np.concatenate([xy, [[0, 0], [W - 1, H - 1], [0, H - 1], [W - 1, 0], [3, 2], [3, 2]]]).astype(np.int32)
        px, st = gs.render_pixels(cam, W, H, xy)
        want = full[xy[:, 1], xy[:, 0]]
        assert np.array_equal(np.nan_to_num(px, nan=-9), np.nan_to_num(want, nan=-9)), name
        o = OracleScene(name, cwd=SCENES)
        o.set_depth(depth)
        _, cnt = o.render_pixels(W, H, xy)
        assert _counts(st) == cnt, name
        with pytest.raises(rtamd.RTError):
            gs.render_pixels(cam, W, H, np.array([[W, 0]], dtype=np.int32))
        gs.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_row_blocks_reassemble(world):
    """The multi-GPU row sets (rtamd/dist.py) rendered one after another on one
    device and reassembled equal the single-call render bit for bit."""
    torch = pytest.importorskip("torch")
    from rtamd.dist import image_rows, row_set
    hs = rtamd.HostScene("test7_s.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    full, st = gs.render_rows(cam, W, H, 0, H)
    img = np.zeros_like(full)
    rays = 0
    for r in range(world):
        y0, b, step, n, per = row_set(H, world, r)
        buf = torch.zeros((per, W, 3), dtype=torch.float32, device="cuda:0")
        gs.render_row_blocks_async(cam, W, H, y0, b, step, n, buf.data_ptr())
        rays += gs.last_stats().rays()
        img[image_rows(H, world, r)] = buf[:n].cpu().numpy()
    assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(full, nan=-9))
    assert rays == st.rays()
    # the synchronous entry point into host memory (the CLI's multi-device path)
    img2 = np.zeros_like(full)
    rays = 0
    for r in range(world):
        y0, b, step, n, per = row_set(H, world, r)
        part, s = gs.render_row_blocks(cam, W, H, y0, b, step, n)
        rays += s.rays()
        img2[image_rows(H, world, r)] = part
    assert np.array_equal(np.nan_to_num(img2, nan=-9), np.nan_to_num(full, nan=-9))
    assert rays == st.rays()


def test_render_into_device_memory():
    torch = pytest.importorskip("torch")
    hs = rtamd.HostScene("four_spheres_s.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    host, st = gs.render_rows(cam, W, H, 0, H)
    dev = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    gs.render_rows_async(cam, W, H, 0, H, dev.data_ptr(), torch.cuda.current_stream().cuda_stream)
    st2 = gs.last_stats()
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)
    assert st2.rays() == st.rays() and st2.kernel_ms > 0


def test_prepare_then_render():
    """rt_scene_prepare builds the BVH and sizes the slots' buffers without
    rendering; renders after it are unchanged."""
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    ref, st = rtamd.GpuScene(hs).render_rows(cam, W, H, 0, H)
    gs = rtamd.GpuScene(hs)
    gs.set_option("inflight", 2)
    gs.prepare(cam, W, H)
    gs.prepare(cam, W, H)                     # idempotent
    img, st2 = gs.render_rows(cam, W, H, 0, H)
    assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9))
    assert _counts(st2) == _counts(st)
    with pytest.raises(rtamd.RTError):
        gs.prepare(cam, 0, H)                 # (1 x H is a valid image: the seam's NaN camera)


@pytest.mark.parametrize("inflight,share", [(2, -1), (3, -1), (2, 1), (3, 4)])
def test_frames_in_flight(inflight, share):
    """Option "inflight": renders issued on different caller streams run on the
    scene's render slots and overlap (each on the grid share "frame_share"
    gives it: auto = half the occupancy grid).  Every frame equals the
    one-at-a-time render bit for bit, its counters are its own, and work queued
    on a caller stream after a render sees the finished image."""
    torch = pytest.importorskip("torch")
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    hs.set_depth(4)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    ref, st = gs.render_rows(cam, W, H, 0, H)
    gs.set_option("inflight", inflight)
    gs.set_option("frame_share", share)
    streams = [torch.cuda.Stream() for _ in range(inflight)]
    frames = 2 * inflight + 1
    outs = [torch.full((H, W, 3), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(frames)]
    sums = []
    for k in range(frames):
        s = streams[k % inflight]
        with torch.cuda.stream(s):
            gs.render_rows_async(cam, W, H, 0, H, outs[k].data_ptr(), s.cuda_stream)
            sums.append(torch.nan_to_num(outs[k], nan=0.0).sum())   # ordered after the render
    st2 = gs.last_stats()
    torch.cuda.synchronize()
    want = float(np.nan_to_num(ref, nan=0.0).astype(np.float64).sum())
    for k in range(frames):
        assert np.array_equal(np.nan_to_num(outs[k].cpu().numpy(), nan=-9), np.nan_to_num(ref, nan=-9)), k
        assert abs(float(sums[k]) - want) <= 1e-3 * max(1.0, abs(want)), k
    assert _counts(st2) == _counts(st)
    assert 0 < st2.kernel_ms < 1000
    gs.set_option("inflight", 1)
    img, _ = gs.render_rows(cam, W, H, 0, H)
    assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9))
    with pytest.raises(rtamd.RTError):
        gs.set_option("inflight", 9)
    for bad in (0, 9, -2):
        with pytest.raises(rtamd.RTError):
            gs.set_option("frame_share", bad)


def test_frame_share_grid_policy():
    """Option frame_share's automatic rule (rt_scene.cpp launch_one): with
    frames in flight, a render of at most 32 pixels per lane of the
    occupancy-sized grid -- a rank's rows at N >= 2 -- runs on half the grid;
    a single render in flight, a whole 4096 x 4096 frame (51 per lane), an
    explicit frame_share 1 and an explicit grid keep theirs.  The image never
    changes."""
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    hs.set_depth(4)

    def grid_of(W, H, **opts):
        hs.set_imsize(W, H)
        cam = hs.camera(W, H)
        gs = rtamd.GpuScene(hs)
        gs.set_option("counters", 0)
        for k, v in opts.items():
            gs.set_option(k, v)
        img, _ = gs.render_rows(cam, W, H, 0, H)
        dbg = gs.debug_counters()
        gs.close()
        return int(dbg[18]), int(dbg[17]) * int(dbg[23]), img
    g1, full, ref = grid_of(1024, 512)                       # 0.5 M pixels, one render in flight
    assert g1 == full
    g2, _, img = grid_of(1024, 512, inflight=2)
    assert g2 == full // 2, (g2, full)
    assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9))
    assert grid_of(1024, 512, inflight=2, frame_share=1)[0] == full
    assert grid_of(1024, 512, inflight=2, frame_share=4)[0] == full // 4
    assert grid_of(1024, 512, inflight=2, grid=100)[0] == 100
    assert grid_of(4096, 4096, inflight=2)[0] == full       # 51 pixels per lane: the whole grid
    _summary["frame_share_grids"] = dict(full=full, share2=g2)


def test_abi_errors():
    L = rtamd.hip_lib()
    import ctypes as C
    hs = rtamd.HostScene("four_spheres_s.txt", cwd=SCENES)
    h = C.c_void_p()
    assert L.rt_scene_create(10_000, hs.desc, C.byref(h)) == -2
    assert L.rt_scene_create(0, None, C.byref(h)) == -1
    gs = rtamd.GpuScene(hs)
    cam = hs.camera()
    buf = np.zeros((4, 64, 3), np.float32)
    st = rtamd.rt_stats()
    assert L.rt_render_rows(gs._h, C.byref(cam), 64, 64, 5, 5, C.c_void_p(buf.ctypes.data), C.byref(st)) == -1
    assert L.rt_render_rows(gs._h, C.byref(cam), 64, 64, 60, 65, C.c_void_p(buf.ctypes.data), C.byref(st)) == -1
    assert L.rt_render_rows(gs._h, C.byref(cam), 0, 64, 0, 1, C.c_void_p(buf.ctypes.data), C.byref(st)) == -1
    hs.set_depth(40)
    with pytest.raises(rtamd.RTError):
        g2 = rtamd.GpuScene(hs)
        g2.render_rows(cam, 64, 64, 0, 4)


CLI = os.path.join(PKG, "lib", "rt")


@pytest.mark.parametrize("name", ["four_spheres.txt", "Test1.txt", "test7.txt", "earth.txt", "house.txt",
                                  "edge_glass_faces.txt"])
def test_cli_drop_in(name, golden, tmp_path):
    """`rt scene.txt` writes <scene>.ppm in the reference's exact P3 format.
    Its values are compared with the reference's PPM (the oracle's
    quantisation, which tests/test_oracle.py pins md5-identical to the
    reference's file): the md5 is equal, or every differing 8-bit value is a
    rounding flip of a float within 1e-4 of a level boundary -- counted in the
    summary (gpurun_out/parity_summary.json, key cli_<scene>)."""
    # run inside the scenes dir (textures are CWD-relative, like the reference)
    tmp_name = "_cli_" + name
    shutil.copy(os.path.join(SCENES, name), os.path.join(SCENES, tmp_name))
    out = os.path.join(SCENES, tmp_name[:-4] + ".ppm")
    fout = str(tmp_path / "f.bin")
    try:
        r = subprocess.run([CLI, tmp_name, "--float-out", fout], cwd=SCENES, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr
        data = open(out, "rb").read()
    finally:
        for p in (os.path.join(SCENES, tmp_name), out):
            if os.path.exists(p):
                os.remove(p)
    g = golden[name]
    W, H = g["width"], g["height"]
    md5 = hashlib.md5(data).hexdigest()
    toks = data.split()
    assert toks[:4] == [b"P3", str(W).encode(), str(H).encode(), b"255"]
    mine = np.array([int(t) for t in toks[4:]], dtype=np.uint64).view(np.int64).reshape(H, W, 3)
    f = np.fromfile(fout, dtype=np.float32).reshape(H, W, 3)
    assert np.array_equal(mine, rtamd.quantize(f))          # the PPM is the float buffer's quantisation
    ref, _ = OracleScene(name, cwd=SCENES).render()
    rec = dict(md5_equal=md5 == g["md5"], float_parity=compare(f, ref))
    rec.update(quantized_flips(f, mine, rtamd.quantize(ref), "cli " + name))
    _summary["cli_" + name] = rec
    assert_parity(f, ref, "cli " + name)
    assert (md5 == g["md5"]) == (rec["flipped"] == 0)


SEAM_EXE = os.path.join(os.path.dirname(PKG), "oracle", "_ref", "SimpleRayTracer_hip")


@pytest.mark.parametrize("name", ["four_spheres.txt", "Test1.txt", "test7.txt", "earth.txt", "house.txt",
                                  "edge_glass_faces.txt"])
def test_reference_main_with_hip_seam(name, golden):
    """The reference's OWN main.cpp (its parser, texture reader and P3 writer)
    with the seam main.cpp:607 routed through integration/rt_hip_binding.cpp
    into librt_hip.so (oracle/Makefile ref-hip).  Its PPM equals the
    reference's: md5-identical, or every differing 8-bit value a counted
    rounding flip of a float within 1e-4 of a level boundary (as for the
    drop-in CLI).  Built in the build container from /root/reference; the
    binary travels in oracle/_ref/."""
    if not os.path.exists(SEAM_EXE):
        pytest.skip("oracle/_ref/SimpleRayTracer_hip not built (needs /root/reference at build time)")
    tmp_name = "_seam_" + name
    shutil.copy(os.path.join(SCENES, name), os.path.join(SCENES, tmp_name))
    out = os.path.join(SCENES, tmp_name[:-4] + ".ppm")
    try:
        env = dict(os.environ, RT_HIP_SEAM_STATS="1")
        r = subprocess.run([SEAM_EXE, tmp_name], cwd=SCENES, capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        data = open(out, "rb").read()
    finally:
        for p in (os.path.join(SCENES, tmp_name), out):
            if os.path.exists(p):
                os.remove(p)
    g = golden[name]
    W, H = g["width"], g["height"]
    # the binding itself says it ran (the reference's own CPU definition of
    # the seam would write the same PPM): its GPU ray counts are the
    # reference's TraceRay calls (gprof counts in the golden)
    marks = [l for l in r.stderr.splitlines() if l.startswith("rt_hip seam: ")]
    assert len(marks) == 1, r.stderr
    f = marks[0].split()
    assert f[2] == f"{W}x{H}", marks[0]
    rays = {f[k]: int(f[k + 1]) for k in range(4, 12, 2)}
    assert rays["primary"] == W * H and sum(rays.values()) == g["trace_calls"], (marks[0], g["trace_calls"])
    toks = data.split()
    assert toks[:4] == [b"P3", str(W).encode(), str(H).encode(), b"255"]
    mine = np.array([int(t) for t in toks[4:]], dtype=np.uint64).view(np.int64).reshape(H, W, 3)
    ref, _ = OracleScene(name, cwd=SCENES).render()
    md5 = hashlib.md5(data).hexdigest()
    rec = dict(md5_equal=md5 == g["md5"])
    # the binary writes only 8-bit values: a flip is checked against the
    # oracle's float, which lies within 255 * 1e-4 of the level boundary
    # whenever a float within 1e-4 of it quantises to the other level
    rec.update(quantized_flips(ref, mine, rtamd.quantize(ref), "seam " + name))
    _summary["seam_" + name] = rec
    assert (md5 == g["md5"]) == (rec["flipped"] == 0)


def _render_both(name, cwd, W=None, H=None, accel=None):
    opts = None if accel is None else {"accel": accel}
    img, st = rtamd.render_scene(name, cwd=cwd, imsize=(W, H) if W else None, options=opts)
    ref, cnt = OracleScene(name, cwd=cwd).render(W, H)
    return img, st, ref, cnt


@pytest.mark.parametrize("W,H", [(2, 2), (3, 5), (67, 13), (130, 9), (9, 130)])
@pytest.mark.parametrize("name,accel", [("Test1.txt", None), ("test7.txt", None), ("_c3_ragged.txt", 1)])
def test_ragged_image_sizes(name, accel, W, H, tmp_path):
    """Image sizes that are not multiples of the 8x8 pixel tile (partial
    tiles, a partial last wave, one-tile-wide images), against the oracle
    with identical ray counts.  `_c3_ragged` is a C3-style scene (2000
    objects, reflection + refraction) through the BVH."""
    cwd = SCENES
    if name.startswith("_"):
        cwd = str(tmp_path)
        open(os.path.join(cwd, name), "w").write(gen.scene_text("C3", w=W, h=H))
    img, st, ref, cnt = _render_both(name, cwd, W, H, accel)
    assert img.shape == (H, W, 3)
    assert_parity(img, ref, f"{name}@{W}x{H}")
    assert _counts(st) == cnt


_HEADER = ("imsize 33 17\neye 0 0 0\nviewdir 0 0 -1\nupdir 0 1 0\nhfov 60\n"
           "bkgcolor 0.1 0.2 0.3 1\nlight -10 10 0 1 0.6 0.6 0.6\n")


@pytest.mark.parametrize("body,kind", [
    ("", "empty"),                                            # no objects: background only
    ("mtlcolor 1 0 0 1 1 1 0.2 0.6 0.5 20 0.3 1.5\n"          # a single glass sphere
     "sphere 0 0 -5 1\n", "one_sphere"),
    ("mtlcolor 0 1 0 1 1 1 0.2 0.6 0.5 20\n"                  # faces only (no spheres)
     "v -1 -1 -4\nv 1 -1 -4\nv 0 1 -5\nv 2 1 -6\nf 1 2 3\nf 2 4 3\n", "faces_only"),
])
@pytest.mark.parametrize("accel", [0, 1])
def test_degenerate_scenes(body, kind, accel, tmp_path):
    """Scenes at the edges of the object counts: nothing to hit, one object,
    faces without spheres -- both search strategies, against the oracle."""
    open(os.path.join(tmp_path, "s.txt"), "w").write(_HEADER + body)
    img, st, ref, cnt = _render_both("s.txt", str(tmp_path), accel=accel)
    assert img.shape == (17, 33, 3)
    assert_parity(img, ref, f"{kind} accel{accel}")
    assert _counts(st) == cnt
    if kind == "empty":
        assert np.all(img == np.float32([0.1, 0.2, 0.3]))
        assert cnt["shadow"] == cnt["reflection"] == cnt["refraction"] == 0


def _many_lights_text(n: int) -> str:
    """A small scene lit by n lights (every 500th directional): more lights
    than a workgroup's LDS holds (64 B each)."""
    import random
    rnd = random.Random(7)
    out = [_HEADER.replace("light -10 10 0 1 0.6 0.6 0.6\n", "")]
    for i in range(n):
        w = 0 if i % 500 == 0 else 1
        out.append(f"light {rnd.uniform(-20, 20):.4f} {rnd.uniform(-5, 20):.4f} {rnd.uniform(-20, 5):.4f} {w} "
                   f"{rnd.uniform(0, 0.004):.5f} {rnd.uniform(0, 0.004):.5f} {rnd.uniform(0, 0.004):.5f}\n")
    out.append("mtlcolor 1 0 0 1 1 1 0.2 0.6 0.5 20 0.3 1.5\nsphere 0 0 -5 1\n")
    out.append("mtlcolor 0.3 0.8 0.2 1 1 1 0.2 0.6 0.2 20\nsphere 1.5 0.5 -7 1\nsphere -1.5 -0.5 -6 0.7\n")
    out.append("v -4 -2 -3\nv 4 -2 -3\nv 0 -2 -12\nf 1 2 3\n")
    return "".join(out)


@pytest.mark.parametrize("accel", [0, 1])
def test_many_lights(accel, tmp_path):
    """3000 lights (192 KB of light records): the lights that do not fit in
    the workgroup's LDS are read from device memory (Params::lights_in_lds), so the
    scene renders -- the reference has no light limit.  Against the oracle,
    identical ray counts, on both search strategies."""
    (tmp_path / "many.txt").write_text(_many_lights_text(3000))
    img, st, ref, cnt = _render_both("many.txt", str(tmp_path), accel=accel)
    assert_parity(img, ref, f"many lights accel{accel}")
    assert _counts(st) == cnt
    assert cnt["shadow"] >= 3000


@pytest.mark.parametrize("n,maxf,split", [(32767, 5, 1), (32768, 17, 0)])
def test_many_lights_meta_limit(n, maxf, split, tmp_path):
    """The split frame slots' instantiations (MAXF 5 and 9) keep the light
    index in 15 bits of a node's meta, the level kinds above it: 32767 lights
    run there (the index reaches 32767 after the last light), 32768 take the
    MAXF 17 instantiation, whose meta keeps 23 bits.  Both against the oracle,
    with identical ray counts (glass and mirror spheres: refraction and
    reflection children on every level)."""
    (tmp_path / "many.txt").write_text(_many_lights_text(n))
    hs = rtamd.HostScene("many.txt", cwd=str(tmp_path))
    gs = rtamd.GpuScene(hs)
    img, st = gs.render_rows(hs.camera(), hs.width, hs.height, 0, hs.height)
    dbg = gs.debug_counters()
    gs.close()
    ref, cnt = OracleScene("many.txt", cwd=str(tmp_path)).render()
    assert_parity(np.asarray(img).reshape(ref.shape), ref, f"{n} lights")
    assert _counts(st) == cnt and cnt["refraction"] > 0 and cnt["reflection"] > 0
    assert (dbg[46], dbg[47]) == (maxf, split)


def _deep_scene_text(w: int = 32, h: int = 32) -> str:
    """Four arms of spheres at geometrically growing distance (1.08^k, k < 200)
    from the view axis and along it: a skewed tree (worst-case stack 27 with
    the device's padding; tools/bvh_check mode 4 estimates it on the host)."""
    import math
    out = [gen.HEADER.format(w=w, h=h), "light -10 10 0 1 0.6 0.6 0.6\n", "light 10 8 -10 1 0.6 0.6 0.6\n"]
    for i in range(800):
        k, arm = i % 200, i // 200
        d, ang = 1.08 ** k, arm * math.pi / 2
        glass = " 0.3 1.5" if i % 10 == 0 else ""
        out.append(f"mtlcolor 0.{i % 7 + 2} 0.5 0.{i % 5 + 3} 1 1 1 0.2 0.6 0.5 20{glass}\n")
        out.append(f"sphere {math.cos(ang) * d * 0.3:.6f} {math.sin(ang) * d * 0.3:.6f} {-(5 + d):.6f} 0.4\n")
    return "".join(out)


_CHECK_SCRIPT = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import rtamd
out = {}
for name, cwd, depth, opts in json.loads(sys.argv[2]):
    hs = rtamd.HostScene(name, cwd=cwd)
    hs.set_depth(depth)
    W, H = hs.width, hs.height
    gs = rtamd.GpuScene(hs)
    for k, v in opts.items():
        gs.set_option(k, v)
    img, st = gs.render_rows(hs.camera(), W, H, 0, H)
    dbg = gs.debug_counters()
    key = name + json.dumps(opts, sort_keys=True)
    np.save(os.path.join(sys.argv[3], str(len(out)) + ".npy"), img)
    out[key] = dict(violations=int(dbg[49]), spills=int(st.stack_spills), rays=st.rays(), idx=len(out))
    gs.close()
print(json.dumps(out))
"""


def test_rt_check_stack_bottom_invariant(tmp_path):
    """The RT_CHECK build (simple-raytracer_amd/lib_check/, never benched)
    checks the BVH stack-bottom invariant -- entry 0 is kEmpty or a refill
    tag kRefill + b with b spilled blocks inside the lane's spill area -- at
    every traversal entry and exit, spill and refill (rt_kernels.hip
    bvh_trace; round 4's suspended-search variant faulted by breaking it).
    On the scenes that spill most (the skewed deep tree and C3 / C5 with a
    12-entry LDS share) no violation is counted, and the images and ray
    counts equal the benched library's bit for bit."""
    lib = os.path.join(PKG, "lib_check", "librt_hip.so")
    if not os.path.exists(lib):
        pytest.fail("lib_check/ missing: __graft_entry__.build() (make -C simple-raytracer_amd check)")
    (tmp_path / "deep.txt").write_text(_deep_scene_text())
    cases = [("deep.txt", str(tmp_path), 4, {}), ("deep.txt", str(tmp_path), 4, {"lds_stack": 12}),
             ("C3_64x64.txt", SCENES, 4, {"lds_stack": 12}), ("C5_8x8.txt", SCENES, 8, {"lds_stack": 12}),
             ("C5_8x8.txt", SCENES, 8, {})]
    env = dict(os.environ, RTAMD_LIB_DIR=os.path.join(PKG, "lib_check"))
    r = subprocess.run([sys.executable, "-c", _CHECK_SCRIPT, PKG, json.dumps(cases), str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    spills = 0
    for name, cwd, depth, opts in cases:
        key = name + json.dumps(opts, sort_keys=True)
        g = got[key]
        assert g["violations"] == 0, (key, g)
        spills += g["spills"]
        hs = rtamd.HostScene(name, cwd=cwd)
        hs.set_depth(depth)
        gs = rtamd.GpuScene(hs)
        for k, v in opts.items():
            gs.set_option(k, v)
        ref, st = gs.render_rows(hs.camera(), hs.width, hs.height, 0, hs.height)
        img = np.load(str(tmp_path / f"{g['idx']}.npy"))
        assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), key
        assert g["rays"] == st.rays() and g["spills"] == st.stack_spills, (key, g, st.rays())
        gs.close()
    assert spills > 0
    _summary["rt_check"] = got


@pytest.mark.parametrize("size", [(1, 7), (7, 1), (1, 1)])
def test_degenerate_image_sizes(size):
    """The seam (main.cpp:670) takes any image size: for a 1-pixel-wide or
    -tall image its camera deltas divide by res - 1 = 0 (main.cpp:709-710),
    every primary ray is NaN and meets nothing, and the image is the
    background.  rt_render_rows does the same, against the oracle's camera
    and render at that size, with identical ray counts.  (The reference's
    parser rejects such an imsize, main.cpp:242; test_host.py checks the CLI
    does too.)"""
    W, H = size
    for name in ("test7_s.txt", "C3_64x64.txt"):
        hs = rtamd.HostScene(name, cwd=SCENES)
        cam = hs.camera(W, H)
        gs = rtamd.GpuScene(hs)
        img, st = gs.render_rows(cam, W, H, 0, H)
        px, _ = gs.render_pixels(cam, W, H, np.array([[W - 1, H - 1]], dtype=np.int32))
        gs.close()
        ref, cnt = OracleScene(name, cwd=SCENES).render(W, H)
        assert_parity(img, ref, f"{name} {W}x{H}")
        assert _counts(st) == cnt
        assert st.primary == W * H
        bkg = OracleScene(name, cwd=SCENES).globals()[:3]
        if W == 1 or H == 1:
            assert np.array_equal(img.reshape(-1, 3), np.broadcast_to(bkg, (W * H, 3))), img
        assert np.array_equal(px[0], img[H - 1, W - 1])


def test_nan_rays_on_the_bvh():
    """Rays with a NaN origin or direction (test7's and Test1's eta = 0
    materials produce them) meet nothing in the reference; the
    BVH answers them without a search (a NaN slab test would enter every box).
    On the BVH path (accel = 1) the image matches the oracle, NaN pixels
    included, with identical ray counts, and such queries did occur."""
    seen = 0
    for name in ("test7_s.txt", "Test1_s.txt"):
        hs = rtamd.HostScene(name, cwd=SCENES)
        W, H = hs.width, hs.height
        gs = rtamd.GpuScene(hs)
        gs.set_option("accel", 1)
        img, st = gs.render_rows(hs.camera(), W, H, 0, H)
        nan_q = gs.debug_counters()[35]
        ref, cnt = OracleScene(name, cwd=SCENES).render()
        assert_parity(img, ref, f"{name} accel1")
        assert _counts(st) == cnt
        seen += nan_q
        _summary[f"nan_rays_{name}"] = dict(nan_queries=nan_q, nan_px=int(np.isnan(img).any(-1).sum()))
    assert seen > 0


def test_deep_stack_tree(tmp_path):
    """The stack spill area is sized per tree (Params::ovf_stride, from the
    deepest of the main and cone trees).  A skewed tree whose worst-case stack
    is about twice the 12-entry LDS share spills two blocks deep and brings
    them back; the image and ray counts match the oracle."""
    (tmp_path / "deep.txt").write_text(_deep_scene_text())
    for opts in ({}, {"lds_stack": 12}):
        hs = rtamd.HostScene("deep.txt", cwd=str(tmp_path))
        W, H = hs.width, hs.height
        gs = rtamd.GpuScene(hs)
        for k, v in opts.items():
            gs.set_option(k, v)
        img, st = gs.render_rows(hs.camera(), W, H, 0, H)
        dbg = gs.debug_counters()
        assert dbg[16] == 2 and dbg[22] >= 24, (dbg[16], dbg[22])      # BVH mode, a deep worst case
        ref, cnt = OracleScene("deep.txt", cwd=str(tmp_path)).render()
        assert_parity(img, ref, f"deep stack {opts}")
        assert _counts(st) == cnt
        _summary[f"deep_stack_{opts}"] = dict(stack=dbg[22], spills=st.stack_spills)


def test_lds_stack_spill():
    """The BVH traversal stack keeps its newest entries in LDS and spills
    older ones to device memory when it runs deep.  A smaller LDS share
    (option lds_stack) spills far more often; the image and ray counts are
    unchanged bit for bit, on C3 (2000 objects) and C5 (100 000 spheres)."""
    for name, depth in (("C3_64x64.txt", 4), ("C5_8x8.txt", 8)):
        hs = rtamd.HostScene(name, cwd=SCENES)
        hs.set_depth(depth)
        W, H = hs.width, hs.height
        cam = hs.camera()
        ref, st = rtamd.GpuScene(hs).render_rows(cam, W, H, 0, H)
        gs = rtamd.GpuScene(hs)
        gs.set_option("lds_stack", 12)    # default 15
        img, st2 = gs.render_rows(cam, W, H, 0, H)
        assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), name
        assert _counts(st2) == _counts(st)
        assert st2.stack_spills > st.stack_spills and st2.stack_spills > 0, (name, st.stack_spills, st2.stack_spills)
        _summary[f"spills_{name}"] = dict(default=st.stack_spills, lds12=st2.stack_spills)
        with pytest.raises(rtamd.RTError):
            gs.set_option("lds_stack", 11)


def test_refill_options_bit_identical():
    """How a wave refills its idle lanes, and when it lets reflection /
    refraction searches run (option gate_x: held back until that many lanes
    have one), decide which lane renders which pixel and when, never a
    pixel's value.  Option chunk (work items taken
    from the pixel counter at a time; default 0 = the idle lanes' count) and
    option refill_min (idle lanes before a refill; default 32 or 48 when the scene
    reflects or refracts, else 64), including chunks that do not align with
    the 8x8 tiles and a ragged 37x23 image: the same image and ray counts bit
    for bit, equal to the oracle's."""
    variants = [{"chunk": c} for c in (1, 16, 64, 100, 256)]
    variants += [{"refill_min": r} for r in (1, 7, 33, 64)]
    variants += [{"chunk": 64, "refill_min": 1}, {"chunk": 100, "refill_min": 48}]
    variants += [{"gate_x": g} for g in (0, 1, 17, 64)] + [{"gate_x": 0, "refill_min": 1}]
    for name, size in (("C3_64x64.txt", None), ("C4_32x32.txt", None), ("test7_s.txt", (37, 23))):
        ref, st = rtamd.render_scene(name, cwd=SCENES, imsize=size)
        o, o_cnt = OracleScene(name, cwd=SCENES).render(*(size or ()))
        assert_parity(ref, o, f"{name} default refill")
        assert _counts(st) == o_cnt
        for opts in variants:
            img, st2 = rtamd.render_scene(name, cwd=SCENES, imsize=size, options=opts)
            assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), (name, opts)
            assert _counts(st2) == _counts(st), (name, opts)
    for bad in ({"chunk": -1}, {"refill_min": 0}, {"refill_min": 65}, {"gate_x": 65}):
        with pytest.raises(rtamd.RTError):
            rtamd.render_scene("test7_s.txt", cwd=SCENES, options=bad)


@pytest.mark.parametrize("name,size", [("C3_64x64.txt", None), ("C4_32x32.txt", None), ("test7_s.txt", (37, 23)),
                                       ("house_s.txt", None), ("edge_glass_faces.txt", None),
                                       ("earth_pyramid_s.txt", None)])
def test_bvh_presplit_bit_identical(name, size):
    """Option bvh_presplit: faces with a shadow factor of 0 or 1 enter the BVH
    as several references with clipped boxes (rt_accel.cpp presplit; off by
    default).  Every
    point of a face stays inside some reference's padded box, a leaf records
    a face once, and a face met twice answers the same: images and per-type
    ray counts bit for bit against the unsplit tree (and the unsplit image
    against the oracle's); the tree did change where faces were split."""
    kw = dict(cwd=SCENES, imsize=size)
    ref, st = rtamd.render_scene(name, options={"accel": 1, "bvh_presplit": 0}, **kw)
    changed = False
    for ps in (2, 4):
        img, st2 = rtamd.render_scene(name, options={"accel": 1, "bvh_presplit": ps}, **kw)
        assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), (name, ps)
        assert _counts(st2) == _counts(st), (name, ps)
        changed |= st2.box_tests != st.box_tests
    _, st_d = rtamd.render_scene(name, options={"accel": 1}, **kw)
    assert st_d.box_tests == st.box_tests          # (off by default)
    if name in ("C3_64x64.txt", "C4_32x32.txt"):
        assert changed
        o, _ = OracleScene(name, cwd=SCENES).render(*(size or ()))
        assert_parity(ref, o, f"{name} presplit")
    with pytest.raises(rtamd.RTError):
        rtamd.render_scene(name, options={"bvh_presplit": 9}, **kw)


def test_last_light_skip_and_recursive_instantiation_bit_identical():
    """Scenes without reflecting or refracting materials render with the
    MAXF = 1 instantiation, which counts a last light's shadow ray whose Phong
    term is exactly 0 without searching it (option last_light_skip; exact:
    its contribution is light colour x mask x 0 whatever the mask).  With the
    skip off, and with the recursive instantiation forced (option recursive,
    which has no skip), on scenes with four lights and back-facing triangles
    (never flipped, main.cpp:869-872): the same image and per-type ray counts
    bit for bit, equal to the oracle's; the skip did fire."""
    extra = "light 5 20 -30 1 0.4 0.3 0.2\nlight -15 -5 -10 1 0.3 0.3 0.5\n"
    fired = 0
    for base in ("C4_32x32.txt", "C2_128x128.txt"):
        name = "_lls_" + base
        p = os.path.join(SCENES, name)
        open(p, "w").write(open(os.path.join(SCENES, base)).read() + extra)
        try:
            ref, st = rtamd.render_scene(name, cwd=SCENES)
            oi, o_cnt = OracleScene(name, cwd=SCENES).render()
            assert_parity(ref, oi, f"{name} default")
            assert _counts(st) == o_cnt
            for opts in ({"last_light_skip": 0}, {"recursive": 1}, {"recursive": 1, "counters": 0},
                         {"last_light_skip": 0, "counters": 0}):
                img, st2 = rtamd.render_scene(name, cwd=SCENES, options=opts)
                assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), (name, opts)
                if opts.get("counters", 1):
                    assert _counts(st2) == _counts(st), (name, opts)
                    if opts.get("last_light_skip", 1) == 0 or opts.get("recursive"):
                        fired += int(st.shadow_known - st2.shadow_known)
                        assert st2.shadow_known <= st.shadow_known
        finally:
            os.remove(p)
    assert fired > 0
    with pytest.raises(rtamd.RTError):
        rtamd.render_scene("test7_s.txt", cwd=SCENES, options={"recursive": 2})


def test_work_bands_counters_bit_identical():
    """Option work_parts (bands of the work items with a pixel counter each,
    auto = one per XCD) and option counters (0: the kernel instantiation
    without the counters, which the bench times) change which lane renders
    which pixel, never a pixel: the image and ray counts equal the default
    render's bit for bit, which equals the oracle's."""
    variants = [{"work_parts": w} for w in (1, 2, 4, 8)] + [{"work_parts": 1, "chunk": 100}]
    # the instantiation without counters renders the same image (its counts are 0)
    variants += [{"counters": 0}, {"counters": 0, "work_parts": 1}, {"counters": 0, "work_parts": 2, "chunk": 64}]
    for name, depth in (("C2_128x128.txt", None), ("C3_64x64.txt", None), ("C5_8x8.txt", 8)):
        ref, st = rtamd.render_scene(name, cwd=SCENES, depth=depth)
        o = OracleScene(name, cwd=SCENES)
        if depth:
            o.set_depth(depth)
        oi, o_cnt = o.render()
        assert_parity(ref, oi, f"{name} default")
        assert _counts(st) == o_cnt
        for opts in variants:
            img, st2 = rtamd.render_scene(name, cwd=SCENES, depth=depth, options=opts)
            assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), (name, opts)
            if opts.get("counters", 1):
                assert _counts(st2) == _counts(st), (name, opts)
            else:
                assert st2.rays() == 0 and st2.box_tests == 0 and st2.kernel_ms > 0, (name, opts)
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    gs = rtamd.GpuScene(hs)
    gs.render_rows(hs.camera(), hs.width, hs.height, 0, hs.height)
    dbg = gs.debug_counters()
    assert dbg[44] == 0 and dbg[48] == 1 and dbg[45] == 8           # counted by default
    st1 = gs.last_stats()
    assert st1.box_tests > 0 and st1.sphere_tests > 0 and st1.face_tests > 0 and st1.rays() > 0
    gs.set_option("counters", 0)
    gs.render_rows(hs.camera(), hs.width, hs.height, 0, hs.height)
    st0 = gs.last_stats()
    assert gs.debug_counters()[48] == 0 and st0.rays() == 0 and st0.box_tests == 0
    # hot_copies: removed in round 6 (an unknown option is refused)
    for bad in ({"hot_copies": 16}, {"work_parts": 3}, {"counters": 2}):
        with pytest.raises(rtamd.RTError):
            rtamd.render_scene("test7_s.txt", cwd=SCENES, options=bad)


@pytest.mark.parametrize("opts", [{"gate_x": 64, "refill_min": 64}, {"gate_x": 64, "refill_min": 1}, {"gate_x": 0, "refill_min": 64}])
def test_extreme_batching_deep_scene(opts):
    """The batching options at their extremes on a depth-8 C5 miniature (long
    shade trees: up to 8 levels of reflection / refraction per pixel): a wave
    that holds every reflection / refraction search until all 64 lanes have
    one, or refills only when all 64 lanes are idle, still drains (a held
    search is released when nothing else would search) and renders the
    oracle's image with its ray counts."""
    img, st = rtamd.render_scene("C5_8x8.txt", cwd=SCENES, depth=8, options=opts)
    o = OracleScene("C5_8x8.txt", cwd=SCENES)
    o.set_depth(8)
    ref, cnt = o.render()
    assert_parity(img, ref, f"C5_8x8 depth 8 {opts}")
    assert _counts(st) == cnt


def test_origin_leaf_pass_bit_identical(tmp_path):
    """Option org_first: a secondary ray first tests the BVH leaf of the object
    it starts on (a closest hit found there bounds the search, an opaque
    occluder there ends a shadow ray), then searches from the root.  Images
    and ray counts are bit for bit those without it, for every combination of
    ray kinds, on C3 (2000 objects, glass), C3G (glass triangles: SKIP_TRANS),
    C3D (a directional light over spheres: cone queries), C5 (100 000
    spheres, depth 8) and test7 (NaN pixels); the automatic setting turns it
    on for C5's dense scene and off for the others."""
    cases = [("C3_64x64.txt", 4, SCENES), ("C5_8x8.txt", 8, SCENES), ("test7_s.txt", 4, SCENES)]
    for cfg in ("C3G", "C3D"):
        (tmp_path / f"{cfg}_40x32.txt").write_text(gen.scene_text(cfg, w=40, h=32))
        cases.append((f"{cfg}_40x32.txt", 4, str(tmp_path)))
    for name, depth, cwd in cases:
        hs = rtamd.HostScene(name, cwd=cwd)
        hs.set_depth(depth)
        W, H = hs.width, hs.height
        cam = hs.camera()
        ref = None
        for v in (0, 1, 2, 4, 7, -1):
            gs = rtamd.GpuScene(hs)
            gs.set_option("accel", 1)
            gs.set_option("org_first", v)
            img, st = gs.render_rows(cam, W, H, 0, H)
            dbg = gs.debug_counters()
            if ref is None:
                ref = (img, _counts(st))
            assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref[0], nan=-9)), (name, v)
            assert _counts(st) == ref[1], (name, v)
            if v == -1:
                auto = int(dbg[40])
                assert auto == (6 if name.startswith("C5") else 0), (name, auto, dbg[41] / 1000)
                _summary[f"org_first_auto_{name}"] = dict(org_first=auto, density=dbg[41] / 1000)
            gs.close()


def test_origin_leaf_pass_special_cases(tmp_path):
    """The origin-leaf pass on the reference's order-dependent cases: glass
    triangles (SKIP_TRANS) and a directional light over spheres (cone
    queries), all ray kinds on, against the oracle with identical counts."""
    for cfg in ("C3G", "C3D"):
        name = f"{cfg}_40x32.txt"
        (tmp_path / name).write_text(gen.scene_text(cfg, w=40, h=32))
        img, st = rtamd.render_scene(name, cwd=str(tmp_path), options={"org_first": 7})
        ref, cnt = OracleScene(name, cwd=str(tmp_path)).render()
        assert_parity(img, ref, f"{cfg} org_first=7")
        assert _counts(st) == cnt


@pytest.mark.parametrize("opts", [{"bvh_collapse": 0}, {"bvh_collapse": 1, "bvh_node": 1000}])
def test_bvh_collapse_parity(opts):
    """The 4-wide tree comes from the binary SAH tree by an SAH-optimal
    collapse (default; the binary tree goes down to single primitives and the
    collapse picks the leaves) or a greedy one (option bvh_collapse = 0): the
    tree changes which boxes are tested, not the result -- parity with the
    oracle and identical ray counts on C3 (2000 objects) and C5 (100 000
    spheres, depth 8), for the greedy collapse and another node cost."""
    for name, depth in (("C3_64x64.txt", 4), ("C5_8x8.txt", 8)):
        img, st = rtamd.render_scene(name, cwd=SCENES, depth=depth, options=opts)
        o = OracleScene(name, cwd=SCENES)
        o.set_depth(depth)
        ref, cnt = o.render()
        tag = ",".join(f"{k}={v}" for k, v in opts.items())
        assert_parity(img, ref, f"{name} {tag}")
        assert _counts(st) == cnt
        _summary[f"collapse_{name}_{tag}"] = dict(box=st.box_tests, face=st.face_tests, sphere=st.sphere_tests)


def test_one_slot_two_streams():
    """With one render slot (inflight = 1), renders issued on two different
    caller streams share the slot's counters and frames: they must run one
    after the other, each bit-identical to a synchronous render."""
    torch = pytest.importorskip("torch")
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    ref, st = gs.render_rows(cam, W, H, 0, H)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.full((H, W, 3), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(6)]
    for k, o in enumerate(outs):
        s = streams[k % 2]
        gs.render_rows_async(cam, W, H, 0, H, o.data_ptr(), s.cuda_stream)
    # and a synchronous render on the scene's own stream while those may run
    img, st2 = gs.render_rows(cam, W, H, 0, H)
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(np.nan_to_num(o.cpu().numpy(), nan=-9), np.nan_to_num(ref, nan=-9))
    assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9))
    assert _counts(st2) == _counts(st)


def test_bvh_rebuild_on_camera_move():
    """The BVH's padding depends on the eye: moving the eye far away rebuilds
    it (the old tree is freed only after the new one is on the device).
    Renders before, after and back again equal fresh scenes' renders."""
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    far = rtamd.rt_camera()
    off = (0.0, 0.0, 900.0)
    for f in ("eye", "ul"):
        for k in range(3):
            getattr(far, f)[k] = getattr(cam, f)[k] + off[k]
    for f in ("dh", "dv"):
        for k in range(3):
            getattr(far, f)[k] = getattr(cam, f)[k]
    gs = rtamd.GpuScene(hs)
    a, sa = gs.render_rows(cam, W, H, 0, H)
    b, sb = gs.render_rows(far, W, H, 0, H)
    c, sc = gs.render_rows(cam, W, H, 0, H)
    assert sb.bvh_build_ms > 0
    fa, _ = rtamd.GpuScene(hs).render_rows(cam, W, H, 0, H)
    fb, _ = rtamd.GpuScene(hs).render_rows(far, W, H, 0, H)
    eq = lambda x, y: np.array_equal(np.nan_to_num(x, nan=-9), np.nan_to_num(y, nan=-9))
    assert eq(a, fa) and eq(c, fa) and eq(b, fb)
    assert _counts(sa) == _counts(sc)


@pytest.mark.parametrize("accel", [0, 1])
@pytest.mark.parametrize("cfg", ["C3D", "C3G"])
def test_special_cases_on_the_bvh(cfg, accel, tmp_path):
    """C3 with a directional light (unnormalised direction against spheres:
    the reference's A = 1 sphere quirk, main.cpp:895) and C3 with glass
    triangles (SKIP_TRANS, main.cpp:1000-1002): the BVH answers both exactly
    -- shadow-region point queries, and the stack top's own root plus an
    any-hit search -- with no brute-force query left; the scan (accel=0)
    agrees.  Against the oracle (pinned to the reference by
    test_float_goldens' C3D/C3G fixtures) with identical ray counts."""
    name = f"{cfg}_48x40.txt"
    (tmp_path / name).write_text(gen.scene_text(cfg, w=48, h=40))
    img, st, ref, cnt = _render_both(name, str(tmp_path), accel=accel)
    assert_parity(img, ref, f"{cfg} accel{accel}")
    assert _counts(st) == cnt
    if accel == 1:
        assert st.bf_queries == 0
    if cfg == "C3G":
        assert cnt["skip_trans"] > 0
    _summary[f"{cfg}@accel{accel}"] = dict(compare(img, ref), counts=_counts(st), bf=st.bf_queries,
                                          tests=dict(box=st.box_tests, face=st.face_tests, sphere=st.sphere_tests))


@pytest.mark.parametrize("u8", [False, True])
def test_deinterleave_rows_device(u8):
    """rt_deinterleave_rows (floats) and rt_deinterleave_rows_u8 (the
    writer's bytes) put gathered row sets (rth_row_set's dealing) back in
    image order on the device, for ragged heights, several ranks, row
    widths with and without the 16-B vector path (W * 3 * element bytes a
    multiple of 16 or not), and a tall narrow image (H > 65535)."""
    torch = pytest.importorskip("torch")
    import ctypes as C
    from rtamd.dist import image_rows, row_set
    L = rtamd.hip_lib()
    f = L.rt_deinterleave_rows_u8 if u8 else L.rt_deinterleave_rows
    # (70001 rows: taller than the grid's y extent, 65535 -- rows are
    # grid-strided; round 5 refused such an image)
    for H, world, W in ((67, 3, 13), (8, 2, 16), (130, 8, 13), (5, 1, 64), (41, 4, 48), (70001, 3, 1)):
        per = row_set(H, world, 0)[4]
        if u8:
            g = torch.randint(0, 256, (world, per, W, 3), dtype=torch.uint8, device="cuda:0")
            img = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda:0")
        else:
            g = torch.rand((world, per, W, 3), dtype=torch.float32, device="cuda:0")
            img = torch.full((H, W, 3), -1.0, dtype=torch.float32, device="cuda:0")
        rc = f(C.c_void_p(g.data_ptr()), world, per, W, H, 8, C.c_void_p(img.data_ptr()),
               C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        torch.cuda.synchronize()
        want = torch.empty_like(img)
        for r in range(world):
            rows = image_rows(H, world, r)
            if rows:
                want[rows] = g[r, : len(rows)]
        assert torch.equal(img, want), (H, world, W)
        assert f(C.c_void_p(g.data_ptr()), world, per - 1 if per > 1 else 0, W, H, 8,
                 C.c_void_p(img.data_ptr()), None) == -1


def test_device_init_repeated():
    """rt_device_init may be called again: a repeated call keeps at most one
    waiting stream per device (each call used to add a stream, and
    with it a hardware queue, to the pool) and scenes created after it render
    the same image, stream reused or not."""
    L = rtamd.hip_lib()
    for _ in range(3):
        assert L.rt_device_init(0) == 0
    imgs = []
    for _ in range(3):
        img, st = rtamd.render_scene("test7_s.txt", cwd=SCENES)
        imgs.append(img)
    for img in imgs[1:]:
        assert np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(imgs[0], nan=-9))
    assert L.rt_device_init(-1) != 0


@pytest.mark.parametrize("block", ["100000", "1", "7", "64"])
def test_cli_streamed_ppm_matches(block, tmp_path):
    """Without --float-out the one-device CLI quantises the image on the
    device and copies 3 bytes per pixel to the host in row blocks, each block
    formatted as soon as it lands (write_ppm_bytes, rth_ppm_write_rows_u8);
    when some value is not 0..255 (test7: NaN pixels) it falls back to the
    floats, copied in row blocks through pinned buffers and written while the
    next block copies (stream_ppm; images of 512 MB and more, or whenever
    RT_PPM_BLOCK_ROWS is set; RT_PPM_FLOATS forces the floats).  Every way
    writes the P3 file byte for byte as the one written from the whole float
    image (--float-out takes that path), for one block and for 1-, 7- and
    64-row blocks on ragged images."""
    import json as _json
    for name, want_from in (("test7_s.txt", "floats"), ("C3_64x64.txt", "bytes")):
        outs, froms = [], []
        modes = [(["--float-out", str(tmp_path / "f.bin")], {}), ([], {"RT_PPM_BLOCK_ROWS": block}),
                 ([], {"RT_PPM_BLOCK_ROWS": block, "RT_PPM_FLOATS": "1"}), ([], {})]
        for args, env in modes:
            tmp_name = "_stream_" + name
            shutil.copy(os.path.join(SCENES, name), os.path.join(SCENES, tmp_name))
            out = os.path.join(SCENES, tmp_name[:-4] + ".ppm")
            sj = str(tmp_path / "stats.json")
            try:
                r = subprocess.run([CLI, tmp_name, "--stats-json", sj] + args, cwd=SCENES, capture_output=True,
                                   text=True, timeout=300, env={**os.environ, **env})
                assert r.returncode == 0, r.stderr
                outs.append(open(out, "rb").read())
                froms.append(_json.load(open(sj))["ppm_from"])
            finally:
                for p in (os.path.join(SCENES, tmp_name), out):
                    if os.path.exists(p):
                        os.remove(p)
        assert len(outs[0]) > 1000 and all(o == outs[0] for o in outs), (name, [len(o) for o in outs])
        assert froms == ["floats", want_from, "floats", want_from], (name, froms)


@pytest.mark.parametrize("name", ["test7_s.txt", "C3_64x64.txt"])
def test_cli_rccl_gather(name, tmp_path):
    """`rt --gpus 1 --gather rccl`: the image goes through the multi-device
    path (row blocks rendered into HBM, ncclGather to the first device, device
    de-interleave, one copy to the host) and equals the single-call render
    bit for bit (float buffer and PPM)."""
    outs = {}
    for mode in ("host", "rccl"):
        tmp_name = f"_cli_{mode}_" + name
        shutil.copy(os.path.join(SCENES, name), os.path.join(SCENES, tmp_name))
        ppm = os.path.join(SCENES, tmp_name[:-4] + ".ppm")
        fout = str(tmp_path / f"{mode}.bin")
        try:
            r = subprocess.run([CLI, tmp_name, "--gpus", "1", "--gather", mode, "--float-out", fout, "--stats"],
                               cwd=SCENES, capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            outs[mode] = (open(ppm, "rb").read(), np.fromfile(fout, dtype=np.float32), r.stderr)
        finally:
            for p in (os.path.join(SCENES, tmp_name), ppm):
                if os.path.exists(p):
                    os.remove(p)
    assert outs["host"][0] == outs["rccl"][0]
    a, b = outs["host"][1], outs["rccl"][1]
    assert np.array_equal(np.nan_to_num(a, nan=-9), np.nan_to_num(b, nan=-9))
    assert "rays primary=" in outs["rccl"][2]


@pytest.mark.parametrize("name,want_from", [("C3_64x64.txt", "bytes"), ("edge_nested_nobkgeta.txt", "floats"),
                                            ("test7_s.txt", None)])
def test_cli_rccl_byte_gather_matches_host(name, want_from, tmp_path):
    """`rt --gather rccl` gathers the P3 writer's values as bytes (3 B per
    pixel, rt_quantize_u8 on each device) and falls back to the floats when
    some value is outside 0..255 (edge_nested_nobkgeta: a background of 1.5
    and -0.25): the PPM is byte for byte `--gather host`'s either way, and
    --stats-json says which crossed the gather (main.cpp:718-719, the row
    loop the gather reassembles)."""
    import json as _json
    outs, froms = {}, {}
    for mode in ("host", "rccl"):
        tmp_name = f"_cli8_{mode}_" + name
        shutil.copy(os.path.join(SCENES, name), os.path.join(SCENES, tmp_name))
        ppm = os.path.join(SCENES, tmp_name[:-4] + ".ppm")
        sj = str(tmp_path / f"{mode}.json")
        try:
            r = subprocess.run([CLI, tmp_name, "--gpus", "1", "--gather", mode, "--stats-json", sj],
                               cwd=SCENES, capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            outs[mode] = open(ppm, "rb").read()
            froms[mode] = _json.load(open(sj))["ppm_from"]
        finally:
            for p in (os.path.join(SCENES, tmp_name), ppm):
                if os.path.exists(p):
                    os.remove(p)
    assert len(outs["host"]) > 100 and outs["host"] == outs["rccl"]
    assert froms["rccl"] == froms["host"], froms
    if want_from:
        assert froms["rccl"] == want_from, froms


def _device_count() -> int:
    import ctypes as C
    return int(rtamd.hip_lib().rt_device_count())


def test_cli_rccl_gather_multi_device(tmp_path):
    """`rt --gpus 2 --gather rccl` (ncclCommInitAll over two devices, one
    grouped ncclGather to the first, device de-interleave) equals
    `--gather host` byte for byte.  Needs two devices: skipped on a one-GPU
    box (the CLI's default stays `host` until this has run)."""
    if _device_count() < 2:
        pytest.skip("needs 2 HIP devices")
    name = "C3_64x64.txt"
    outs = {}
    # rccl8: without --float-out the gather carries the writer's bytes
    for mode in ("host", "rccl", "rccl8"):
        tmp_name = f"_cli2_{mode}_" + name
        shutil.copy(os.path.join(SCENES, name), os.path.join(SCENES, tmp_name))
        ppm = os.path.join(SCENES, tmp_name[:-4] + ".ppm")
        fout = str(tmp_path / f"{mode}.bin")
        extra = [] if mode == "rccl8" else ["--float-out", fout]
        try:
            r = subprocess.run([CLI, tmp_name, "--gpus", "2", "--gather", mode[:4]] + extra,
                               cwd=SCENES, capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            outs[mode] = (open(ppm, "rb").read(), np.fromfile(fout, dtype=np.float32) if extra else None)
        finally:
            for p in (os.path.join(SCENES, tmp_name), ppm):
                if os.path.exists(p):
                    os.remove(p)
    assert outs["host"][0] == outs["rccl"][0] == outs["rccl8"][0]
    assert np.array_equal(np.nan_to_num(outs["host"][1], nan=-9), np.nan_to_num(outs["rccl"][1], nan=-9))


def test_quantize_u8_device():
    """rt_quantize_u8 (the gather's 3-byte pixels) equals the P3 writer's
    values (rth_quantize, main.cpp:760) wherever those are 0..255, and flags
    every other value -- NaN, infinities, above 1, at or below -1/255 -- on
    random colours and the boundaries, for lengths that are and are not
    multiples of 4."""
    torch = pytest.importorskip("torch")
    from rtamd.dist import quantize_u8_device
    rng = np.random.default_rng(7)
    edge = np.array([0.0, -0.0, 1.0, 0.5, 1 / 255, 254.999 / 255, 255.999 / 255, -0.5 / 255,
                     -0.999 / 255, np.nextafter(np.float32(-1 / 255), np.float32(0)), 1e-30, -1e-30],
                    dtype=np.float32)
    bad = np.array([np.nan, np.inf, -np.inf, 1.5, 256 / 255, -1 / 255, -2.0, 3e9], dtype=np.float32)
    for n in (1, 3, 4, 7, 1000, 4099):
        good = np.concatenate([edge, rng.random(n, dtype=np.float32)])[:max(n, 1)]
        for vals, expect_flag in ((good, False), (np.concatenate([good, bad[: 1 + n % len(bad)]]), True)):
            ref = rtamd.quantize(vals.reshape(-1))
            x = torch.from_numpy(vals.copy()).cuda()
            out = torch.full((vals.size,), 77, dtype=torch.uint8, device="cuda")
            flag = torch.zeros(1, dtype=torch.int32, device="cuda")
            quantize_u8_device(rtamd, torch, x, out, flag)
            torch.cuda.synchronize()
            o = out.cpu().numpy().astype(np.int64)
            inr = (ref >= 0) & (ref <= 255)
            assert np.array_equal(o[inr], ref[inr]), n
            assert (o[~inr] == 0).all()
            assert inr.all() != expect_flag, (n, ref[~inr])        # the host writer agrees on the cases
            assert bool(flag.item() & 1) == expect_flag, n


@pytest.mark.parametrize("fmt", ["f32", "auto"])
def test_multi_rank_hip_path_gloo(fmt):
    """The N > 1 bench data path with the HIP renderer (not the oracle): two
    ranks on one GPU (gloo gather staged through the host), each rendering
    its interleaved row set; rank 0 checks the gathered image bit for bit
    against one whole-image render (bench.py --verify) -- float rows, and
    (auto) the P3 writer's values as bytes, quantised on each rank."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--verify", "--steps", "2", "--warmup", "1",
           "--config", "C2", "--cpu-baseline", "off", "--gather-format", fmt]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["verified"] is True and line["n_gpus"] == 2
    assert line["config"]["gather_format"].startswith("f32" if fmt == "f32" else "u8"), line["config"]
    _summary[f"multi_rank_gloo_C2_{fmt}"] = dict(value=line["value"], verified=line["verified"])


def test_bvh_upload_failure_leaves_no_stale_tree():
    """A BVH rebuild whose device upload fails returns RT_E_NOMEM and leaves
    no tree marked valid (the old one is freed, nothing dangles); the next
    render rebuilds and is identical to a fresh scene's."""
    hs = rtamd.HostScene("C3_64x64.txt", cwd=SCENES)
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs)
    a, _ = gs.render_rows(cam, W, H, 0, H)
    gs.set_option("fail_bvh_upload", 1)
    gs.set_option("bvh_leaf", 8)                  # forces a rebuild at the next render
    with pytest.raises(rtamd.RTError):
        gs.render_rows(cam, W, H, 0, H)
    with pytest.raises(rtamd.RTError):            # still failing: retried, not a stale tree
        gs.render_rows(cam, W, H, 0, H)
    gs.set_option("fail_bvh_upload", 0)
    b, sb = gs.render_rows(cam, W, H, 0, H)
    assert np.array_equal(np.nan_to_num(a, nan=-9), np.nan_to_num(b, nan=-9))
    assert gs.debug_counters()[16] == 2           # BVH mode again


def _random_scene_text(seed: int) -> tuple[str, int, dict]:
    """A seeded random scene for the state machine's corners: nested and
    overlapping transparent spheres (deep medium stacks, exits without an
    entry), glass and mirror materials, eta 1 (F0 = 0), opaque and zero-ks
    objects, faces with and without vertex normals, point and directional
    lights, a background brighter than 1 or negative, an eye inside a glass
    sphere (refraction exits with an empty medium stack: ub_back), up to ~120
    spheres (the BVH by default), a depth from 1 to 10 -- the MAXF 5, 9 and
    17 instantiations -- and in about a third of the scenes small random P3
    textures on spheres and faces (texture coordinates beyond [0, 1] too; a
    second random stream, so the untextured scenes stay as they were).
    Returns (text, depth, {texture file: its text})."""
    import random
    r = random.Random(1000 + seed)
    tr = random.Random(7000 + seed)
    files = {}
    if tr.random() < 0.35:
        for k in range(tr.randint(1, 2)):
            tw, th = tr.randint(1, 6), tr.randint(1, 6)
            vals = " ".join(str(tr.randint(0, 255)) for _ in range(tw * th * 3))
            files[f"tex{k}.ppm"] = f"P3\n{tw} {th}\n255\n{vals}\n"
    uvs = []                                                     # vt lines, 1-based
    W, H = r.randint(6, 22), r.randint(5, 18)
    bk = [r.choice([0.1, 0.3, 0.7, 1.4, -0.2]) for _ in range(3)]
    bkg = f"bkgcolor {bk[0]} {bk[1]} {bk[2]}" + (f" {r.choice([1, 1.33])}" if r.random() < 0.7 else "")
    out = [f"eye {r.uniform(-0.5, 0.5):.3f} {r.uniform(-0.5, 0.5):.3f} 0\nviewdir {r.uniform(-0.2, 0.2):.3f} "
           f"{r.uniform(-0.2, 0.2):.3f} -1\nupdir 0 1 0\nhfov {r.randint(35, 80)}\nimsize {W} {H}\n{bkg}\n"]
    for _ in range(r.randint(1, 4)):
        w = 1 if r.random() < 0.7 else 0
        p = (r.uniform(-8, 8), r.uniform(-2, 9), r.uniform(-9, 3)) if w else (r.uniform(-1, 1), r.uniform(-1, 0.2),
                                                                                r.uniform(-1, 0.3))
        c = [r.uniform(0.1, 1) for _ in range(3)]
        out.append(f"light {p[0]:.3f} {p[1]:.3f} {p[2]:.3f} {w} {c[0]:.3f} {c[1]:.3f} {c[2]:.3f}\n")

    def mtl():
        od = [r.uniform(0, 1) for _ in range(3)]
        os_ = [r.uniform(0.5, 1) for _ in range(3)]
        ks = r.choice([0.0, 0.2, 0.5, 0.9])
        base = (f"mtlcolor {od[0]:.3f} {od[1]:.3f} {od[2]:.3f} {os_[0]:.2f} {os_[1]:.2f} {os_[2]:.2f} "
                f"{r.uniform(0.05, 0.3):.2f} {r.uniform(0.2, 0.8):.2f} {ks} {r.choice([2, 10, 40])}")
        kind = r.random()
        if kind < 0.35:
            return base + "\n"                                   # opaque, no eta
        op = r.choice([0.1, 0.3, 0.6, 0.9, 1.0])
        eta = r.choice([1.0, 1.33, 1.5, 2.4])
        return base + f" {op} {eta}\n"

    def tex():                                                   # after a mtlcolor: maybe textured
        if files and tr.random() < 0.5:
            return f"texture {tr.choice(sorted(files))}\n"
        return ""

    if r.random() < 0.15:                                        # the eye inside a glass sphere
        out.append(f"mtlcolor 0.9 0.9 0.9 1 1 1 0.1 0.3 0.5 20 {r.choice([0.2, 0.7])} {r.choice([1.2, 1.5])}\n")
        out.append("sphere 0 0 0 25\n")
    for _ in range(r.randint(2, 14) if r.random() < 0.8 else r.randint(30, 60)):   # spheres, some nested
        out.append(mtl() + tex())
        cx, cy, cz, rad = r.uniform(-3, 3), r.uniform(-2, 2), r.uniform(-12, -3), r.uniform(0.3, 1.6)
        out.append(f"sphere {cx:.3f} {cy:.3f} {cz:.3f} {rad:.3f}\n")
        if r.random() < 0.35:                                    # a concentric inner sphere
            out.append(mtl())
            out.append(f"sphere {cx:.3f} {cy:.3f} {cz:.3f} {rad * r.uniform(0.3, 0.8):.3f}\n")
    nv = 0
    for _ in range(r.randint(0, 10)):                            # triangles
        out.append(mtl())
        tx = tex()
        out.append(tx)
        c = (r.uniform(-3, 3), r.uniform(-2, 2), r.uniform(-12, -3))
        for _ in range(3):
            out.append(f"v {c[0] + r.uniform(-2, 2):.3f} {c[1] + r.uniform(-2, 2):.3f} {c[2] + r.uniform(-1.5, 1.5):.3f}\n")
        if r.random() < 0.4:
            out.append(f"vn {r.uniform(-1, 1):.3f} {r.uniform(-1, 1):.3f} {r.uniform(0.2, 1):.3f}\n"
                       f"vn {r.uniform(-1, 1):.3f} {r.uniform(-1, 1):.3f} {r.uniform(0.2, 1):.3f}\n"
                       f"vn {r.uniform(-1, 1):.3f} {r.uniform(-1, 1):.3f} {r.uniform(0.2, 1):.3f}\n")
            vn = True
        else:
            vn = False
        if tx:                                                   # texture coordinates, some beyond [0, 1]
            for _ in range(3):
                out.append(f"vt {tr.uniform(-0.3, 1.3):.3f} {tr.uniform(-0.3, 1.3):.3f}\n")
            t0 = len(uvs) + 1
            uvs += [0, 0, 0]
            if vn:
                out.append(f"f {nv + 1}/{t0}/{nv + 1} {nv + 2}/{t0 + 1}/{nv + 2} {nv + 3}/{t0 + 2}/{nv + 3}\n")
            else:
                out.append(f"f {nv + 1}/{t0} {nv + 2}/{t0 + 1} {nv + 3}/{t0 + 2}\n")
        elif vn:
            out.append(f"f {nv + 1}//{nv + 1} {nv + 2}//{nv + 2} {nv + 3}//{nv + 3}\n")
        else:
            out.append(f"f {nv + 1} {nv + 2} {nv + 3}\n")
        nv += 3
    return "".join(out), r.randint(1, 10), files


@pytest.mark.parametrize("seed", range(256))
def test_random_scenes_parity(seed, tmp_path):
    """256 seeded random scenes (`_random_scene_text`) against the oracle on
    the scan or the BVH (every third seed forced onto the tree), with
    identical ray counts; the seeds span depths 1-10, so all three recursive
    instantiations and their frame layouts (split slots for MAXF 5 / 9, whole
    32-B slots for 17) run."""
    text, depth, files = _random_scene_text(seed)
    (tmp_path / "rnd.txt").write_text(text)
    for name, body in files.items():
        (tmp_path / name).write_text(body)
    accel = 1 if seed % 3 == 0 else None
    img, st = rtamd.render_scene("rnd.txt", cwd=str(tmp_path), depth=depth,
                                 options=None if accel is None else {"accel": accel})
    o = OracleScene("rnd.txt", cwd=str(tmp_path))
    o.set_depth(depth)
    ref, cnt = o.render()
    assert_parity(img, ref, f"seed {seed} depth {depth}")
    assert _counts(st) == cnt, (seed, depth)
