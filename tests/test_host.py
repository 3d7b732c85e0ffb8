"""Host front end (librt_host.so) vs the oracle: parser, camera, quantiser,
PPM writer; plus the reference's error behaviour.  CPU only."""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess

import numpy as np
import pytest

import rtamd
from conftest import PKG, ROOT, SCENES, golden_names
from oracle_py import OracleScene, ppm_bytes, quantize as oq

NAMES = golden_names()


def host_objects(hs: rtamd.HostScene) -> np.ndarray:
    d = hs.desc
    rows = []
    for i in range(d.n_faces):
        f = d.faces[i]
        m = f.mat
        r = np.zeros(48, np.float32)
        r[0], r[1] = 0, f.texture
        r[2:14] = list(m.diffuse) + list(m.specular) + [m.ka, m.kd, m.ks, m.n, m.opacity, m.eta]
        r[18:27] = [x for k in range(3) for x in f.v[k]]
        r[27:36] = [x for k in range(3) for x in f.vn[k]]
        r[36:42] = [x for k in range(3) for x in f.vt[k]]
        r[42] = f.smooth
        rows.append(r)
    for i in range(d.n_spheres):
        s = d.spheres[i]
        m = s.mat
        r = np.zeros(48, np.float32)
        r[0], r[1] = 1, s.texture
        r[2:14] = list(m.diffuse) + list(m.specular) + [m.ka, m.kd, m.ks, m.n, m.opacity, m.eta]
        r[14:18] = list(s.center) + [s.radius]
        rows.append(r)
    return np.array(rows, np.float32).reshape(-1, 48)


@pytest.mark.parametrize("name", NAMES)
def test_parser_matches_oracle(name):
    hs = rtamd.HostScene(name, cwd=SCENES)
    os_ = OracleScene(name, cwd=SCENES)
    assert (hs.width, hs.height) == (os_.width, os_.height)
    a, b = host_objects(hs), os_.objects()
    assert a.shape == b.shape
    np.testing.assert_array_equal(a, b)
    d = hs.desc
    lights = np.array([list(d.lights[i].xyz) + [d.lights[i].w] + list(d.lights[i].color) + [0]
                       for i in range(d.n_lights)], np.float32).reshape(-1, 8)
    np.testing.assert_array_equal(lights, os_.lights())
    g = os_.globals()
    np.testing.assert_array_equal(np.array(list(d.bkg) + [d.eta_bkg, d.epsilon, d.depth], np.float32), g)
    for t in range(d.n_textures):
        tx = d.textures[t]
        arr = np.ctypeslib.as_array(tx.rgb, shape=(tx.height, tx.width, 3))
        np.testing.assert_array_equal(arr, os_.texture(t))


@pytest.mark.parametrize("name", NAMES)
def test_camera_matches_oracle(name):
    hs = rtamd.HostScene(name, cwd=SCENES)
    os_ = OracleScene(name, cwd=SCENES)
    # (1, 7), (7, 1), (1, 1): the seam's division by res - 1 = 0
    # (main.cpp:709-710) -- inf / NaN deltas, equal NaN for NaN
    for W, H in [(hs.width, hs.height), (37, 23), (1, 7), (7, 1), (1, 1)]:
        cam = hs.camera(W, H)
        mine = np.array([*cam.eye, *cam.ul, *cam.dh, *cam.dv], np.float32)
        np.testing.assert_array_equal(mine, os_.camera(W, H))


def test_quantize_and_writer_match_reference_format():
    rng = np.random.default_rng(3)
    img = rng.uniform(-0.5, 1.5, size=(7, 9, 3)).astype(np.float32)
    img[0, 0, 0] = np.nan
    img[1, 1, 1] = np.inf
    img[2, 2, 2] = -np.inf
    img[3, 3, 0] = 1e20
    img[3, 3, 1] = -0.0
    np.testing.assert_array_equal(rtamd.quantize(img), oq(img))
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "x.ppm")
        rtamd.write_ppm(p, img, threads=3)
        assert open(p, "rb").read() == ppm_bytes(img)
    # NaN prints as the reference's size_t(INT_MIN)
    assert b"18446744071562067968" in ppm_bytes(img)


def test_byte_writer_matches_float_writer():
    """rth_write_ppm_u8 / rth_ppm_write_rows_u8 (the CLI's 3-byte path: the
    device quantises, the host formats bytes) write the float writer's file
    byte for byte whenever every value is 0..255 -- including the level
    boundaries 0 and 255 (1.0 * 255 = 255)."""
    import tempfile
    rng = np.random.default_rng(11)
    img = rng.uniform(0, 1, size=(123, 77, 3)).astype(np.float32)
    img[0, 0] = [0.0, 1.0, np.nextafter(np.float32(1.0), np.float32(0))]
    img[1, 1] = [1 / 255, 254.99998 / 255, 0.5]
    q = rtamd.quantize(img)
    assert q.min() >= 0 and q.max() <= 255
    v = q.astype(np.uint8)
    with tempfile.TemporaryDirectory() as td:
        a, b = os.path.join(td, "a.ppm"), os.path.join(td, "b.ppm")
        rtamd.write_ppm(a, img, threads=4)
        rtamd.write_ppm_u8(b, v, threads=3)
        assert open(a, "rb").read() == open(b, "rb").read() == ppm_bytes(img)
        L = rtamd.host_lib()
        import ctypes as C
        h = C.c_void_p()
        assert L.rth_ppm_open(os.fsencode(b), 77, 123, 2, C.byref(h)) == 0
        for y in range(0, 123, 50):
            n = min(50, 123 - y)
            assert L.rth_ppm_write_rows_u8(h, v[y:y + n].ctypes.data, n) == 0
        assert L.rth_ppm_close(h) == 0
        assert open(b, "rb").read() == ppm_bytes(img)


def test_writer_large_parallel_matches():
    rng = np.random.default_rng(5)
    img = rng.uniform(0, 1, size=(300, 701, 3)).astype(np.float32)
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "x.ppm")
        rtamd.write_ppm(p, img, threads=8)
        assert hashlib.md5(open(p, "rb").read()).hexdigest() == hashlib.md5(ppm_bytes(img)).hexdigest()


def test_writer_in_row_blocks_matches():
    """The streaming writer (rth_ppm_open / write_rows / close: the CLI's
    copy-and-write overlap) gives write_ppm's bytes for any block size,
    including blocks that do not divide the height and NaN / out-of-range
    values; a short write (rows missing at close) fails."""
    rng = np.random.default_rng(9)
    img = rng.uniform(-0.5, 1.5, size=(67, 131, 3)).astype(np.float32)
    img[5, 7, 1] = np.nan
    img[60, 3, 2] = 3e9
    import tempfile
    ref = ppm_bytes(img)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "x.ppm")
        for block, threads in ((1, 1), (8, 3), (13, 8), (67, 2), (100, 4)):
            rtamd.write_ppm_blocks(p, img, block, threads)
            assert open(p, "rb").read() == ref, (block, threads)
        L = rtamd.host_lib()
        import ctypes as C
        h = C.c_void_p()
        assert L.rth_ppm_open(os.fsencode(p), 131, 67, 2, C.byref(h)) == 0
        assert L.rth_ppm_write_rows(h, img.ctypes.data, 10) == 0
        assert L.rth_ppm_write_rows(h, img.ctypes.data, 60) == -1      # past the height
        assert L.rth_ppm_close(h) == -1                                # 10 of 67 rows


def test_output_path_is_remove_extension():
    assert rtamd.output_path("a/b/scene.txt") == "a/b/scene.ppm"
    assert rtamd.output_path("scene") == "scene.ppm"
    assert rtamd.output_path("./scene") == ".ppm"          # rfind('.') quirk
    assert rtamd.output_path("dir.v2/scene") == "dir.ppm"


def _write(tmp_path, text, name="s.txt"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


BASE = "imsize 8 8\neye 0 0 0\nviewdir 0 0 -1\nupdir 0 1 0\nhfov 60\nbkgcolor 0 0 0\n"


@pytest.mark.parametrize("text,kind,last", [
    (BASE.replace("eye 0 0 0", "eye  0 0 0"), "oor", "basic_string::at"),
    (BASE + "sphere 0 0 -3 1\n", "inv", "ERROR: Command 'sphere' is undefined. Please verify input."),
    (BASE + "mtlcolor 1 1 1\n", "inv", "ERROR: Command 'mtlcolor' is undefined. Please verify input."),
    (BASE.replace("hfov 60", "hfov abc"), "inv", "ERROR: Command 'hfov' is undefined. Please verify input."),
    (BASE.replace("imsize 8 8", "imsize 1 8"), "inv", "ERROR: Command 'imsize' is undefined. Please verify input."),
    (BASE + "texture missing.ppm\n", "inv", "ERROR: Command 'texture' is undefined. Please verify input."),
])
def test_parse_errors(tmp_path, text, kind, last):
    p = _write(tmp_path, text)
    with pytest.raises(rtamd.ParseError) as ei:
        rtamd.HostScene(p)
    assert ei.value.code == (-2 if kind == "oor" else -1)
    assert ei.value.lines[-1].startswith(last)
    o = OracleScene(p)
    assert o.rc < 0


@pytest.mark.parametrize("drop", ["imsize", "eye", "viewdir", "updir", "hfov", "bkgcolor"])
def test_missing_command(tmp_path, drop):
    text = "\n".join(l for l in BASE.splitlines() if not l.startswith(drop + " ")) + "\n"
    p = _write(tmp_path, text)
    with pytest.raises(rtamd.MissingCommand) as ei:
        rtamd.HostScene(p)
    assert str(ei.value) == f"Error: Requires command '{drop}'"


def test_ignored_lines(tmp_path):
    """'#', unknown keywords, commands without arguments and trailing spaces
    are ignored (main.cpp:119-137); stof accepts prefixes ("1git")."""
    text = BASE + "# comment line\nfoo 1 2\neye\nmtlcolor 1 1 1 1 1 1 .1 .2 .3 10\nsphere 0 0 -4 1git \n"
    hs = rtamd.HostScene(_write(tmp_path, text))
    assert hs.desc.n_spheres == 1
    assert hs.desc.spheres[0].radius == 1.0


CLI = os.path.join(PKG, "lib", "rt")


def test_cli_messages(tmp_path):
    r = subprocess.run([CLI], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("Error: Incorrect number of arguments")
    r = subprocess.run([CLI, str(tmp_path / "nope.txt")], capture_output=True, text=True)
    assert r.returncode == 0
    assert r.stdout.strip() == f"ERROR: Issue reading input file '{tmp_path / 'nope.txt'}'. Please verify path."
    p = _write(tmp_path, BASE.replace("hfov 60\n", ""))
    r = subprocess.run([CLI, p], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "Error: Requires command 'hfov'"
    p = _write(tmp_path, BASE + "sphere 0 0 -3 1\n", "bad.txt")
    r = subprocess.run([CLI, p], capture_output=True, text=True)
    assert r.returncode != 0
    assert "ERROR: Must define a 'mtlcolor'. Please verify." in r.stderr
    assert "ERROR: Command 'sphere' is undefined. Please verify input." in r.stderr


REF_BIN = os.path.join(ROOT, "oracle", "_ref", "SimpleRayTracer")

# Scenes on which the reference stops before rendering: an uncaught exception
# (abort, main.cpp:114 for an empty token, :558-561 for the parser's
# rethrows) or a missing required command (message, exit 0, main.cpp:574-602).
# A missing texture file is left out: read_texture then uses uninitialised
# width / height (src/utility.h:62, :113) -- undefined behaviour that here
# either wrote an image or was killed allocating; the CLI reports an error.
REF_ERROR_SCENES = {
    "double_space": BASE.replace("eye 0 0 0", "eye  0 0 0"),
    "sphere_before_mtlcolor": BASE + "sphere 0 0 -3 1\n",
    "mtlcolor_3_args": BASE + "mtlcolor 1 1 1\n",
    "hfov_not_a_number": BASE.replace("hfov 60", "hfov abc"),
    # a 1-pixel-wide or -tall image: the reference's parser rejects it
    # (main.cpp:242) before the seam's division by res - 1 = 0 is reached
    "imsize_width_1": BASE.replace("imsize 8 8", "imsize 1 8"),
    "imsize_1_7": BASE.replace("imsize 8 8", "imsize 1 7"),
    "imsize_7_1": BASE.replace("imsize 8 8", "imsize 7 1"),
    "imsize_1_1": BASE.replace("imsize 8 8", "imsize 1 1"),
    "light_3_args": BASE + "light 1 1 1\n",
    **{f"missing_{k}": "\n".join(l for l in BASE.splitlines() if not l.startswith(k + " ")) + "\n"
       for k in ("imsize", "eye", "viewdir", "updir", "hfov", "bkgcolor")},
}


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="reference binary not built (oracle/Makefile ref)")
@pytest.mark.parametrize("name", sorted(REF_ERROR_SCENES) + ["nifty_pattern", "no_args", "no_such_file"])
def test_cli_error_behaviour_matches_reference_binary(tmp_path, name):
    """The drop-in CLI and the real reference binary on scenes the reference
    rejects: identical stdout, stderr and exit status (or abort signal).  No
    GPU is touched: both stop in the parser."""
    if name == "nifty_pattern":           # showcases/nifty_pattern.txt: 'eye  0.0' (double space)
        p = os.path.join(SCENES, "nifty_pattern.txt")
        args = [p]
    elif name == "no_args":
        args = []
    elif name == "no_such_file":
        args = [str(tmp_path / "nope.txt")]
    else:
        args = [_write(tmp_path, REF_ERROR_SCENES[name])]
    ref = subprocess.run([REF_BIN] + args, capture_output=True, text=True, timeout=60, cwd=str(tmp_path))
    got = subprocess.run([CLI] + args, capture_output=True, text=True, timeout=60, cwd=str(tmp_path))
    assert (got.returncode, got.stdout, got.stderr) == (ref.returncode, ref.stdout, ref.stderr)
