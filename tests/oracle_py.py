"""ctypes access to the CPU oracle (oracle/liboracle.so) -- TEST CHECKER ONLY.

The oracle restates the reference's path on the CPU (oracle/rt_oracle.c);
tests use it to check the HIP path, never as the thing under test.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-C", ORACLE_DIR, "all"], check=True, stdout=subprocess.DEVNULL)
        L = C.CDLL(path)
        L.oracle_load.argtypes = [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
        L.oracle_free.argtypes = [C.c_void_p]
        L.oracle_width.argtypes = [C.c_void_p]
        L.oracle_height.argtypes = [C.c_void_p]
        L.oracle_set_depth.argtypes = [C.c_void_p, C.c_int]
        L.oracle_render_rows.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                         C.c_void_p, C.c_void_p]
        L.oracle_render_pixels.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                           C.c_void_p, C.c_void_p]
        L.oracle_write_ppm.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
        L.oracle_quantize.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p]
        L.oracle_counts_objects.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                            C.POINTER(C.c_int)]
        L.oracle_object.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_light.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_globals.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_camera.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.oracle_texture.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                     C.POINTER(C.POINTER(C.c_ubyte))]
        _lib = L
    return _lib


class OracleScene:
    def __init__(self, path: str, cwd: str | None = None):
        h = C.c_void_p()
        err = C.create_string_buffer(1024)
        old = os.getcwd()
        try:
            if cwd:
                os.chdir(cwd)
            rc = lib().oracle_load(os.fsencode(path), C.byref(h), err, len(err))
        finally:
            os.chdir(old)
        self.rc = rc
        self.msg = err.value.decode()
        self._h = h if rc == 0 else None

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_free(self._h)
            self._h = None

    @property
    def width(self) -> int:
        return lib().oracle_width(self._loaded())

    @property
    def height(self) -> int:
        return lib().oracle_height(self._loaded())

    def set_depth(self, d: int) -> None:
        lib().oracle_set_depth(self._loaded(), d)

    def _loaded(self):
        if not self._h:
            raise RuntimeError(f"scene not loaded (rc {self.rc}): {self.msg}")
        return self._h

    def counts(self):
        nf, ns, nl = C.c_int(), C.c_int(), C.c_int()
        lib().oracle_counts_objects(self._loaded(), C.byref(nf), C.byref(ns), C.byref(nl))
        return nf.value, ns.value, nl.value

    def objects(self) -> np.ndarray:
        nf, ns, _ = self.counts()
        out = np.zeros((nf + ns, 48), dtype=np.float32)
        for i in range(nf + ns):
            lib().oracle_object(self._loaded(), i, out[i].ctypes.data)
        return out

    def lights(self) -> np.ndarray:
        _, _, nl = self.counts()
        out = np.zeros((nl, 8), dtype=np.float32)
        for i in range(nl):
            lib().oracle_light(self._loaded(), i, out[i].ctypes.data)
        return out

    def globals(self) -> np.ndarray:
        out = np.zeros(6, dtype=np.float32)
        lib().oracle_globals(self._loaded(), out.ctypes.data)
        return out

    def texture(self, i: int) -> np.ndarray:
        w, h, p = C.c_int(), C.c_int(), C.POINTER(C.c_ubyte)()
        lib().oracle_texture(self._loaded(), i, C.byref(w), C.byref(h), C.byref(p))
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()

    def camera(self, W: int, H: int) -> np.ndarray:
        out = np.zeros(12, dtype=np.float32)
        lib().oracle_camera(self._loaded(), W, H, out.ctypes.data)
        return out

    def render(self, W: int | None = None, H: int | None = None, rows=None, threads: int = 0):
        """-> (float32 [len(rows), W, 3], counts dict)"""
        W = W or self.width
        H = H or self.height
        rows = np.arange(H, dtype=np.int32) if rows is None else np.asarray(rows, dtype=np.int32)
        out = np.empty((len(rows), W, 3), dtype=np.float32)
        cnt = np.zeros(6, dtype=np.int64)
        lib().oracle_render_rows(self._loaded(), W, H, rows.ctypes.data, len(rows), threads, out.ctypes.data,
                                 cnt.ctypes.data)
        names = ["primary", "shadow", "refraction", "reflection", "skip_trans", "ub_back"]
        return out, dict(zip(names, (int(c) for c in cnt)))

    def render_pixels(self, W: int, H: int, xy, threads: int = 0):
        """Pixels (x, y) of the W x H image -> (float32 [n, 3], counts dict)."""
        xy = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1, 2)
        out = np.empty((len(xy), 3), dtype=np.float32)
        cnt = np.zeros(6, dtype=np.int64)
        lib().oracle_render_pixels(self._loaded(), W, H, xy.ctypes.data, len(xy), threads, out.ctypes.data,
                                   cnt.ctypes.data)
        names = ["primary", "shadow", "refraction", "reflection", "skip_trans", "ub_back"]
        return out, dict(zip(names, (int(c) for c in cnt)))


def quantize(rgb: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.empty(a.shape, dtype=np.int64)
    lib().oracle_quantize(a.ctypes.data, a.size, out.ctypes.data)
    return out


def ppm_bytes(rgb: np.ndarray) -> bytes:
    """The reference's P3 text for a float image (via the oracle writer)."""
    import tempfile
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    with tempfile.NamedTemporaryFile(suffix=".ppm", delete=False) as f:
        path = f.name
    try:
        lib().oracle_write_ppm(os.fsencode(path), a.ctypes.data, a.shape[1], a.shape[0])
        return open(path, "rb").read()
    finally:
        os.remove(path)
