"""ctypes bindings for the MI355X renderer's two C ABIs.

  librt_host.so  include/rt_host.h  scene parser, camera, quantiser, PPM writer
  librt_hip.so   include/rt_hip.h   gfx950 kernels (the hot path)

Mirrors the reference's single entry point
``create_view_window_and_ray_trace`` (main.cpp:670) as :func:`render_scene`
and its ``main`` (main.cpp:60-657) as :func:`render_file`.  There is no CPU
fallback: when the HIP library or a device is missing these functions raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.environ.get("RTAMD_LIB_DIR") or os.path.join(PKG_DIR, "lib")   # A/B variants: lib_<x>/

RT_OK = 0
ERRORS = {-1: "invalid argument", -2: "no such HIP device", -3: "HIP runtime error",
          -4: "out of device memory", -5: "unsupported"}


class RTError(RuntimeError):
    pass


class rt_material(C.Structure):
    _fields_ = [("diffuse", C.c_float * 3), ("specular", C.c_float * 3), ("ka", C.c_float),
                ("kd", C.c_float), ("ks", C.c_float), ("n", C.c_float), ("opacity", C.c_float),
                ("eta", C.c_float)]


class rt_sphere_desc(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("radius", C.c_float), ("mat", rt_material),
                ("texture", C.c_int)]


class rt_face_desc(C.Structure):
    _fields_ = [("v", (C.c_float * 3) * 3), ("vn", (C.c_float * 3) * 3), ("vt", (C.c_float * 2) * 3),
                ("smooth", C.c_int), ("mat", rt_material), ("texture", C.c_int)]


class rt_light_desc(C.Structure):
    _fields_ = [("xyz", C.c_float * 3), ("w", C.c_float), ("color", C.c_float * 3)]


class rt_texture_desc(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("rgb", C.POINTER(C.c_ubyte))]


class rt_scene_desc(C.Structure):
    _fields_ = [("n_spheres", C.c_int), ("spheres", C.POINTER(rt_sphere_desc)),
                ("n_faces", C.c_int), ("faces", C.POINTER(rt_face_desc)),
                ("n_lights", C.c_int), ("lights", C.POINTER(rt_light_desc)),
                ("n_textures", C.c_int), ("textures", C.POINTER(rt_texture_desc)),
                ("bkg", C.c_float * 3), ("eta_bkg", C.c_float), ("epsilon", C.c_float),
                ("depth", C.c_int)]


class rt_camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("ul", C.c_float * 3), ("dh", C.c_float * 3),
                ("dv", C.c_float * 3)]


class rt_stats(C.Structure):
    _fields_ = [("primary", C.c_ulonglong), ("shadow", C.c_ulonglong),
                ("refraction", C.c_ulonglong), ("reflection", C.c_ulonglong),
                ("skip_trans", C.c_ulonglong), ("ub_back", C.c_ulonglong),
                ("kernel_ms", C.c_double), ("box_tests", C.c_ulonglong),
                ("face_tests", C.c_ulonglong), ("sphere_tests", C.c_ulonglong),
                ("shadow_known", C.c_ulonglong), ("bf_queries", C.c_ulonglong),
                ("stack_spills", C.c_ulonglong), ("bvh_build_ms", C.c_double)]

    def rays(self) -> int:
        return int(self.primary + self.shadow + self.refraction + self.reflection)

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_host = None
_hip = None

HOST_SYMBOLS = ["rth_parse_file", "rth_free", "rth_desc", "rth_set_depth", "rth_set_imsize",
                "rth_width", "rth_height", "rth_camera", "rth_quantize", "rth_write_ppm",
                "rth_output_path", "rth_row_set", "rth_ppm_open", "rth_ppm_write_rows", "rth_ppm_close",
                "rth_write_ppm_u8", "rth_ppm_write_rows_u8"]
HIP_SYMBOLS = ["rt_device_count", "rt_device_init", "rt_scene_create", "rt_scene_destroy", "rt_render_rows",
               "rt_render_rows_async", "rt_render_row_blocks_async", "rt_render_row_blocks", "rt_render_pixels",
               "rt_scene_last_stats", "rt_scene_prepare",
               "rt_scene_set_option", "rt_scene_debug_counters", "rt_scene_debug_wavelog", "rt_scene_debug_ub_pixels",
               "rt_deinterleave_rows", "rt_deinterleave_rows_u8", "rt_quantize_u8",
               "rt_strerror"]


def host_lib() -> C.CDLL:
    global _host
    if _host is None:
        path = os.path.join(LIB_DIR, "librt_host.so")
        if not os.path.exists(path):
            raise RTError(f"{path} missing: run `make -C simple-raytracer_amd` (or __graft_entry__.build())")
        L = C.CDLL(path)
        L.rth_parse_file.argtypes = [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
        L.rth_free.argtypes = [C.c_void_p]
        L.rth_desc.argtypes = [C.c_void_p]
        L.rth_desc.restype = C.POINTER(rt_scene_desc)
        L.rth_set_depth.argtypes = [C.c_void_p, C.c_int]
        L.rth_set_imsize.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.rth_width.argtypes = [C.c_void_p]
        L.rth_height.argtypes = [C.c_void_p]
        L.rth_camera.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(rt_camera)]
        L.rth_quantize.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p]
        L.rth_write_ppm.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.rth_output_path.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        if hasattr(L, "rth_ppm_open"):    # absent from round-1..3 libraries (A/B baselines)
            L.rth_ppm_open.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
            L.rth_ppm_write_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
            L.rth_ppm_close.argtypes = [C.c_void_p]
        if hasattr(L, "rth_write_ppm_u8"):   # absent from round-1..4 libraries (A/B baselines)
            L.rth_write_ppm_u8.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
            L.rth_ppm_write_rows_u8.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        if hasattr(L, "rth_row_set"):     # absent from round-1 libraries (A/B baselines)
            L.rth_row_set.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_int)] * 4
        _host = L
    return _host


def hip_lib() -> C.CDLL:
    """The HIP layer.  Raises (never falls back) when it is missing."""
    global _hip
    if _hip is None:
        path = os.path.join(LIB_DIR, "librt_hip.so")
        if not os.path.exists(path):
            raise RTError(f"{path} missing: the HIP path is required (no CPU fallback)")
        # One HIP runtime per process: torch ships its own libamdhip64.so with
        # the same soname as /opt/rocm's.  Whichever is loaded first serves
        # both; loading ours first leaves torch without devices, so let torch
        # load its runtime first when it is installed.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(path)
        L.rt_device_count.restype = C.c_int
        if hasattr(L, "rt_device_init"):        # absent from round-1..4 libraries (A/B baselines)
            L.rt_device_init.argtypes = [C.c_int]
        L.rt_scene_create.argtypes = [C.c_int, C.POINTER(rt_scene_desc), C.POINTER(C.c_void_p)]
        L.rt_scene_destroy.argtypes = [C.c_void_p]
        L.rt_render_rows.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                     C.c_int, C.c_void_p, C.POINTER(rt_stats)]
        L.rt_render_rows_async.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int,
                                           C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.rt_render_row_blocks_async.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int,
                                                 C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                                 C.c_void_p]
        L.rt_render_row_blocks.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                           C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(rt_stats)]
        if hasattr(L, "rt_render_pixels"):   # absent from round-1/2 libraries (A/B baselines)
            L.rt_render_pixels.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_void_p,
                                           C.c_int, C.c_void_p, C.POINTER(rt_stats)]
        L.rt_scene_last_stats.argtypes = [C.c_void_p, C.POINTER(rt_stats)]
        L.rt_scene_prepare.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int]
        L.rt_scene_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
        if hasattr(L, "rt_scene_debug_ub_pixels"):  # absent from round-1..3 libraries (A/B baselines)
            L.rt_scene_debug_ub_pixels.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
        if hasattr(L, "rt_scene_debug_wavelog"):   # absent from round-1..3 libraries (A/B baselines)
            L.rt_scene_debug_wavelog.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
        if hasattr(L, "rt_deinterleave_rows"):
            L.rt_deinterleave_rows.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                               C.c_void_p, C.c_void_p]
        if hasattr(L, "rt_deinterleave_rows_u8"):  # absent from round-1..4 libraries (A/B baselines)
            L.rt_deinterleave_rows_u8.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                  C.c_void_p, C.c_void_p]
        if hasattr(L, "rt_quantize_u8"):           # absent from round-1..3 libraries (A/B baselines)
            L.rt_quantize_u8.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
        L.rt_scene_set_option.argtypes = [C.c_void_p, C.c_char_p, C.c_longlong]
        L.rt_strerror.argtypes = [C.c_int]
        L.rt_strerror.restype = C.c_char_p
        _hip = L
    return _hip


def _check(rc: int, what: str) -> None:
    if rc != RT_OK:
        raise RTError(f"{what}: {ERRORS.get(rc, rc)} ({rc})")


class ParseError(RTError):
    """The reference would abort (uncaught exception).  .lines = its std::cerr output."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.lines = msg.split("\n")


class MissingCommand(RTError):
    """The reference would print .message on stdout and exit 0 without an image."""


class HostScene:
    """A parsed scene file (main.cpp:88-602).  Texture paths resolve against
    the current directory, or against `cwd` when given."""

    def __init__(self, path: str, cwd: str | None = None):
        L = host_lib()
        h = C.c_void_p()
        buf = C.create_string_buffer(1 << 16)
        old = os.getcwd()
        try:
            if cwd:
                os.chdir(cwd)
            rc = L.rth_parse_file(os.fsencode(path), C.byref(h), buf, len(buf))
        finally:
            os.chdir(old)
        msg = buf.value.decode(errors="replace")
        if rc > 0:
            raise MissingCommand(msg)
        if rc < 0:
            raise ParseError(rc, msg)
        self._h = h
        self.path = path

    def close(self) -> None:
        if getattr(self, "_h", None):
            try:
                host_lib().rth_free(self._h)
            except Exception:        # interpreter shutdown
                pass
            self._h = None

    __del__ = close

    @property
    def desc(self) -> rt_scene_desc:
        return host_lib().rth_desc(self._h).contents

    def set_depth(self, depth: int) -> None:
        host_lib().rth_set_depth(self._h, depth)

    def set_imsize(self, w: int, h: int) -> None:
        host_lib().rth_set_imsize(self._h, w, h)

    @property
    def width(self) -> int:
        return host_lib().rth_width(self._h)

    @property
    def height(self) -> int:
        return host_lib().rth_height(self._h)

    def camera(self, W: int | None = None, H: int | None = None) -> rt_camera:
        cam = rt_camera()
        _check(host_lib().rth_camera(self._h, W or self.width, H or self.height, C.byref(cam)),
               "rth_camera")
        return cam


def quantize(rgb: np.ndarray) -> np.ndarray:
    """main.cpp:760-762: the reference's size_t pixel values (as int64)."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.empty(a.shape, dtype=np.int64)
    host_lib().rth_quantize(a.ctypes.data, a.size, out.ctypes.data)
    return out


def quantize_u8_device(rgb_ptr: int, n: int, out_ptr: int, flag_ptr: int, stream: int = 0) -> None:
    """rt_quantize_u8 on device buffers: the P3 writer's values of n floats
    as bytes; bit 0 of the uint32 at flag_ptr is set when a value is not 0..255."""
    _check(hip_lib().rt_quantize_u8(C.c_void_p(rgb_ptr), n, C.c_void_p(out_ptr), C.c_void_p(flag_ptr),
                                    C.c_void_p(stream)), "rt_quantize_u8")


def deinterleave_rows_device(gathered_ptr: int, world: int, rows_per: int, W: int, H: int, block: int,
                             image_ptr: int, u8: bool, stream: int = 0) -> None:
    """rt_deinterleave_rows(_u8) on device buffers: `world` gathered row sets
    (rows_per x W x 3 floats or bytes each) -> the H x W x 3 image in row order."""
    L = hip_lib()
    f = L.rt_deinterleave_rows_u8 if u8 else L.rt_deinterleave_rows
    _check(f(C.c_void_p(gathered_ptr), world, rows_per, W, H, block, C.c_void_p(image_ptr), C.c_void_p(stream)),
           "rt_deinterleave_rows")


def write_ppm(path: str, rgb: np.ndarray, threads: int = 0) -> None:
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    H, W = a.shape[:2]
    if host_lib().rth_write_ppm(os.fsencode(path), a.ctypes.data, W, H, threads) != 0:
        raise RTError(f"cannot write {path}")


def write_ppm_u8(path: str, v: np.ndarray, threads: int = 0) -> None:
    """The P3 file from the pixel values as bytes (rth_write_ppm_u8): the
    values rt_quantize_u8 makes when all are 0..255."""
    a = np.ascontiguousarray(v, dtype=np.uint8)
    H, W = a.shape[:2]
    if host_lib().rth_write_ppm_u8(os.fsencode(path), a.ctypes.data, W, H, threads) != 0:
        raise RTError(f"cannot write {path}")


def write_ppm_blocks(path: str, rgb: np.ndarray, block: int, threads: int = 0) -> None:
    """The P3 file written in blocks of `block` rows (rth_ppm_open / rth_ppm_write_rows /
    rth_ppm_close): byte-identical to write_ppm."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    H, W = a.shape[:2]
    L = host_lib()
    h = C.c_void_p()
    if L.rth_ppm_open(os.fsencode(path), W, H, threads, C.byref(h)) != 0:
        raise RTError(f"cannot open {path}")
    ok = True
    for y in range(0, H, block):
        n = min(block, H - y)
        ok = L.rth_ppm_write_rows(h, a[y:y + n].ctypes.data, n) == 0 and ok
    if L.rth_ppm_close(h) != 0 or not ok:
        raise RTError(f"cannot write {path}")


def output_path(scene_path: str) -> str:
    buf = C.create_string_buffer(4096)
    host_lib().rth_output_path(os.fsencode(scene_path), buf, len(buf))
    return buf.value.decode()


def device_count() -> int:
    return hip_lib().rt_device_count()


class GpuScene:
    """A scene uploaded to one HIP device (rt_scene_create)."""

    def __init__(self, host: HostScene, device: int = 0):
        L = hip_lib()
        h = C.c_void_p()
        _check(L.rt_scene_create(device, host.desc, C.byref(h)), "rt_scene_create")
        self._h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None):
            try:
                hip_lib().rt_scene_destroy(self._h)
            except Exception:        # interpreter shutdown
                pass
            self._h = None

    __del__ = close

    def set_option(self, key: str, value: int) -> None:
        _check(hip_lib().rt_scene_set_option(self._h, key.encode(), int(value)), "rt_scene_set_option")

    def render_rows(self, cam: rt_camera, W: int, H: int, y0: int, y1: int, out=None):
        """Synchronous render of rows [y0, y1).  `out` may be a numpy array
        (host) or an int device pointer; returns (out, rt_stats)."""
        st = rt_stats()
        if out is None:
            # into a device buffer filled with NaN first: a pixel the kernel
            # never wrote shows up (a host buffer goes through the library's
            # staging buffer, which may still hold an earlier render)
            import torch
            dev = torch.full((y1 - y0, W, 3), float("nan"), dtype=torch.float32, device=f"cuda:{self.device}")
            # the fill runs on torch's stream, the render on the scene's own
            # (non-blocking) stream: nothing orders the two but this wait
            torch.cuda.synchronize(self.device)
            _check(hip_lib().rt_render_rows(self._h, C.byref(cam), W, H, y0, y1, C.c_void_p(dev.data_ptr()),
                                            C.byref(st)), "rt_render_rows")
            return dev.cpu().numpy(), st
        ptr = out if isinstance(out, int) else out.ctypes.data
        _check(hip_lib().rt_render_rows(self._h, C.byref(cam), W, H, y0, y1, C.c_void_p(ptr),
                                        C.byref(st)), "rt_render_rows")
        return out, st

    def render_rows_async(self, cam: rt_camera, W: int, H: int, y0: int, y1: int, dev_ptr: int,
                          stream: int | None = None) -> None:
        _check(hip_lib().rt_render_rows_async(self._h, C.byref(cam), W, H, y0, y1,
                                              C.c_void_p(dev_ptr), C.c_void_p(stream or 0)),
               "rt_render_rows_async")

    def render_row_blocks_async(self, cam: rt_camera, W: int, H: int, y0: int, block: int, step: int,
                                nrows: int, dev_ptr: int, stream: int | None = None) -> None:
        _check(hip_lib().rt_render_row_blocks_async(self._h, C.byref(cam), W, H, y0, block, step, nrows,
                                                    C.c_void_p(dev_ptr), C.c_void_p(stream or 0)),
               "rt_render_row_blocks_async")

    def render_row_blocks(self, cam: rt_camera, W: int, H: int, y0: int, block: int, step: int, nrows: int,
                          out=None):
        """Synchronous block-interleaved row set into a numpy array (host):
        local row k is image row y0 + (k // block) * step + k % block."""
        st = rt_stats()
        if out is None:
            out = np.empty((nrows, W, 3), dtype=np.float32)
        _check(hip_lib().rt_render_row_blocks(self._h, C.byref(cam), W, H, y0, block, step, nrows,
                                              C.c_void_p(out.ctypes.data), C.byref(st)),
               "rt_render_row_blocks")
        return out, st

    def render_pixels(self, cam: rt_camera, W: int, H: int, xy):
        """rt_render_pixels: the colours of the listed (x, y) pixels of the
        W x H image -> (float32 [n, 3], rt_stats of those pixels' rays)."""
        xy = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1, 2)
        out = np.empty((len(xy), 3), dtype=np.float32)
        st = rt_stats()
        _check(hip_lib().rt_render_pixels(self._h, C.byref(cam), W, H, C.c_void_p(xy.ctypes.data), len(xy),
                                          C.c_void_p(out.ctypes.data), C.byref(st)), "rt_render_pixels")
        return out, st

    def prepare(self, cam: rt_camera, W: int, H: int) -> None:
        """rt_scene_prepare: BVH for this camera + every slot's buffers, no render."""
        _check(hip_lib().rt_scene_prepare(self._h, C.byref(cam), W, H), "rt_scene_prepare")

    def last_stats(self) -> rt_stats:
        st = rt_stats()
        _check(hip_lib().rt_scene_last_stats(self._h, C.byref(st)), "rt_scene_last_stats")
        return st

    def debug_counters(self) -> list[int]:
        """Raw device counters of the last render (rt_scene_debug_counters)."""
        buf = (C.c_ulonglong * 64)()
        rc = hip_lib().rt_scene_debug_counters(self._h, buf, 64)
        if rc == -1:                  # libraries of rounds 1-4 (A/B baselines) have 32 / 40 / 48 slots
            rc = hip_lib().rt_scene_debug_counters(self._h, buf, 48)
        if rc == -1:
            rc = hip_lib().rt_scene_debug_counters(self._h, buf, 40)
        if rc == -1:
            rc = hip_lib().rt_scene_debug_counters(self._h, buf, 32)
        _check(rc, "rt_scene_debug_counters")
        return list(buf)

    def debug_ub_pixels(self, cap: int = 4096):
        """The last render's back()-of-an-empty-stack events (main.cpp:1028):
        (events, int32 array of the first min(events, cap) events' pixels as
        (x, y) image coordinates) -- rt_scene_debug_ub_pixels."""
        import numpy as np
        buf = (C.c_int * (2 * cap))()
        n = hip_lib().rt_scene_debug_ub_pixels(self._h, buf, cap)
        if n < 0:
            _check(n, "rt_scene_debug_ub_pixels")
        k = min(n, cap)
        return n, np.array(buf[:2 * k], dtype=np.int32).reshape(k, 2)

    def debug_wavelog(self, max_waves: int = 16384) -> list[list[int]] | None:
        """Per-wave timeline of the last render (rt_scene_debug_wavelog; RT_PROF
        builds only, else None): [start, prologue done, drained, end, first
        trace step done, HW_ID << 32 | XCC_ID, iterations, refills] per wave."""
        L = hip_lib()
        if not hasattr(L, "rt_scene_debug_wavelog"):
            return None
        buf = (C.c_ulonglong * (8 * max_waves))()
        n = L.rt_scene_debug_wavelog(self._h, buf, 8 * max_waves)
        if n < 0:
            return None
        return [list(buf[i:i + 8]) for i in range(0, n, 8)]


def render_scene(path: str, cwd: str | None = None, device: int = 0, depth: int | None = None,
                 imsize: tuple[int, int] | None = None, rows: tuple[int, int] | None = None,
                 options: dict | None = None):
    """Parse + render a scene file on the GPU: returns (float32 HxWx3, rt_stats).
    `options` are rt_scene_set_option knobs, e.g. {"accel": 1}."""
    hs = HostScene(path, cwd=cwd)
    if depth is not None:
        hs.set_depth(depth)
    if imsize is not None:
        hs.set_imsize(*imsize)
    W, H = hs.width, hs.height
    cam = hs.camera(W, H)
    y0, y1 = rows if rows else (0, H)
    gs = GpuScene(hs, device)
    for k, v in (options or {}).items():
        gs.set_option(k, v)
    try:
        img, st = gs.render_rows(cam, W, H, y0, y1)
    finally:
        gs.close()
        hs.close()
    return img, st


def render_file(path: str, device: int = 0) -> str:
    """The reference's main(): render `path` and write <stem>.ppm; returns it."""
    img, _ = render_scene(path, device=device)
    out = output_path(path)
    write_ppm(out, img)
    return out
