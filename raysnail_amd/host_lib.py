"""ctypes binding of libraysnail_host.so, the C++ host layer (include/raysnail.hpp).

The C++ layer holds the SDL front end (src/sdl_parser.rs restated) and the Rust-shaped object API;
these two C entry points expose it to Python:

* ``sdl_build(path, width, height, api, scene)`` -- parse an SDL file, apply the CLI's scene
  conventions (src/bin/raysnail.rs:340-373) and replay the world into any scene sink (a table of
  the rs_* scene-building functions: libraysnail_hip's own, or the CPU oracle's in the tests);
  returns the camera.
* ``sdl_render(path, width, height, settings)`` -- the same scene rendered on the GPU through the
  C++ World / TakePhotoSettings path. Raises if the library is missing: there is no fallback.
* ``sdl_render_passes(...)`` -- the CLI's progressive pass loop (render_passes); ``write_png`` --
  the CLI's quantisation (clamp * 255.5 -> u8) and PNG output.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi as A

_LIB = None
_F = C.CFUNCTYPE


class rsh_sink_api(C.Structure):
    """struct rsh_sink_api (include/raysnail.hpp): the scene-building half of the C-ABI as a table."""
    _fields_ = [(name, C.c_void_p) for name in (
        "material", "sphere", "aarect", "box", "quadric", "triangles", "intersection", "difference",
        "transformed", "world_add", "lights_add", "set_background", "set_time_range", "perlin", "image",
        "constant_medium", "last_error")]


def sink_api_of(lib, prefix: str) -> rsh_sink_api:
    """A sink table from a library exporting <prefix>material, <prefix>sphere, ... (rs_ or orc_)."""
    api = rsh_sink_api()
    for name, _ in rsh_sink_api._fields_:
        setattr(api, name, C.cast(getattr(lib, prefix + name), C.c_void_p).value)
    return api


def lib_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libraysnail_host.so")


def load() -> C.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    A.load()  # libraysnail_hip first (the host library links it through $ORIGIN)
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError(f"libraysnail_host.so not built ({path}); run __graft_entry__.build()")
    lib = C.CDLL(path)
    lib.rsh_sdl_build.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(rsh_sink_api), C.c_void_p,
                                  C.POINTER(A.rs_camera_desc)]
    lib.rsh_sdl_build.restype = C.c_int
    lib.rsh_sdl_render.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(A.rs_render_settings), C.c_void_p,
                                   C.POINTER(A.rs_render_stats)]
    lib.rsh_sdl_render.restype = C.c_int
    lib.rsh_sdl_render_passes.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                          C.c_int, C.c_void_p, C.c_void_p]
    lib.rsh_sdl_render_passes.restype = C.c_int
    lib.rsh_write_png.argtypes = [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]
    lib.rsh_write_png.restype = C.c_int
    lib.rsh_last_error.restype = C.c_char_p
    lib.rsh_obj_load.argtypes = [C.c_char_p, C.c_double, C.POINTER(C.c_double), C.c_double, C.c_int,
                                 C.POINTER(C.c_uint32), C.POINTER(C.POINTER(C.c_double)),
                                 C.POINTER(C.POINTER(C.c_double))]
    lib.rsh_obj_load.restype = C.c_int
    lib.rsh_perlin_tables.argtypes = [C.c_uint64, C.c_uint32, C.c_int, C.c_void_p, C.c_void_p]
    lib.rsh_perlin_tables.restype = C.c_int
    lib.rsh_png_load.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.POINTER(C.c_uint8))]
    lib.rsh_png_load.restype = C.c_int
    lib.rsh_free.argtypes = [C.c_void_p]
    _LIB = lib
    return lib


class HostError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _check(rc: int):
    if rc != 0:
        raise HostError(rc, load().rsh_last_error().decode())


def sdl_build(path: str, width: int, height: int, api: rsh_sink_api, scene) -> A.rs_camera_desc:
    cam = A.rs_camera_desc()
    _check(load().rsh_sdl_build(os.fsencode(path), width, height, C.byref(api), scene, C.byref(cam)))
    return cam


def sdl_render(path: str, width: int, height: int, settings: A.rs_render_settings):
    out = np.zeros((height, width, 4), dtype=np.float32)
    stats = A.rs_render_stats()
    _check(load().rsh_sdl_render(os.fsencode(path), width, height, C.byref(settings),
                                 out.ctypes.data_as(C.c_void_p), C.byref(stats)))
    return out, stats


def sdl_render_passes(path: str, width: int, height: int, samples: int, passes: int, seed: int,
                      adaptive: bool = False):
    """The CLI's pass loop (render_passes): combined image and per-pass [noise min, max, count]."""
    out = np.zeros((height, width, 4), dtype=np.float32)
    noise = np.zeros((passes, 3), dtype=np.float32)
    _check(load().rsh_sdl_render_passes(os.fsencode(path), width, height, samples, passes, seed, int(adaptive),
                                        out.ctypes.data_as(C.c_void_p), noise.ctypes.data_as(C.c_void_p)))
    return out, noise


def write_png(path: str, rgba: np.ndarray) -> None:
    rgba = np.ascontiguousarray(rgba, dtype=np.float32)
    h, w = rgba.shape[:2]
    _check(load().rsh_write_png(os.fsencode(path), rgba.ctypes.data_as(C.c_void_p), w, h))


def obj_load(path: str, scale: float, offset, rotation_angle: float, axis: int):
    """TriangleMesh::load's geometry: (n, 9) positions and (n, 9) vertex normals."""
    lib = load()
    n = C.c_uint32()
    pos, nrm = C.POINTER(C.c_double)(), C.POINTER(C.c_double)()
    _check(lib.rsh_obj_load(os.fsencode(path), float(scale), (C.c_double * 3)(*map(float, offset)),
                            float(rotation_angle), int(axis), C.byref(n), C.byref(pos), C.byref(nrm)))
    try:
        P = np.ctypeslib.as_array(pos, shape=(n.value * 9,)).copy().reshape(-1, 9) if n.value else np.zeros((0, 9))
        N = np.ctypeslib.as_array(nrm, shape=(n.value * 9,)).copy().reshape(-1, 9) if n.value else np.zeros((0, 9))
    finally:
        lib.rsh_free(pos)
        lib.rsh_free(nrm)
    return P, N


def perlin_tables(seed: int, point_count: int, vector: bool):
    """Perlin::new(point_count, vector, FastRng(seed)) tables: values and perm_x|perm_y|perm_z (uint32)."""
    values = np.zeros(point_count * (3 if vector else 1), dtype=np.float64)
    perms = np.zeros(3 * point_count, dtype=np.uint32)
    _check(load().rsh_perlin_tables(int(seed), int(point_count), int(vector), values.ctypes.data_as(C.c_void_p),
                                    perms.ctypes.data_as(C.c_void_p)))
    return values, perms


def png_load(path: str) -> np.ndarray:
    """Image::new: decoded (H, W, 3) uint8."""
    lib = load()
    w, h = C.c_uint32(), C.c_uint32()
    p = C.POINTER(C.c_uint8)()
    _check(lib.rsh_png_load(os.fsencode(path), C.byref(w), C.byref(h), C.byref(p)))
    try:
        return np.ctypeslib.as_array(p, shape=(h.value * w.value * 3,)).copy().reshape(h.value, w.value, 3)
    finally:
        lib.rsh_free(p)
