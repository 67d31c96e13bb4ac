"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from raysnail_amd import _abi as A
from raysnail_amd.api import World, realize, _check

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
# the same restatement calling glibc's sin / cos / pow instead of include/rs_crmath.h
GLIBC_LIB_PATH = os.path.join(HERE, "build", "liboracle_glibc.so")
_LIBS = {}


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def load(path: str = LIB_PATH) -> C.CDLL:
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    for name, (res, args) in A.SCENE_SIGNATURES.items():
        f = getattr(lib, "orc_" + name)
        f.restype, f.argtypes = res, args
    lib.orc_last_error.restype = C.c_char_p
    lib.orc_scene_create.restype = C.c_void_p
    lib.orc_scene_destroy.argtypes = [C.c_void_p]
    lib.orc_commit.argtypes = [C.c_void_p]
    lib.orc_commit.restype = C.c_int
    lib.orc_render.argtypes = [C.c_void_p, C.POINTER(A.rs_camera_desc), C.POINTER(A.rs_render_settings), C.c_void_p,
                               C.c_void_p, C.c_int, C.POINTER(A.rs_render_stats)]
    lib.orc_render.restype = C.c_int
    lib.orc_sample_radiance.argtypes = [C.c_void_p, C.POINTER(A.rs_camera_desc), C.POINTER(A.rs_render_settings),
                                        C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_double),
                                        C.POINTER(C.c_uint64)]
    lib.orc_sample_radiance.restype = C.c_int
    lib.orc_stream_key.restype = C.c_uint64
    lib.orc_stream_key.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32]
    lib.orc_rng_u32.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_uint32)]
    lib.orc_rng_u32_from_words.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]
    lib.orc_rng_gen.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]
    lib.orc_world_hit.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_double, C.c_double,
                                  C.c_double, C.POINTER(C.c_double)]
    lib.orc_world_hit.restype = C.c_int
    lib.orc_tf_apply.argtypes = [C.POINTER(A.rs_transform), C.c_uint32, C.POINTER(C.c_double), C.c_double, C.c_int,
                                 C.POINTER(C.c_double)]
    lib.orc_camera_ray.argtypes = [C.POINTER(A.rs_camera_desc), C.c_double, C.c_double, C.c_uint64,
                                   C.POINTER(C.c_double)]
    lib.orc_scatter.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint64,
                                C.POINTER(C.c_double)]
    lib.orc_scatter.restype = C.c_int
    lib.orc_set_trace.argtypes = [C.c_int]
    lib.orc_set_variant.argtypes = [C.c_int]
    lib.orc_set_axis_bits.argtypes = [C.c_uint64]
    lib.orc_chacha_block.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_uint32)]
    lib.orc_rtow_balls.argtypes = [C.c_uint64, C.POINTER(C.c_double), C.c_int]
    lib.orc_rtow_balls.restype = C.c_int
    lib.orc_rtow_scene.argtypes = [C.c_void_p, C.c_uint64]
    lib.orc_rtow_scene.restype = C.c_int
    _LIBS[path] = lib
    return lib


# Diagnostic semantics switches (oracle.cpp ORC_VAR_*): hypotheses about the code version behind the
# reference's own render. Every parity test runs with 0 (the checkout's semantics).
VAR_LIGHT_RADIUS = 1
VAR_LIGHT_FROM_POINT = 2
VAR_SORTED_ROOTS = 4
VAR_REF_TREE = 8
VAR_RECT_CLOSED_END = 16
VAR_TREE_FILE_ORDER = 32


class variant:
    """with variant(VAR_...): scenes committed and rendered inside use that semantics."""

    def __init__(self, bits: int, axis_bits: int = 0, path: str = LIB_PATH):
        self.lib, self.bits, self.axis_bits = load(path), bits, axis_bits

    def __enter__(self):
        self.lib.orc_set_variant(self.bits)
        self.lib.orc_set_axis_bits(self.axis_bits)
        return self

    def __exit__(self, *exc):
        self.lib.orc_set_variant(0)
        self.lib.orc_set_axis_bits(0)
        return False


class OracleScene:
    """The same World replayed into the CPU restatement (or, with world=None, filled by
    `fill(api, handle)` through a sink table -- e.g. the C++ SDL front end)."""

    def __init__(self, world: World = None, fill=None, lib_path: str = LIB_PATH, rtow_seed: int = None):
        """rtow_seed: the RTIOW final scene (examples/rtow_13_1.rs) built by the oracle's own C++
        generator (oracle/scene_gen.cpp), independent of raysnail_amd/scenes.py."""
        self.lib = load(lib_path)
        self.h = C.c_void_p(self.lib.orc_scene_create())
        if rtow_seed is not None:
            _check(self.lib, self.lib.orc_rtow_scene(self.h, rtow_seed), "orc_")
        elif world is not None:
            realize(world, self.lib, self.h, "orc_")
        else:
            from raysnail_amd.host_lib import sink_api_of
            self.api = sink_api_of(self.lib, "orc_")
            self.fill_result = fill(self.api, self.h)
        _check(self.lib, self.lib.orc_commit(self.h), "orc_")

    def __del__(self):
        try:
            self.lib.orc_scene_destroy(self.h)
        except Exception:
            pass

    def render(self, cam: A.rs_camera_desc, st: A.rs_render_settings, threads: int = 0, mask=None, out=None):
        H, W = cam.height, cam.width
        if out is None:
            out = np.zeros((H, W, 4), dtype=np.float32)
        mptr = None
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint8).reshape(H * W)
            mptr = mask.ctypes.data_as(C.c_void_p)
        stats = A.rs_render_stats()
        _check(self.lib, self.lib.orc_render(self.h, C.byref(cam), C.byref(st), mptr,
                                             out.ctypes.data_as(C.c_void_p), threads, C.byref(stats)), "orc_")
        return out, stats

    def sample_radiance(self, cam, st, x, y, s):
        out = (C.c_double * 3)()
        seg = C.c_uint64()
        _check(self.lib, self.lib.orc_sample_radiance(self.h, C.byref(cam), C.byref(st), x, y, s, out, C.byref(seg)),
               "orc_")
        return np.array(list(out)), seg.value

    def world_hit(self, o, d, time=0.0, tmin=1e-4, tmax=float("inf")):
        out = (C.c_double * 13)()
        _check(self.lib, self.lib.orc_world_hit(self.h, (C.c_double * 3)(*o), (C.c_double * 3)(*d), time, tmin, tmax,
                                                out), "orc_")
        return list(out)


def rtow_balls(seed: int = 7) -> np.ndarray:
    """The oracle's own RTIOW ball list (scene_gen.cpp): rows cx cy cz r kind checker r g b param 0 0."""
    lib = load()
    n = lib.orc_rtow_balls(seed, None, 0)
    out = np.zeros((n, 12))
    lib.orc_rtow_balls(seed, out.ctypes.data_as(C.POINTER(C.c_double)), n)
    return out
