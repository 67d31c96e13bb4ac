"""ctypes mirror of include/raysnail_hip.h and the loader for libraysnail_hip.so.

The library is built in-tree (raysnail_amd/lib/libraysnail_hip.so, see csrc/Makefile). There is
no fallback: if the shared object is missing or fails to load, import of the GPU path raises.
"""
from __future__ import annotations

import ctypes as C
import os

RS_OK = 0
RS_E_INVALID = -1
RS_E_NO_LIGHTS = -2
RS_E_HIP = -3
RS_E_STATE = -4
RS_E_UNSUPPORTED = -5
RS_E_NOMEM = -6

RS_TEX_SOLID = 0
RS_TEX_CHECKER = 1
RS_TEX_PERLIN = 2
RS_TEX_IMAGE = 3

RS_PERLIN_NORMAL = 0
RS_PERLIN_TURBULENCE = 1
RS_PERLIN_MARBLE = 2
RS_SMOOTH_NONE = 0
RS_SMOOTH_LINEAR = 1
RS_SMOOTH_HERMITE = 2

RS_MAT_LAMBERTIAN = 0
RS_MAT_METAL = 1
RS_MAT_DIFFUSE_METAL = 2
RS_MAT_DIELECTRIC = 3
RS_MAT_DIFFUSE_LIGHT = 4
RS_MAT_MIXED = 5
RS_MAT_ISOTROPIC = 6
RS_MAT_BLINN_PHONG = 7
RS_NO_MATERIAL = -1

RS_PLANE_XY = 0
RS_PLANE_XZ = 1
RS_PLANE_YZ = 2

RS_TF_TRANSLATE = 0
RS_TF_ROTATE_X = 1
RS_TF_ROTATE_Y = 2
RS_TF_ROTATE_Z = 3
RS_TF_SCALE = 4

RS_MODE_AUTO = 0
RS_MODE_MEGAKERNEL = 1
RS_MODE_WAVEFRONT = 2


class rs_texture_desc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("data", C.c_int32), ("even", C.c_float * 4), ("odd", C.c_float * 4),
                ("scale", C.c_double)]


class rs_material_desc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("glass", C.c_int32), ("texture", rs_texture_desc), ("refractive", C.c_double),
                ("exponent", C.c_double), ("multiplier", C.c_double), ("mix_a", C.c_int32), ("mix_b", C.c_int32),
                ("mix_p", C.c_double), ("phong_factor", C.c_double), ("phong_exponent", C.c_int32),
                ("_pad", C.c_int32), ("k_specular", C.c_double)]


class rs_perlin_desc(C.Structure):
    _fields_ = [("point_count", C.c_uint32), ("vector", C.c_int32), ("smooth", C.c_int32), ("type", C.c_int32),
                ("depth", C.c_uint32), ("_pad", C.c_int32), ("scale", C.c_double),
                ("values", C.POINTER(C.c_double)), ("perm_x", C.POINTER(C.c_uint32)),
                ("perm_y", C.POINTER(C.c_uint32)), ("perm_z", C.POINTER(C.c_uint32))]


class rs_transform(C.Structure):
    _fields_ = [("kind", C.c_int32), ("_pad", C.c_int32), ("v", C.c_double * 3)]


class rs_camera_desc(C.Structure):
    _fields_ = [("look_from", C.c_double * 3), ("look_at", C.c_double * 3), ("vup", C.c_double * 3),
                ("fov", C.c_double), ("aperture", C.c_double), ("focus", C.c_double), ("shutter", C.c_double),
                ("width", C.c_uint32), ("height", C.c_uint32)]


class rs_render_settings(C.Structure):
    _fields_ = [("samples", C.c_uint32), ("depth", C.c_uint32), ("gamma", C.c_int32), ("mode", C.c_int32),
                ("seed", C.c_uint64), ("pass_", C.c_uint32), ("row_begin", C.c_uint32), ("row_end", C.c_uint32),
                ("row_step", C.c_uint32)]


class rs_noise_stats(C.Structure):
    _fields_ = [("min", C.c_float), ("max", C.c_float), ("count", C.c_uint64)]


class rs_render_stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("ms", C.c_double), ("path_ms", C.c_double),
                ("launches", C.c_uint32), ("kernel_launches", C.c_uint32), ("kernel_ms", C.c_double),
                ("kernel_bytes", C.c_uint64), ("kernel_id", C.c_int32), ("tree_arity", C.c_int32)]


class rs_scene_info(C.Structure):
    _fields_ = [("tree_arity", C.c_int32), ("ref_order", C.c_int32), ("scene_mode", C.c_int32),
                ("tree_depth", C.c_int32), ("stack_need", C.c_int32), ("stack_lds", C.c_int32),
                ("n_nodes", C.c_uint64), ("n_objects", C.c_uint64), ("n_world", C.c_uint64),
                ("n_devices", C.c_int32), ("class_mask", C.c_uint32)]


KERNEL_NAMES = {0: None, 1: "k_path_mega", 2: "k_wf_extend", 3: "k_wfs_extend"}


D3 = C.c_double * 3
F3 = C.c_float * 3
VP = C.c_void_p
U32P = C.POINTER(C.c_uint32)
I32P = C.POINTER(C.c_int32)

# (name suffix, restype, argtypes) shared by libraysnail_hip (prefix "rs_") and the test oracle
# (prefix "orc_", oracle/binding.py) so one scene realisation drives both.
SCENE_SIGNATURES = {
    "material": (C.c_int, [VP, C.POINTER(rs_material_desc), I32P]),
    "sphere": (C.c_int, [VP, C.POINTER(C.c_double), C.c_double, C.POINTER(C.c_double), C.c_int32, U32P]),
    "aarect": (C.c_int, [VP, C.c_int32, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, C.c_int32, U32P]),
    "box": (C.c_int, [VP, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int32, U32P]),
    "quadric": (C.c_int, [VP, C.POINTER(C.c_double), C.c_int32, U32P]),
    "triangles": (C.c_int, [VP, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint32, C.c_int32, U32P]),
    "intersection": (C.c_int, [VP, C.c_uint32, C.c_uint32, C.c_int32, U32P]),
    "difference": (C.c_int, [VP, C.c_uint32, C.c_uint32, C.c_int32, U32P]),
    "transformed": (C.c_int, [VP, C.c_uint32, C.POINTER(rs_transform), C.c_uint32, U32P]),
    "world_add": (C.c_int, [VP, C.c_uint32]),
    "lights_add": (C.c_int, [VP, C.c_uint32]),
    "set_background": (C.c_int, [VP, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "set_time_range": (C.c_int, [VP, C.c_double, C.c_double]),
    "perlin": (C.c_int, [VP, C.POINTER(rs_perlin_desc), I32P]),
    "image": (C.c_int, [VP, C.c_void_p, C.c_uint32, C.c_uint32, I32P]),
    "constant_medium": (C.c_int, [VP, C.c_uint32, C.POINTER(C.c_float), C.c_double, U32P]),
}

# rs_row_callback: (user, y, row_rgba, width)
ROW_CALLBACK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32, C.POINTER(C.c_float), C.c_uint32)

_LIB = None
ABI_VERSION = 6  # include/raysnail_hip.h RS_ABI_VERSION


def lib_path() -> str:
    # RS_HIP_LIB: a dev variant of the same library (tools/build_variant.sh), e.g. to bisect in tests
    return os.environ.get("RS_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                        "libraysnail_hip.so")


def load() -> C.CDLL:
    """Load libraysnail_hip.so (in-tree build). Raises if it is missing: no fallback path."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError(f"libraysnail_hip.so not built ({path}); run __graft_entry__.build() "
                           "or make -C raysnail_amd/csrc")
    lib = C.CDLL(path)
    for name, (res, args) in SCENE_SIGNATURES.items():
        f = getattr(lib, "rs_" + name)
        f.restype, f.argtypes = res, args
    lib.rs_abi_version.restype = C.c_int
    lib.rs_last_error.restype = C.c_char_p
    lib.rs_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.rs_stream_key.restype = C.c_uint64
    lib.rs_stream_key.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32]
    lib.rs_medium_uniform.restype = C.c_double
    lib.rs_medium_uniform.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    lib.rs_scene_create.argtypes = [C.POINTER(VP)]
    lib.rs_scene_destroy.argtypes = [VP]
    lib.rs_scene_commit.argtypes = [VP]
    lib.rs_combine_pixels_device.argtypes = [VP, VP, C.c_uint64, C.c_float, VP]
    lib.rs_combine_pixels_device.restype = C.c_int
    lib.rs_noise_map_device.argtypes = [VP, C.c_uint32, C.c_uint32, C.c_float, VP, VP, C.POINTER(rs_noise_stats)]
    lib.rs_noise_map_device.restype = C.c_int
    lib.rs_noise_map.argtypes = [VP, C.c_uint32, C.c_uint32, C.c_float, VP, C.POINTER(rs_noise_stats)]
    lib.rs_noise_map.restype = C.c_int
    lib.rs_probe_samples.argtypes = [VP, C.POINTER(rs_camera_desc), C.POINTER(rs_render_settings), C.c_uint32,
                                     C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    lib.rs_probe_samples.restype = C.c_int
    lib.rs_render.argtypes = [VP, C.POINTER(rs_camera_desc), C.POINTER(rs_render_settings), VP, VP,
                              C.POINTER(rs_render_stats)]
    lib.rs_render_device.argtypes = [VP, C.POINTER(rs_camera_desc), C.POINTER(rs_render_settings), VP, VP, VP,
                                     C.POINTER(rs_render_stats)]
    lib.rs_render_device_passes.argtypes = [VP, C.POINTER(rs_camera_desc), C.POINTER(rs_render_settings), C.c_uint32,
                                            C.POINTER(VP), VP, C.POINTER(rs_render_stats)]
    lib.rs_render_device_passes.restype = C.c_int
    lib.rs_probe_world_hit.argtypes = [VP, VP, C.c_uint32, C.c_double, C.c_double, VP]
    lib.rs_scene_get_info.argtypes = [VP, C.POINTER(rs_scene_info)]
    lib.rs_scene_commit_devices.argtypes = [VP, C.POINTER(C.c_int), C.c_int]
    lib.rs_scene_set_lanes.argtypes = [VP, C.c_uint32]
    lib.rs_scene_set_frames_in_flight.argtypes = [VP, C.c_uint32]
    lib.rs_render_rows.argtypes = [VP, C.POINTER(rs_camera_desc), C.POINTER(rs_render_settings), VP, VP, C.c_uint32,
                                   ROW_CALLBACK, VP, C.POINTER(rs_render_stats)]
    lib.rs_render_rows.restype = C.c_int
    lib.rs_scene_set_workspace.argtypes = [VP, C.c_uint64, C.c_uint64]
    for fn in ("rs_probe_world_hit", "rs_scene_get_info", "rs_scene_set_lanes", "rs_scene_set_frames_in_flight",
               "rs_scene_set_workspace", "rs_scene_commit_devices", "rs_scene_create", "rs_scene_destroy",
               "rs_scene_commit", "rs_render", "rs_render_device", "rs_device_count"):
        getattr(lib, fn).restype = C.c_int
    if lib.rs_abi_version() != ABI_VERSION:
        raise RuntimeError("libraysnail_hip.so ABI mismatch")
    _LIB = lib
    return lib


# every symbol include/raysnail_hip.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "rs_abi_version", "rs_last_error", "rs_device_count", "rs_stream_key", "rs_medium_uniform", "rs_scene_create",
    "rs_scene_destroy", "rs_perlin", "rs_image", "rs_material", "rs_sphere", "rs_aarect", "rs_box", "rs_quadric", "rs_triangles", "rs_intersection",
    "rs_difference", "rs_transformed", "rs_constant_medium", "rs_world_add", "rs_lights_add", "rs_set_background", "rs_set_time_range",
    "rs_scene_commit", "rs_scene_commit_devices", "rs_scene_get_info", "rs_scene_set_lanes",
    "rs_scene_set_frames_in_flight", "rs_scene_set_workspace", "rs_render", "rs_render_rows", "rs_render_device", "rs_render_device_passes", "rs_combine_pixels_device", "rs_noise_map_device", "rs_noise_map",
    "rs_probe_world_hit", "rs_probe_samples",
]
