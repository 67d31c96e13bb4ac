"""The C-ABI library loads without a GPU, exports exactly what include/raysnail_hip.h declares,
and validates input before touching the device. CPU only (no compute calls)."""
import ctypes as C
import os
import re

import pytest

from raysnail_amd import _abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "raysnail_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rs_[a-z_0-9]+)\s*\(", text)))


def test_header_lists_all_exports():
    assert header_symbols() == sorted(A.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(hip_lib):
    for name in header_symbols():
        assert hasattr(hip_lib, name), name
    assert hip_lib.rs_abi_version() == 3


def _scene(lib):
    h = C.c_void_p()
    assert lib.rs_scene_create(C.byref(h)) == 0
    return h


def test_invalid_inputs_return_codes_not_aborts(hip_lib):
    lib = hip_lib
    s = _scene(lib)
    d = A.rs_material_desc()
    d.kind = 42
    mid = C.c_int32()
    assert lib.rs_material(s, C.byref(d), C.byref(mid)) == A.RS_E_INVALID
    assert b"material" in lib.rs_last_error()
    out = C.c_uint32()
    assert lib.rs_sphere(s, A.D3(0, 0, 0), 1.0, None, 5, C.byref(out)) == A.RS_E_INVALID  # unknown material
    assert lib.rs_aarect(s, 1, 0.0, 1.0, 0.0, 0.0, 1.0, -1, C.byref(out)) == A.RS_E_INVALID  # a0 >= a1
    assert lib.rs_intersection(s, 7, 8, -1, C.byref(out)) == A.RS_E_INVALID
    assert lib.rs_scene_create(None) == A.RS_E_INVALID
    cam = A.rs_camera_desc()
    st = A.rs_render_settings()
    assert lib.rs_render(s, C.byref(cam), C.byref(st), None, None, None) == A.RS_E_INVALID
    lib.rs_scene_destroy(s)


def test_render_before_commit_is_state_error(hip_lib):
    lib = hip_lib
    s = _scene(lib)
    cam = A.rs_camera_desc(); cam.width = cam.height = 4
    st = A.rs_render_settings(); st.samples = 1; st.depth = 1
    import numpy as np
    out = np.zeros((4, 4, 4), np.float32)
    assert lib.rs_render(s, C.byref(cam), C.byref(st), None, out.ctypes.data, None) == A.RS_E_STATE
    lib.rs_scene_destroy(s)


def test_no_lights_with_pdf_material_is_rejected_at_commit(hip_lib):
    """list.rs:49-52 would panic on % 0; the ABI returns RS_E_NO_LIGHTS before any device work."""
    lib = hip_lib
    s = _scene(lib)
    d = A.rs_material_desc()
    d.kind = A.RS_MAT_LAMBERTIAN
    d.refractive = 1.0
    mid = C.c_int32()
    assert lib.rs_material(s, C.byref(d), C.byref(mid)) == 0
    h = C.c_uint32()
    assert lib.rs_sphere(s, A.D3(0, 0, 0), 1.0, None, mid.value, C.byref(h)) == 0
    assert lib.rs_world_add(s, h.value) == 0
    assert lib.rs_scene_commit(s) == A.RS_E_NO_LIGHTS
    lib.rs_scene_destroy(s)
