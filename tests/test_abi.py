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
    assert hip_lib.rs_abi_version() == 6


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
    # rs_render_device_passes: argument checks before any device work (no GPU needed)
    ptrs = (C.c_void_p * 2)(C.c_void_p(0x1000), C.c_void_p(0x2000))
    assert lib.rs_render_device_passes(s, C.byref(cam), C.byref(st), 2, ptrs, None, None) == A.RS_E_STATE
    assert lib.rs_render_device_passes(None, C.byref(cam), C.byref(st), 2, ptrs, None, None) == A.RS_E_INVALID
    assert lib.rs_render_device_passes(s, C.byref(cam), C.byref(st), 2, None, None, None) == A.RS_E_INVALID
    holes = (C.c_void_p * 2)(C.c_void_p(0x1000), None)
    assert lib.rs_render_device_passes(s, C.byref(cam), C.byref(st), 2, holes, None, None) == A.RS_E_INVALID
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


# ---------------------------------------------------------------- struct layouts ----
# The C structs of the boundary and the #[repr(C)] mirrors a Rust caller declares.
C_OF_RUST = {"RsTexture": "rs_texture_desc", "RsMaterial": "rs_material_desc", "RsPerlin": "rs_perlin_desc",
             "RsTransform": "rs_transform", "RsCamera": "rs_camera_desc", "RsSettings": "rs_render_settings",
             "RsStats": "rs_render_stats", "RsSceneInfo": "rs_scene_info", "RsNoiseStats": "rs_noise_stats"}
LAYOUT = os.path.join(ROOT, "tests", "golden", "abi_layout.json")


def header_structs():
    """typedef struct name { fields } name; of the header -> [(field, array length or None)]"""
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "raysnail_hip.h")).read(), flags=re.S)
    out = {}
    for body, name in re.findall(r"typedef struct \w+ \{(.*?)\} (\w+);", text, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            m = re.match(r"(.*?)([\w\s,\[\]\d*]+)$", decl)
            typ = decl.split()[0] if not decl.startswith("const") else " ".join(decl.split()[:2])
            names = decl[len(typ):].replace("*", " ").split(",")
            for n in names:
                n = n.strip()
                arr = re.match(r"(\w+)\[(\d+)\]", n)
                fields.append((arr.group(1), int(arr.group(2))) if arr else (n, None))
        out[name] = fields
    return out


def c_layout(tmp_path):
    """offsetof / sizeof of every field of every header struct, measured by gcc"""
    import subprocess
    structs = header_structs()
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "raysnail_hip.h"', "int main(void) {"]
    for name, fields in structs.items():
        lines.append(f'printf("S {name} %zu %zu\\n", sizeof({name}), _Alignof({name}));')
        for f, _ in fields:
            lines.append(f'printf("F {name} {f} %zu %zu\\n", offsetof({name}, {f}), sizeof((({name}*)0)->{f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    res = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        k = line.split()
        if k[0] == "S":
            res.setdefault(k[1], {"fields": []}).update(size=int(k[2]), align=int(k[3]))
        else:
            res[k[1]]["fields"].append([k[2], int(k[3]), int(k[4])])
    return res


def test_c_layout_matches_committed_table(tmp_path):
    """The layout table a foreign-language binding mirrors (tests/golden/abi_layout.json) is the
    header's, as gcc lays it out on this ABI (x86-64 SysV, the same as the GPU box)."""
    import json
    got = c_layout(tmp_path)
    if os.environ.get("RS_WRITE_ABI_LAYOUT"):
        json.dump(got, open(LAYOUT, "w"), indent=1)
    assert got == json.load(open(LAYOUT))


RUST_SIZE = {"i32": (4, 4), "u32": (4, 4), "f32": (4, 4), "f64": (8, 8), "u64": (8, 8), "i64": (8, 8), "u8": (1, 1)}


def rust_structs():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index("```rust"):]
    block = block[:block.index("```", 7)]
    out = {}
    for name, body in re.findall(r"pub struct (\w+) \{(.*?)\}", block, flags=re.S):
        body = re.sub(r"//[^\n]*", "", body)
        out[name] = [(f, t.strip()) for f, t in re.findall(r"pub (\w+): ([^,]+?)(?:,|$)", body.strip())]
    return out


def rust_layout(structs, name, cache):
    if name in cache:
        return cache[name]
    off, align, fields = 0, 1, []
    for f, t in structs[name]:
        arr = re.match(r"\[(\w+); (\d+)\]", t)
        if arr:
            sz, al = RUST_SIZE[arr.group(1)]
            sz *= int(arr.group(2))
        elif t.startswith("*"):
            sz, al = 8, 8
        elif t in RUST_SIZE:
            sz, al = RUST_SIZE[t]
        else:
            sub = rust_layout(structs, t, cache)
            sz, al = sub["size"], sub["align"]
        off = (off + al - 1) // al * al
        fields.append([f, off, sz])
        off += sz
        align = max(align, al)
    cache[name] = {"size": (off + align - 1) // align * align, "align": align, "fields": fields}
    return cache[name]


def test_integration_rust_layout_matches_c():
    """Every #[repr(C)] struct of INTEGRATION.md's FFI block has the C struct's size, alignment and
    field offsets / sizes, field by field in order (names may differ: `type` is a Rust keyword)."""
    import json
    c = json.load(open(LAYOUT))
    rs = rust_structs()
    assert set(rs) == set(C_OF_RUST), set(rs) ^ set(C_OF_RUST)
    assert set(C_OF_RUST.values()) == set(c)
    cache = {}
    for rname, cname in C_OF_RUST.items():
        r = rust_layout(rs, rname, cache)
        assert (r["size"], r["align"]) == (c[cname]["size"], c[cname]["align"]), rname
        assert [f[1:] for f in r["fields"]] == [f[1:] for f in c[cname]["fields"]], rname


def test_integration_declares_every_export():
    """INTEGRATION.md's FFI block declares every function of the header, with its arity."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index("```rust"):]
    block = block[:block.index("```", 7)]
    rust = {m.group(1): m.group(2) for m in re.finditer(r"pub fn (rs_\w+)\((.*?)\)\s*(?:->[^;]*)?;", block, flags=re.S)}
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "raysnail_hip.h")).read(), flags=re.S)
    c = {m.group(1): m.group(2) for m in re.finditer(r"\b(rs_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", hdr)}
    assert set(c) == set(rust), set(c) ^ set(rust)
    for name, args in c.items():
        n_c = 0 if args.strip() in ("", "void") else args.count(",") + 1
        n_r = 0 if not rust[name].strip() else rust[name].count(",") + 1
        assert n_c == n_r, name


def _rust_ffi_block():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index("```rust"):]
    return block[:block.index("```", 7)]


def _c_param_type(decl):
    """a C parameter declaration -> the Rust type a #[repr(C)] binding must give it"""
    base = {"uint32_t": "u32", "int32_t": "i32", "uint64_t": "u64", "int64_t": "i64", "double": "f64", "float": "f32",
            "uint8_t": "u8", "int": "i32", "void": "c_void", "char": "c_char", "rs_scene": "RsScene",
            "rs_row_callback": "RsRowCallback"}
    base.update({c: r for r, c in C_OF_RUST.items()})
    decl = decl.strip()
    arr = re.search(r"\[\d+\]\s*$", decl)
    decl = re.sub(r"\[\d+\]\s*$", "", decl)
    toks = decl.replace("*", " * ").split()
    const = toks[0] == "const"  # `const` qualifies what is to its left (the base type when it leads)
    if const:
        toks = toks[1:]
    t = base[toks[0]]
    rest = toks[1:]
    if rest and rest[0] == "const":
        const, rest = True, rest[1:]
    for k, tok in enumerate(rest):
        if tok != "*":
            continue
        t = ("*const " if const else "*mut ") + t
        const = k + 1 < len(rest) and rest[k + 1] == "const"  # `T* const*`: the outer pointer's pointee is const
    if arr:
        t = ("*const " if const else "*mut ") + t
    return t


def _rust_type(t):
    t = t.strip().replace("std::ffi::c_void", "c_void").replace("std::os::raw::c_char", "c_char")
    return "*mut c_void" if t == "HipStream" else t


def test_integration_ffi_types_match_c():
    """Every function of INTEGRATION.md's FFI block has the header's parameter types in order (and its return
    type): const T* <-> *const T, T* <-> *mut T, fixed arrays as pointers, hipStream_t (void*) as HipStream."""
    block = _rust_ffi_block()
    rust = {m.group(1): (m.group(2), m.group(3)) for m in
            re.finditer(r"pub fn (rs_\w+)\((.*?)\)\s*(?:->\s*([^;]*))?;", block, flags=re.S)}
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "raysnail_hip.h")).read(), flags=re.S)
    hdr = re.sub(r"typedef void \(\*rs_row_callback\)\([^)]*\);", "", hdr)
    for m in re.finditer(r"([\w\s\*]+?)\b(rs_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", hdr):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3)
        c_params = [] if args.strip() in ("", "void") else [_c_param_type(a.rsplit(None, 1)[0] if not re.search(r"\[\d+\]$", a.strip()) else re.sub(r"\w+\s*(\[\d+\])$", r"\1", a.strip())) for a in args.split(",")]
        r_args, r_ret = rust[name]
        r_params = [_rust_type(a.split(":", 1)[1]) for a in r_args.split(",") if a.strip()]
        assert c_params == r_params, (name, c_params, r_params)
        c_ret = _c_param_type(ret) if ret not in ("int",) else "i32"
        assert c_ret == _rust_type(r_ret or ""), (name, c_ret, r_ret)


def test_integration_row_callback_matches_c():
    """RsRowCallback (the Rust side of rs_row_callback) and the drop-in's forward_row trampoline (INTEGRATION.md
    §3) have the header typedef's parameter types, and the drop-in renders through rs_render_rows (rows delivered
    as their bands finish, painter.rs:214, then the sentinel, painter.rs:332), not rs_render."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    hdr = open(os.path.join(ROOT, "include", "raysnail_hip.h")).read()
    c_args = re.search(r"typedef void \(\*rs_row_callback\)\(([^)]*)\);", hdr).group(1)
    c_params = [_c_param_type(a.rsplit(None, 1)[0]) for a in c_args.split(",")]
    alias = re.search(r"pub type RsRowCallback = extern \"C\" fn\(([^)]*)\);", _rust_ffi_block()).group(1)
    assert [_rust_type(a.split(":", 1)[1]) for a in alias.split(",")] == c_params
    sec3 = text[text.index("## 3. The drop-in call"):text.index("## 4. Multi-GPU")]
    tramp = re.search(r"extern \"C\" fn forward_row\(([^)]*)\)", sec3).group(1)
    assert [_rust_type(a.split(":", 1)[1]) for a in tramp.split(",")] == c_params
    assert "rs_render_rows(" in sec3 and "forward_row" in sec3.split("rs_render_rows(", 1)[1]
    assert "rs_render(" not in sec3.replace("rs_render_rows(", "")
